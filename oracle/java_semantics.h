/*
 * ORACLE / TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is linked into the
 * product library; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker.
 *
 * Java numeric semantics the reference's hot path relies on (JLS §5.1.3,
 * java.lang.Math).  Restated from the published Java specification, not from
 * any JDK source:
 *   - (int)d / (long)d : NaN -> 0, saturate at MIN/MAX, truncate toward zero
 *     (JLS 5.1.3).  Used e.g. DefaultController.java:77 `(int)(node.passQps())`,
 *     WarmUpController.java:115 `(long) node.passQps()`.
 *   - Math.round(double): nearest long, ties toward +infinity (javadoc since
 *     Java 7).  Used RateLimiterController.java:59.
 *   - Math.nextUp(double): adjacent value toward +infinity.  WarmUpController.java:127.
 *   - String.hashCode(): s[0]*31^(n-1)+... over UTF-16 code units, i32 wrap.
 *     EnvoySentinelRuleConverter.java:67-72.
 * Everything here is compiled with -ffp-contract=off (no FMA contraction) so the
 * double expressions round exactly like the JVM's strictfp evaluation.
 */
#ifndef SENTINEL_ORACLE_JAVA_SEMANTICS_H
#define SENTINEL_ORACLE_JAVA_SEMANTICS_H

#include <stdint.h>
#include <string.h>
#include <math.h>

static inline int32_t j_d2i(double d) {
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d; /* C truncates toward zero in range */
}

static inline int64_t j_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX; /* 2^63 */
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}

static inline uint64_t j_dbits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

/* Math.round(double): round half up (toward +inf) without the floor(x+0.5)
 * double-rounding error.  Restated from the javadoc contract: the result is the
 * long closest to the argument, ties rounding to positive infinity; NaN -> 0;
 * values outside the long range saturate. */
static inline int64_t j_round(double a) {
    uint64_t bits = j_dbits(a);
    int64_t biased_exp = (int64_t)((bits & 0x7FF0000000000000ULL) >> 52);
    int64_t shift = (52 - 1 + 1023) - biased_exp; /* bits below the 0.5 position */
    if ((shift & -64LL) == 0) { /* 0 <= shift < 64 */
        int64_t r = (int64_t)((bits & 0x000FFFFFFFFFFFFFULL) | 0x0010000000000000ULL);
        if ((int64_t)bits < 0) r = -r;
        /* r * 2^(e) with one extra fractional bit: add half and drop it */
        return ((r >> shift) + 1) >> 1;
    }
    /* |a| < 0.5 (shift >= 64 -> 0 after rounding) or integral/huge/NaN */
    if (shift >= 64) return 0;
    return j_d2l(a);
}

static inline double j_next_up(double d) {
    if (d != d || d == INFINITY) return d;
    return nextafter(d, INFINITY);
}

/* String.hashCode over UTF-16 code units of a UTF-8 encoded C string. */
static inline int32_t j_string_hash_utf8(const char *s, size_t len) {
    uint32_t h = 0;
    size_t i = 0;
    while (i < len) {
        unsigned char c = (unsigned char)s[i];
        uint32_t cp;
        int n;
        if (c < 0x80) { cp = c; n = 1; }
        else if ((c >> 5) == 0x6 && i + 1 < len) { cp = ((c & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu); n = 2; }
        else if ((c >> 4) == 0xE && i + 2 < len) {
            cp = ((c & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu); n = 3;
        } else if ((c >> 3) == 0x1E && i + 3 < len) {
            cp = ((c & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu);
            n = 4;
        } else { cp = 0xFFFD; n = 1; }
        if (cp >= 0x10000) { /* surrogate pair */
            uint32_t v = cp - 0x10000;
            h = h * 31u + (0xD800u + (v >> 10));
            h = h * 31u + (0xDC00u + (v & 0x3FFu));
        } else {
            h = h * 31u + cp;
        }
        i += (size_t)n;
    }
    return (int32_t)h;
}

#endif
