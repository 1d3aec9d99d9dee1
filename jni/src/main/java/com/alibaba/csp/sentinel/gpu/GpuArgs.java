package com.alibaba.csp.sentinel.gpu;

import java.lang.reflect.Array;
import java.nio.charset.StandardCharsets;
import java.util.Collection;

import com.alibaba.csp.sentinel.slots.block.flow.param.ParamFlowArgument;

/**
 * The engine's view of {@code Object... args} (include/sentinel_amd.h SGA_EV_ARGS): two words per argument --
 * kind << 62 | list length, then the value's 64-bit key or the offset of a Collection / array's elements,
 * which follow the pairs.  ParamFlowChecker.passCheck unwraps a ParamFlowArgument (ParamFlowChecker.java:63-66)
 * and ParamFlowChecker.passLocalCheck checks every element of a Collection / array (:79-106).
 */
final class GpuArgs {

    static final long SCALAR = 0L, NULL = 1L << 62, LIST = 2L << 62;

    private GpuArgs() {}

    /**
     * A 64-bit key per parameter object, typed like equals(): ParameterMetric compares values with equals, so
     * Long(5), Integer(5) and "5" are three keys.  Longs are their value; every other type mixes a type tag
     * with its bits (a collision with a Long or across types has probability 2^-64).  Hot items are mapped the
     * same way ({@link GpuRuleSync}).
     */
    static long key(Object p) {
        if (p instanceof Long) {
            return (Long) p;
        }
        if (p instanceof Integer) {
            return mix(1, (Integer) p);
        }
        if (p instanceof Short) {
            return mix(2, (Short) p);
        }
        if (p instanceof Byte) {
            return mix(3, (Byte) p);
        }
        if (p instanceof Boolean) {
            return mix(4, ((Boolean) p) ? 1 : 0);
        }
        if (p instanceof Character) {
            return mix(5, (Character) p);
        }
        if (p instanceof Double) {
            return mix(6, Double.doubleToLongBits((Double) p));
        }
        if (p instanceof Float) {
            return mix(7, Float.floatToIntBits((Float) p));
        }
        long h = 0xcbf29ce484222325L;  // FNV-1a 64 of the UTF-8 bytes, then typed
        for (byte b : (p instanceof String ? (String) p : String.valueOf(p)).getBytes(StandardCharsets.UTF_8)) {
            h ^= (b & 0xff);
            h *= 0x100000001b3L;
        }
        return mix(p instanceof String ? 8 : 9, h);
    }

    private static long mix(long tag, long v) {  // splitmix64 of the tagged value
        long z = v ^ (tag << 56) ^ 0x5EB7F00DL;
        z = (z ^ (z >>> 30)) * 0xBF58476D1CE4E5B9L;
        z = (z ^ (z >>> 27)) * 0x94D049BB133111EBL;
        return z ^ (z >>> 31);
    }

    private static Object unwrap(Object v) {
        return v instanceof ParamFlowArgument ? ((ParamFlowArgument) v).paramFlowKey() : v;
    }

    /** The words of args (pairs first, then list elements); words.length may exceed 2 * args.length. */
    static long[] encode(Object[] args) {
        if (args == null) {
            args = new Object[0];
        }
        int n = args.length, extra = 0;
        for (Object a : args) {
            Object v = unwrap(a);
            if (v instanceof Collection) {
                extra += ((Collection<?>) v).size();
            } else if (v != null && v.getClass().isArray()) {
                extra += Array.getLength(v);
            }
        }
        long[] w = new long[2 * n + extra];
        int pos = 2 * n;
        for (int k = 0; k < n; k++) {
            Object v = unwrap(args[k]);
            if (v == null) {
                w[2 * k] = NULL;
            } else if (v instanceof Collection) {
                Collection<?> c = (Collection<?>) v;
                w[2 * k] = LIST | c.size();
                w[2 * k + 1] = pos;
                for (Object x : c) {
                    w[pos++] = key(x);
                }
            } else if (v.getClass().isArray()) {
                int len = Array.getLength(v);
                w[2 * k] = LIST | len;
                w[2 * k + 1] = pos;
                for (int i = 0; i < len; i++) {
                    w[pos++] = key(Array.get(v, i));
                }
            } else {
                w[2 * k] = SCALAR;
                w[2 * k + 1] = key(v);
            }
        }
        return w;
    }
}
