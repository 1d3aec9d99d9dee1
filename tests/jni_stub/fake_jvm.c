/* Test-only JNIEnv for driving jni/native/sentinel_amd_jni.c without a JVM (tests/test_jni_live_gpu.py):
 * Java arrays, strings and direct ByteBuffers are small wrappers around caller-owned memory, and the
 * JNIEnv functions the JNI file uses (tests/jni_stub/jni.h) read and write through them with the JNI
 * specification's semantics (Get<T>ArrayElements hands out the array's storage, Release is then a
 * no-op, Set<T>ArrayRegion copies in, GetDirectBufferAddress returns the buffer's address). */
#include <stdlib.h>
#include <string.h>

#include "jni.h"

typedef struct {
    jsize len;
    void *data;
} fake_arr;
typedef struct {
    char *s;
} fake_str;
typedef struct {
    void *addr;
} fake_buf;

static jstring f_new_string(JNIEnv *env, const char *s) {
    (void)env;
    fake_str *x = (fake_str *)malloc(sizeof(*x));
    const size_t n = strlen(s ? s : "") + 1;
    x->s = (char *)malloc(n);
    memcpy(x->s, s ? s : "", n);
    return (jstring)x;
}
static jsize f_len(JNIEnv *env, jarray a) {
    (void)env;
    return ((fake_arr *)a)->len;
}
static const char *f_chars(JNIEnv *env, jstring s, jboolean *copy) {
    (void)env;
    if (copy) *copy = 0;
    return ((fake_str *)s)->s;
}
static void f_rel_chars(JNIEnv *env, jstring s, const char *c) {
    (void)env;
    (void)s;
    (void)c;
}
static jlong *f_get_l(JNIEnv *env, jlongArray a, jboolean *copy) {
    (void)env;
    if (copy) *copy = 0;
    return (jlong *)((fake_arr *)a)->data;
}
static void f_rel_l(JNIEnv *env, jlongArray a, jlong *p, jint mode) {
    (void)env;
    (void)a;
    (void)p;
    (void)mode;
}
static jdouble *f_get_d(JNIEnv *env, jdoubleArray a, jboolean *copy) {
    (void)env;
    if (copy) *copy = 0;
    return (jdouble *)((fake_arr *)a)->data;
}
static void f_rel_d(JNIEnv *env, jdoubleArray a, jdouble *p, jint mode) {
    (void)env;
    (void)a;
    (void)p;
    (void)mode;
}
static jint *f_get_i(JNIEnv *env, jintArray a, jboolean *copy) {
    (void)env;
    if (copy) *copy = 0;
    return (jint *)((fake_arr *)a)->data;
}
static void f_rel_i(JNIEnv *env, jintArray a, jint *p, jint mode) {
    (void)env;
    (void)a;
    (void)p;
    (void)mode;
}
static void f_set_i(JNIEnv *env, jintArray a, jsize at, jsize n, const jint *v) {
    (void)env;
    memcpy((jint *)((fake_arr *)a)->data + at, v, sizeof(jint) * (size_t)n);
}
static void f_set_l(JNIEnv *env, jlongArray a, jsize at, jsize n, const jlong *v) {
    (void)env;
    memcpy((jlong *)((fake_arr *)a)->data + at, v, sizeof(jlong) * (size_t)n);
}
static void f_set_d(JNIEnv *env, jdoubleArray a, jsize at, jsize n, const jdouble *v) {
    (void)env;
    memcpy((jdouble *)((fake_arr *)a)->data + at, v, sizeof(jdouble) * (size_t)n);
}
static void *f_buf(JNIEnv *env, jobject o) {
    (void)env;
    return ((fake_buf *)o)->addr;
}

static const struct JNINativeInterface_ fake_if = {f_new_string, f_len,   f_chars, f_rel_chars, f_get_l,
                                                    f_rel_l,      f_get_d, f_rel_d, f_get_i,     f_rel_i,
                                                    f_set_i,      f_set_l, f_set_d, f_buf};
static JNIEnv fake_env_v = &fake_if;

JNIEXPORT JNIEnv *fake_env(void) { return &fake_env_v; }
/* a Java int[] / long[] / double[] over `len` elements the caller owns at `data` */
JNIEXPORT jobject fake_array(jsize len, void *data) {
    fake_arr *a = (fake_arr *)malloc(sizeof(*a));
    a->len = len;
    a->data = data;
    return (jobject)a;
}
JNIEXPORT jobject fake_string(const char *s) { return (jobject)f_new_string(&fake_env_v, s); }
JNIEXPORT const char *fake_string_chars(jobject s) { return ((fake_str *)s)->s; }
/* a direct ByteBuffer over caller-owned memory */
JNIEXPORT jobject fake_buffer(void *addr) {
    fake_buf *b = (fake_buf *)malloc(sizeof(*b));
    b->addr = addr;
    return (jobject)b;
}
JNIEXPORT void fake_free(jobject o) { free(o); }
JNIEXPORT void fake_free_string(jobject o) {
    if (o) free(((fake_str *)o)->s);
    free(o);
}
