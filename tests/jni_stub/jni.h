/* Test-only stand-in for <jni.h>: just the types and JNIEnv functions jni/native/sentinel_amd_jni.c
 * uses, so tests/test_jni_glue.py can compile the JNI file without a JDK.  The real build uses the
 * JDK's header (the signatures here follow the JNI specification). */
#ifndef SGA_TEST_JNI_STUB_H
#define SGA_TEST_JNI_STUB_H
#include <stdint.h>
typedef int32_t jint;
typedef int64_t jlong;
typedef uint8_t jboolean;
typedef double jdouble;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass, jstring, jarray, jintArray, jlongArray, jdoubleArray;
#define JNI_ABORT 2
#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
    jstring (*NewStringUTF)(JNIEnv *, const char *);
    jsize (*GetArrayLength)(JNIEnv *, jarray);
    const char *(*GetStringUTFChars)(JNIEnv *, jstring, jboolean *);
    void (*ReleaseStringUTFChars)(JNIEnv *, jstring, const char *);
    jlong *(*GetLongArrayElements)(JNIEnv *, jlongArray, jboolean *);
    void (*ReleaseLongArrayElements)(JNIEnv *, jlongArray, jlong *, jint);
    jdouble *(*GetDoubleArrayElements)(JNIEnv *, jdoubleArray, jboolean *);
    void (*ReleaseDoubleArrayElements)(JNIEnv *, jdoubleArray, jdouble *, jint);
    jint *(*GetIntArrayElements)(JNIEnv *, jintArray, jboolean *);
    void (*ReleaseIntArrayElements)(JNIEnv *, jintArray, jint *, jint);
    void (*SetIntArrayRegion)(JNIEnv *, jintArray, jsize, jsize, const jint *);
    void (*SetLongArrayRegion)(JNIEnv *, jlongArray, jsize, jsize, const jlong *);
    void (*SetDoubleArrayRegion)(JNIEnv *, jdoubleArray, jsize, jsize, const jdouble *);
    void *(*GetDirectBufferAddress)(JNIEnv *, jobject);
};
#endif
