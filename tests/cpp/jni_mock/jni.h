/* Minimal stand-in for a JDK's jni.h in this JDK-less image: the types and the JNIEnv functions
 * integration/jni/hdrf_jni.c calls, with the JNI specification's signatures (the table's layout is
 * this header's own, not the JDK's).  tests/cpp/jni_driver.c implements the table (direct buffers,
 * arrays, strings, a pending exception per thread) and drives the shim's entry points the way a
 * DataNode's HipReductionScheme would (tests/test_jni.py). */
#pragma once
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef jint jsize;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jlongArray;
typedef jarray jintArray;
typedef jobject jstring;
typedef uint8_t jboolean;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
struct JNINativeInterface_ {
    jclass (*FindClass)(JNIEnv *env, const char *name);
    jint (*ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
    void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
    jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
    jsize (*GetArrayLength)(JNIEnv *env, jarray array);
    jlong *(*GetLongArrayElements)(JNIEnv *env, jlongArray array, unsigned char *isCopy);
    void (*ReleaseLongArrayElements)(JNIEnv *env, jlongArray array, jlong *elems, jint mode);
    jint *(*GetIntArrayElements)(JNIEnv *env, jintArray array, jboolean *isCopy);
    void (*ReleaseIntArrayElements)(JNIEnv *env, jintArray array, jint *elems, jint mode);
    jbyteArray (*NewByteArray)(JNIEnv *env, jsize len);
    void (*SetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, const jbyte *buf);
    const char *(*GetStringUTFChars)(JNIEnv *env, jstring string, jboolean *isCopy);
    void (*ReleaseStringUTFChars)(JNIEnv *env, jstring string, const char *utf);
    jobject (*NewDirectByteBuffer)(JNIEnv *env, void *address, jlong capacity);
    jbyte *(*GetByteArrayElements)(JNIEnv *env, jbyteArray array, jboolean *isCopy);
    void (*ReleaseByteArrayElements)(JNIEnv *env, jbyteArray array, jbyte *elems, jint mode);
};
