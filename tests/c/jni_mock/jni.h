/*
 * jni.h -- a TEST DOUBLE of the JNI header, for tests/c/jni_caller.c only.
 *
 * This image has no JDK, so jni/rsketch_jni.c cannot be built against the real
 * <jni.h>.  This header declares the subset of the JNI types and of the
 * JNINativeInterface / JNIInvokeInterface function tables that rsketch_jni.c
 * uses, with the real names and calling forms ((*env)->Fn(env, ...),
 * (*vm)->Fn(vm, ...)), so the glue compiles unchanged against it and
 * tests/c/jni_caller.c can run it against a fake JVM (objects are host
 * structs; attach failures and allocation failures can be injected).  The
 * table layout is NOT the JDK's: the glue is source-compatible with the real
 * header, and nothing built against this one may be loaded by a JVM.
 */
#ifndef RSK_TEST_JNI_MOCK_H
#define RSK_TEST_JNI_MOCK_H
#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_OK 0
#define JNI_ERR (-1)
#define JNI_EDETACHED (-2)
#define JNI_VERSION_1_6 0x00010006
#define JNI_TRUE 1
#define JNI_FALSE 0

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

typedef struct mock_obj *jobject;
typedef jobject jclass, jstring, jarray, jthrowable, jobjectArray, jbooleanArray, jbyteArray, jintArray,
    jlongArray, jdoubleArray;
typedef struct mock_method *jmethodID;

struct JNINativeInterface_;
struct JNIInvokeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;
typedef const struct JNIInvokeInterface_ *JavaVM;

struct JNINativeInterface_ {
  jclass (*FindClass)(JNIEnv *, const char *);
  jint (*ThrowNew)(JNIEnv *, jclass, const char *);
  jboolean (*ExceptionCheck)(JNIEnv *);
  void (*ExceptionClear)(JNIEnv *);
  jobject (*NewGlobalRef)(JNIEnv *, jobject);
  void (*DeleteGlobalRef)(JNIEnv *, jobject);
  void (*DeleteLocalRef)(JNIEnv *, jobject);
  jmethodID (*GetStaticMethodID)(JNIEnv *, jclass, const char *, const char *);
  void (*CallStaticVoidMethod)(JNIEnv *, jclass, jmethodID, ...);
  const char *(*GetStringUTFChars)(JNIEnv *, jstring, jboolean *);
  void (*ReleaseStringUTFChars)(JNIEnv *, jstring, const char *);
  jsize (*GetArrayLength)(JNIEnv *, jarray);
  jobject (*GetObjectArrayElement)(JNIEnv *, jobjectArray, jsize);
  jbooleanArray (*NewBooleanArray)(JNIEnv *, jsize);
  void (*SetBooleanArrayRegion)(JNIEnv *, jbooleanArray, jsize, jsize, const jboolean *);
  jbyteArray (*NewByteArray)(JNIEnv *, jsize);
  void (*SetByteArrayRegion)(JNIEnv *, jbyteArray, jsize, jsize, const jbyte *);
  void (*GetByteArrayRegion)(JNIEnv *, jbyteArray, jsize, jsize, jbyte *);
  void (*GetIntArrayRegion)(JNIEnv *, jintArray, jsize, jsize, jint *);
  void (*GetLongArrayRegion)(JNIEnv *, jlongArray, jsize, jsize, jlong *);
  void (*SetLongArrayRegion)(JNIEnv *, jlongArray, jsize, jsize, const jlong *);
  void (*SetDoubleArrayRegion)(JNIEnv *, jdoubleArray, jsize, jsize, const jdouble *);
  void *(*GetDirectBufferAddress)(JNIEnv *, jobject);
  jlong (*GetDirectBufferCapacity)(JNIEnv *, jobject);
};

struct JNIInvokeInterface_ {
  jint (*GetEnv)(JavaVM *, void **, jint);
  jint (*AttachCurrentThreadAsDaemon)(JavaVM *, void **, void *);
};

#endif
