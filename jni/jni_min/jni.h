/*
 * jni_min/jni.h -- a declaration-only stand-in for <jni.h>, used ONLY by the
 * CPU test that type-checks jni/mbx_jni.c in this image, which has no JDK
 * (tests/test_jni_glue.py: gcc -std=c11 -Wall -Wextra -Werror -fsyntax-only).
 * It is not used to build libmbx_jni.so; jni/Makefile builds against
 * $JAVA_HOME/include/jni.h.
 *
 * Contents follow the JNI specification's C binding (the JNIEnv function
 * table and its types), restricted to exactly the functions the glue calls;
 * the test checks that the two sets are equal.  As in the real header's C
 * mode, every reference type is an alias of jobject.
 */
#ifndef MBX_JNI_MIN_H
#define MBX_JNI_MIN_H

#include <stdarg.h>
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_COMMIT 1
#define JNI_ABORT 2

typedef int32_t jint;
typedef int64_t jlong;
typedef int8_t jbyte;
typedef uint8_t jboolean;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject *jobject;
typedef jobject jclass;
typedef jobject jthrowable;
typedef jobject jstring;
typedef jobject jarray;
typedef jarray jbooleanArray;
typedef jarray jbyteArray;
typedef jarray jcharArray;
typedef jarray jshortArray;
typedef jarray jintArray;
typedef jarray jlongArray;
typedef jarray jfloatArray;
typedef jarray jdoubleArray;
typedef jarray jobjectArray;

struct _jfieldID;
typedef struct _jfieldID *jfieldID;
struct _jmethodID;
typedef struct _jmethodID *jmethodID;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_ *JNIEnv;

struct JNINativeInterface_ {
  /* classes, exceptions, local references */
  jclass (*FindClass)(JNIEnv *env, const char *name);
  jint (*Throw)(JNIEnv *env, jthrowable obj);
  jint (*ThrowNew)(JNIEnv *env, jclass clazz, const char *msg);
  void (*ExceptionClear)(JNIEnv *env);
  jboolean (*ExceptionCheck)(JNIEnv *env);
  void (*DeleteLocalRef)(JNIEnv *env, jobject obj);
  /* objects, fields */
  jmethodID (*GetMethodID)(JNIEnv *env, jclass clazz, const char *name, const char *sig);
  jobject (*NewObject)(JNIEnv *env, jclass clazz, jmethodID methodID, ...);
  jfieldID (*GetFieldID)(JNIEnv *env, jclass clazz, const char *name, const char *sig);
  jobject (*GetObjectField)(JNIEnv *env, jobject obj, jfieldID fieldID);
  jint (*GetIntField)(JNIEnv *env, jobject obj, jfieldID fieldID);
  jfloat (*GetFloatField)(JNIEnv *env, jobject obj, jfieldID fieldID);
  /* strings */
  jstring (*NewStringUTF)(JNIEnv *env, const char *utf);
  jsize (*GetStringUTFLength)(JNIEnv *env, jstring str);
  const char *(*GetStringUTFChars)(JNIEnv *env, jstring str, jboolean *isCopy);
  void (*ReleaseStringUTFChars)(JNIEnv *env, jstring str, const char *chars);
  /* arrays */
  jsize (*GetArrayLength)(JNIEnv *env, jarray array);
  jobjectArray (*NewObjectArray)(JNIEnv *env, jsize len, jclass clazz, jobject init);
  jobject (*GetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index);
  void (*SetObjectArrayElement)(JNIEnv *env, jobjectArray array, jsize index, jobject val);
  jbyteArray (*NewByteArray)(JNIEnv *env, jsize len);
  jintArray (*NewIntArray)(JNIEnv *env, jsize len);
  jlongArray (*NewLongArray)(JNIEnv *env, jsize len);
  jfloatArray (*NewFloatArray)(JNIEnv *env, jsize len);
  jshort *(*GetShortArrayElements)(JNIEnv *env, jshortArray array, jboolean *isCopy);
  jint *(*GetIntArrayElements)(JNIEnv *env, jintArray array, jboolean *isCopy);
  jlong *(*GetLongArrayElements)(JNIEnv *env, jlongArray array, jboolean *isCopy);
  void (*ReleaseShortArrayElements)(JNIEnv *env, jshortArray array, jshort *elems, jint mode);
  void (*ReleaseIntArrayElements)(JNIEnv *env, jintArray array, jint *elems, jint mode);
  void (*ReleaseLongArrayElements)(JNIEnv *env, jlongArray array, jlong *elems, jint mode);
  void (*GetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, jbyte *buf);
  void (*GetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, jlong *buf);
  void (*SetByteArrayRegion)(JNIEnv *env, jbyteArray array, jsize start, jsize len, const jbyte *buf);
  void (*SetIntArrayRegion)(JNIEnv *env, jintArray array, jsize start, jsize len, const jint *buf);
  void (*SetLongArrayRegion)(JNIEnv *env, jlongArray array, jsize start, jsize len, const jlong *buf);
  void (*SetFloatArrayRegion)(JNIEnv *env, jfloatArray array, jsize start, jsize len, const jfloat *buf);
  /* NIO */
  void *(*GetDirectBufferAddress)(JNIEnv *env, jobject buf);
  jlong (*GetDirectBufferCapacity)(JNIEnv *env, jobject buf);
};

#endif /* MBX_JNI_MIN_H */
