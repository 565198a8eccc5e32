/*
 * jni_min/jni.h -- TEST INFRASTRUCTURE ONLY.  This image has no JDK, so tests/c/jni_harness.c
 * compiles the JNI glue (jvm/akka-dispatch-gpu/src/main/c/agx_jni.c) against this header and calls
 * it through a fake JNIEnv.  It declares the JNI types and the JNINativeInterface_ function table
 * with every slot at its index from the JNI specification (slots the glue does not call are
 * untyped void*); the harness asserts the indices of the typed slots.  A real build uses the
 * JDK's own <jni.h> (agx_jni.c's header comment gives the command).
 */
#ifndef AGX_JNI_MIN_H
#define AGX_JNI_MIN_H
#include <stdint.h>

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL
#define JNI_OK 0

typedef uint8_t jboolean;
#define JNI_FALSE 0
#define JNI_TRUE 1
typedef int8_t jbyte;
typedef uint16_t jchar;
typedef int16_t jshort;
typedef int32_t jint;
typedef int64_t jlong;
typedef float jfloat;
typedef double jdouble;
typedef jint jsize;

struct _jobject;
typedef struct _jobject* jobject;
typedef jobject jclass;
typedef jobject jstring;
typedef jobject jthrowable;
typedef jobject jarray;
typedef jarray jbyteArray;
typedef jarray jintArray;
typedef jarray jlongArray;

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

struct JNINativeInterface_ {
  void* reserved[4];                                                                  /* 0-3 */
  void* s4_5[2];                                                                      /* GetVersion, DefineClass */
  jclass (*FindClass)(JNIEnv*, const char*);                                          /* 6 */
  void* s7_13[7];
  jint (*ThrowNew)(JNIEnv*, jclass, const char*);                                     /* 14 */
  void* s15_166[152];
  jstring (*NewStringUTF)(JNIEnv*, const char*);                                      /* 167 */
  void* s168_170[3];
  jsize (*GetArrayLength)(JNIEnv*, jarray);                                           /* 171 */
  void* s172_199[28];
  void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);              /* 200 */
  void* s201_202[2];
  void (*GetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, jint*);                 /* 203 */
  void (*GetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, jlong*);              /* 204 */
  void* s205_207[3];
  void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*);        /* 208 */
  void* s209_210[2];
  void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);           /* 211 */
  void (*SetLongArrayRegion)(JNIEnv*, jlongArray, jsize, jsize, const jlong*);        /* 212 */
  void* s213_229[17];
  void* (*GetDirectBufferAddress)(JNIEnv*, jobject);                                  /* 230 */
  jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);                                 /* 231 */
  void* s232_233[2];                                                                  /* GetObjectRefType, GetModule */
};

#endif
