/*
 * jni_min.h — the subset of the JNI interface (Java Native Interface Specification, "JNI
 * Functions": types, calling convention and the JNIEnv function table) that sdfs_cdc_jni.c uses,
 * written from the specification because this image has no JDK.  The table keeps the
 * specification's slot numbering: every slot is a pointer, the slots the glue calls are typed,
 * the others are padding, so the struct is layout-compatible with the JDK's JNINativeInterface_.
 * Where a JDK exists, build with -DSDFS_USE_JDK_JNI -I$JAVA_HOME/include{,/linux} instead.
 */
#ifndef SDFS_JNI_MIN_H
#define SDFS_JNI_MIN_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef uint8_t jboolean;
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

#define JNI_FALSE 0
#define JNI_TRUE 1
#define JNI_OK 0
#define JNI_COMMIT 1
#define JNI_ABORT 2

#define JNIEXPORT __attribute__((visibility("default")))
#define JNICALL

struct JNINativeInterface_;
typedef const struct JNINativeInterface_* JNIEnv;

/* slot n of the table = the n-th function of the specification's list (0-based) */
struct JNINativeInterface_ {
    void* reserved0;
    void* reserved1;
    void* reserved2;
    void* reserved3;
    void* slots_4_5[2];                                                      /* GetVersion, DefineClass */
    jclass (*FindClass)(JNIEnv*, const char*);                               /* 6 */
    void* slots_7_13[7];
    jint (*ThrowNew)(JNIEnv*, jclass, const char*);                          /* 14 */
    void* slots_15_166[152];
    jstring (*NewStringUTF)(JNIEnv*, const char*);                           /* 167 */
    void* slots_168_170[3];
    jsize (*GetArrayLength)(JNIEnv*, jarray);                                /* 171 */
    void* slots_172_199[28];
    void (*GetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, jbyte*);   /* 200 */
    void* slots_201_207[7];
    void (*SetByteArrayRegion)(JNIEnv*, jbyteArray, jsize, jsize, const jbyte*); /* 208 */
    void* slots_209_210[2];
    void (*SetIntArrayRegion)(JNIEnv*, jintArray, jsize, jsize, const jint*);    /* 211 */
    void* slots_212_227[16];
    jboolean (*ExceptionCheck)(JNIEnv*);                                     /* 228 */
    void* slot_229;                                                          /* NewDirectByteBuffer */
    void* (*GetDirectBufferAddress)(JNIEnv*, jobject);                       /* 230 */
    jlong (*GetDirectBufferCapacity)(JNIEnv*, jobject);                      /* 231 */
    void* slots_232_233[2];                                                  /* GetObjectRefType, GetModule */
};

/* the specification's slot numbers of the typed entries */
#include <stddef.h>
#define SDFS_JNI_SLOT(f, n) _Static_assert(offsetof(struct JNINativeInterface_, f) == (n) * sizeof(void*), #f)
SDFS_JNI_SLOT(FindClass, 6);
SDFS_JNI_SLOT(ThrowNew, 14);
SDFS_JNI_SLOT(NewStringUTF, 167);
SDFS_JNI_SLOT(GetArrayLength, 171);
SDFS_JNI_SLOT(GetByteArrayRegion, 200);
SDFS_JNI_SLOT(SetByteArrayRegion, 208);
SDFS_JNI_SLOT(SetIntArrayRegion, 211);
SDFS_JNI_SLOT(ExceptionCheck, 228);
SDFS_JNI_SLOT(GetDirectBufferAddress, 230);
SDFS_JNI_SLOT(GetDirectBufferCapacity, 231);
#undef SDFS_JNI_SLOT

#ifdef __cplusplus
}
#endif
#endif /* SDFS_JNI_MIN_H */
