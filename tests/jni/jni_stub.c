/*
 * jni_stub.c — a stand-in JNIEnv for driving jni/sdfs_cdc_jni.c without a JVM (test
 * infrastructure only).  Java arrays are host structs {kind, length, bytes}; FindClass returns
 * the class name; ThrowNew records the pending exception (class + message) that ExceptionCheck
 * reports.  Only the slots the glue calls are filled; any other slot is NULL, so a call the glue
 * should not make crashes the test instead of passing silently.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../jni/jni_min.h"

struct _jobject {
    int kind;   /* 1 = byte[], 2 = int[], 3 = String, 4 = class, 5 = direct buffer */
    int32_t len;
    uint8_t* data;
};

static __thread char t_exc_class[128];
static __thread char t_exc_msg[512];
static __thread int t_pending;

static jclass stub_FindClass(JNIEnv* env, const char* name) {
    (void)env;
    struct _jobject* o = calloc(1, sizeof(*o));
    o->kind = 4;
    o->len = (int32_t)strlen(name);
    o->data = (uint8_t*)strdup(name);
    return o;
}

static jint stub_ThrowNew(JNIEnv* env, jclass c, const char* msg) {
    (void)env;
    snprintf(t_exc_class, sizeof t_exc_class, "%s", c && c->data ? (const char*)c->data : "?");
    snprintf(t_exc_msg, sizeof t_exc_msg, "%s", msg ? msg : "");
    t_pending = 1;
    free(c->data);
    free(c);
    return 0;
}

static jstring stub_NewStringUTF(JNIEnv* env, const char* s) {
    (void)env;
    struct _jobject* o = calloc(1, sizeof(*o));
    o->kind = 3;
    o->len = (int32_t)strlen(s);
    o->data = (uint8_t*)strdup(s);
    return o;
}

static jsize stub_GetArrayLength(JNIEnv* env, jarray a) {
    (void)env;
    return a->len;
}

static int range_ok(jarray a, jsize start, jsize n) {
    if (start < 0 || n < 0 || start + n > a->len) {
        snprintf(t_exc_class, sizeof t_exc_class, "java/lang/ArrayIndexOutOfBoundsException");
        t_exc_msg[0] = 0;
        t_pending = 1;
        return 0;
    }
    return 1;
}

static __thread int t_fail_region;  /* next GetByteArrayRegion raises (stub_fail_next_region) */

static void stub_GetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize n, jbyte* buf) {
    (void)env;
    if (t_fail_region) {  /* as a JVM does for a bad region: nothing copied, exception pending */
        t_fail_region = 0;
        snprintf(t_exc_class, sizeof t_exc_class, "java/lang/ArrayIndexOutOfBoundsException");
        snprintf(t_exc_msg, sizeof t_exc_msg, "stub: injected");
        t_pending = 1;
        return;
    }
    if (a->kind == 1 && range_ok(a, start, n)) memcpy(buf, a->data + start, (size_t)n);
}

void stub_fail_next_region(void) { t_fail_region = 1; }

static void stub_SetByteArrayRegion(JNIEnv* env, jbyteArray a, jsize start, jsize n, const jbyte* buf) {
    (void)env;
    if (a->kind == 1 && range_ok(a, start, n)) memcpy(a->data + start, buf, (size_t)n);
}

static void stub_SetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize n, const jint* buf) {
    (void)env;
    if (a->kind == 2 && range_ok(a, start, n)) memcpy(a->data + 4 * (size_t)start, buf, 4 * (size_t)n);
}

static jboolean stub_ExceptionCheck(JNIEnv* env) {
    (void)env;
    return t_pending ? JNI_TRUE : JNI_FALSE;
}

static void* stub_GetDirectBufferAddress(JNIEnv* env, jobject o) {
    (void)env;
    return o && o->kind == 5 ? o->data : NULL;
}

static jlong stub_GetDirectBufferCapacity(JNIEnv* env, jobject o) {
    (void)env;
    return o && o->kind == 5 ? o->len : -1;
}

static struct JNINativeInterface_ g_table;
static const struct JNINativeInterface_* g_env = &g_table;

/* ---- helpers for the Python test (ctypes) ---- */
JNIEnv* stub_env(void) {
    g_table.FindClass = stub_FindClass;
    g_table.ThrowNew = stub_ThrowNew;
    g_table.NewStringUTF = stub_NewStringUTF;
    g_table.GetArrayLength = stub_GetArrayLength;
    g_table.GetByteArrayRegion = stub_GetByteArrayRegion;
    g_table.SetByteArrayRegion = stub_SetByteArrayRegion;
    g_table.SetIntArrayRegion = stub_SetIntArrayRegion;
    g_table.ExceptionCheck = stub_ExceptionCheck;
    g_table.GetDirectBufferAddress = stub_GetDirectBufferAddress;
    g_table.GetDirectBufferCapacity = stub_GetDirectBufferCapacity;
    return (JNIEnv*)&g_env;
}

/* kind 1 = byte[] (elem 1), 2 = int[] (elem 4), 5 = direct buffer over caller memory */
jobject stub_new_array(int kind, int32_t len, const void* init) {
    struct _jobject* o = calloc(1, sizeof(*o));
    o->kind = kind;
    o->len = len;
    if (kind == 5) {
        o->data = (uint8_t*)init;
        return o;
    }
    const size_t bytes = (size_t)len * (kind == 2 ? 4 : 1);
    o->data = calloc(bytes ? bytes : 1, 1);
    if (init && bytes) memcpy(o->data, init, bytes);
    return o;
}

void* stub_array_data(jobject o) { return o->data; }
int32_t stub_array_len(jobject o) { return o->len; }

void stub_free(jobject o) {
    if (!o) return;
    if (o->kind != 5) free(o->data);
    free(o);
}

/* pending exception: returns 1 and copies class / message, or 0 */
int stub_take_exception(char* cls, int cls_n, char* msg, int msg_n) {
    if (!t_pending) return 0;
    snprintf(cls, (size_t)cls_n, "%s", t_exc_class);
    snprintf(msg, (size_t)msg_n, "%s", t_exc_msg);
    t_pending = 0;
    return 1;
}
