/*
 * sdfs_cdc_jni.c — JNI glue of org.opendedup.hashing.HipVariableSha256HashEngine
 * (jni/HipVariableSha256HashEngine.java) onto the C-ABI of include/sdfs_cdc.h.
 *
 * The Java class implements AbstractHashEngine (AbstractHashEngine.java:24-39) the way
 * VariableSha256HashEngine does (VariableSha256HashEngine.java:41-121) and is selected by one
 * branch in HashFunctionPool.getHashEngine() (HashFunctionPool.java:102-121).
 *
 *   nativeCreate     new VariableSha256HashEngine(...) / new VariableMD5HashEngine()
 *                    (failure -> IOException; the factory then logs fatal + System.exit(5),
 *                    HashFunctionPool.java:116-119)
 *   nativeGetChunks  getChunks(byte[], uuid) (VariableSha256HashEngine.java:71-86); a failure
 *                    throws java.io.IOException, as writeCache expects (SparseDedupFile.java:578-580).
 *                    The uuid's hash is the write-stream key: on a device set (all GPUs) one
 *                    stream's buffers stay on one GPU.
 *   nativeGetHash    getHash(byte[]) (VariableSha256HashEngine.java:58-67)
 *   nativeRegister   page-locks a direct ByteBuffer the shim uses as a flush buffer
 *
 * Java arrays are copied in and out with Get/Set<Type>ArrayRegion rather than held with
 * GetPrimitiveArrayCritical: a getChunks call blocks for a GPU pass (~1 ms), and a JVM cannot
 * start a collection while any thread is inside a critical region, so 100+ flush threads holding
 * one would stall the collector.  getChunks copies its byte[] once, with GetByteArrayRegion
 * straight into the engine's pinned staging (sdfs_cdc_get_chunks_fill); getHash goes through a
 * per-thread native buffer.
 *
 * Every `new HipVariableSha256HashEngine` (static, pooled or one-shot) gets a handle to the ONE
 * process-wide engine of its parameters (include/sdfs_cdc.h "Sharing"), so all of SDFS's engine
 * instances feed the same coalescing queue(s).
 *
 * Built against jni/jni_min.h here (no JDK in this image); -DSDFS_USE_JDK_JNI uses the JDK's jni.h.
 */
#ifdef SDFS_USE_JDK_JNI
#include <jni.h>
#else
#include "jni_min.h"
#endif

#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/sdfs_cdc.h"

#define CLS(f) Java_org_opendedup_hashing_HipVariableSha256HashEngine_##f
#define ENG(h) ((sdfs_cdc_engine*)(intptr_t)(h))

/* ---- per-thread native scratch (input copy + result arrays), freed when the thread exits ---- */
struct scratch {
    uint8_t* in;
    size_t in_cap;
    uint32_t* st;
    uint32_t* ln;
    uint8_t* dg;
    size_t out_cap; /* entries */
};

static pthread_key_t g_key;
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

static void scratch_free(void* p) {
    struct scratch* s = (struct scratch*)p;
    if (!s) return;
    free(s->in);
    free(s->st);
    free(s->ln);
    free(s->dg);
    free(s);
}

static void key_init(void) { (void)pthread_key_create(&g_key, scratch_free); }

static struct scratch* scratch_get(size_t in_bytes, size_t entries) {
    pthread_once(&g_once, key_init);
    struct scratch* s = (struct scratch*)pthread_getspecific(g_key);
    if (!s) {
        s = (struct scratch*)calloc(1, sizeof(*s));
        if (!s || pthread_setspecific(g_key, s) != 0) {
            free(s);
            return NULL;
        }
    }
    if (in_bytes > s->in_cap) {
        uint8_t* p = (uint8_t*)realloc(s->in, in_bytes);
        if (!p) return NULL;
        s->in = p;
        s->in_cap = in_bytes;
    }
    if (entries > s->out_cap) {
        uint32_t* a = (uint32_t*)realloc(s->st, entries * sizeof(uint32_t));
        if (a) s->st = a;
        uint32_t* b = (uint32_t*)realloc(s->ln, entries * sizeof(uint32_t));
        if (b) s->ln = b;
        uint8_t* c = (uint8_t*)realloc(s->dg, entries * 32);
        if (c) s->dg = c;
        if (!a || !b || !c) return NULL;
        s->out_cap = entries;
    }
    return s;
}

static void throw_java(JNIEnv* env, const char* cls, const char* msg) {
    if ((*env)->ExceptionCheck(env)) return;
    jclass c = (*env)->FindClass(env, cls);
    if (c) (*env)->ThrowNew(env, c, msg && *msg ? msg : "sdfs_cdc error");
}

/* predKind/predA/predB: the boundary detector's form (sdfs_cdc_params.pred_kind): SDFS_CDC_PRED_MASK
 * -> (fp & predA) == predB, SDFS_CDC_PRED_DIV -> fp % predA == predB (the Java class reads them
 * from the "sdfs.hip.boundary" system property; the default is the bitmask 0xFFF / 0). */
JNIEXPORT jlong JNICALL CLS(nativeCreate)(JNIEnv* env, jclass cls, jlong poly, jint window, jint minLen,
                                          jint maxLen, jint chunkLength, jint algo, jint device, jint predKind,
                                          jlong predA, jlong predB) {
    (void)cls;
    sdfs_cdc_params p;
    sdfs_cdc_params_default(&p, 0);
    p.pred_kind = (uint32_t)predKind;
    if (predKind == SDFS_CDC_PRED_DIV) {
        p.pred_div = (uint64_t)predA;
        p.pred_rem = (uint64_t)predB;
    } else {
        p.pred_mask = (uint64_t)predA;
        p.pred_value = (uint64_t)predB;
    }
    p.poly = (uint64_t)poly;
    p.window = (uint32_t)window;
    p.min_len = (uint32_t)minLen;
    p.max_len = (uint32_t)maxLen;
    p.chunk_length = (uint32_t)chunkLength;
    p.hash_algo = (uint32_t)algo;
    p.device = device;
    sdfs_cdc_engine* e = NULL;
    if (sdfs_cdc_create(&p, &e) != SDFS_CDC_OK) {
        throw_java(env, "java/io/IOException", sdfs_cdc_last_error());
        return 0;
    }
    return (jlong)(intptr_t)e;
}

JNIEXPORT void JNICALL CLS(nativeDestroy)(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    sdfs_cdc_destroy(ENG(h));
}

JNIEXPORT jint JNICALL CLS(nativeSlotCap)(JNIEnv* env, jclass cls, jlong h, jint len) {
    (void)env;
    (void)cls;
    return (jint)sdfs_cdc_slot_cap(ENG(h), (uint64_t)(len > 0 ? len : 0));
}

JNIEXPORT jint JNICALL CLS(nativeDigestLen)(JNIEnv* env, jclass cls, jlong h) {
    (void)env;
    (void)cls;
    return (jint)sdfs_cdc_digest_len(ENG(h));
}

/* The fill callback of sdfs_cdc_get_chunks_fill: the byte[] is copied ONCE, straight into the
 * space the engine reserved for this call in its pinned staging. */
struct fill_ctx {
    JNIEnv* env;
    jbyteArray data;
};

static int fill_from_array(void* ctx, uint8_t* dst, uint32_t len) {
    struct fill_ctx* f = (struct fill_ctx*)ctx;
    (*f->env)->GetByteArrayRegion(f->env, f->data, 0, (jsize)len, (jbyte*)dst);
    return (*f->env)->ExceptionCheck(f->env) ? -1 : 0;
}

/* Chunks data[0 .. data.length) of write stream `key` (the uuid's hashCode as an unsigned 32-bit
 * value, or -1 for none) into starts/lens (jint each) and digests (digest_len bytes each,
 * packed); returns the chunk count, or -1 with a pending IOException. */
JNIEXPORT jint JNICALL CLS(nativeGetChunks)(JNIEnv* env, jclass cls, jlong h, jbyteArray data, jlong key,
                                            jintArray starts, jintArray lens, jbyteArray digests) {
    (void)cls;
    sdfs_cdc_engine* e = ENG(h);
    if (!e || !data || !starts || !lens || !digests) {
        throw_java(env, "java/io/IOException", "null engine or array");
        return -1;
    }
    const jsize n = (*env)->GetArrayLength(env, data);
    const jsize cap = (*env)->GetArrayLength(env, starts);
    const int dl = sdfs_cdc_digest_len(e);
    if (dl <= 0) {
        throw_java(env, "java/io/IOException", sdfs_cdc_last_error());
        return -1;
    }
    if ((*env)->GetArrayLength(env, lens) < cap || (*env)->GetArrayLength(env, digests) < (jsize)((int64_t)cap * dl)) {
        throw_java(env, "java/io/IOException", "output arrays shorter than the chunk capacity");
        return -1;
    }
    struct scratch* s = scratch_get(1, (size_t)(cap > 0 ? cap : 1));
    if (!s) {
        throw_java(env, "java/lang/OutOfMemoryError", "sdfs_cdc_jni scratch");
        return -1;
    }
    struct fill_ctx f = {env, data};
    uint32_t count = 0;
    const uint64_t stream = key < 0 ? SDFS_CDC_NO_STREAM : (uint64_t)key;
    const int rc = sdfs_cdc_get_chunks_fill(e, stream, (uint32_t)n, fill_from_array, &f, s->st, s->ln, s->dg,
                                            (uint32_t)cap, &count);
    if (rc != SDFS_CDC_OK) {
        throw_java(env, "java/io/IOException", sdfs_cdc_last_error());  /* keeps a pending exception */
        return -1;
    }
    (*env)->SetIntArrayRegion(env, starts, 0, (jsize)count, (const jint*)s->st);
    (*env)->SetIntArrayRegion(env, lens, 0, (jsize)count, (const jint*)s->ln);
    (*env)->SetByteArrayRegion(env, digests, 0, (jsize)((int64_t)count * dl), (const jbyte*)s->dg);
    return (*env)->ExceptionCheck(env) ? -1 : (jint)count;
}

/* getHash(data) into out[0 .. digest_len); 0, or -1 with a pending IllegalStateException (the
 * interface's getHash declares no checked exception). */
JNIEXPORT jint JNICALL CLS(nativeGetHash)(JNIEnv* env, jclass cls, jlong h, jbyteArray data, jbyteArray out) {
    (void)cls;
    sdfs_cdc_engine* e = ENG(h);
    if (!e || !data || !out) {
        throw_java(env, "java/lang/IllegalStateException", "null engine or array");
        return -1;
    }
    const jsize n = (*env)->GetArrayLength(env, data);
    const int dl = sdfs_cdc_digest_len(e);
    if ((*env)->GetArrayLength(env, out) < dl) {
        throw_java(env, "java/lang/IllegalStateException", "digest array too short");
        return -1;
    }
    struct scratch* s = scratch_get((size_t)(n > 0 ? n : 1), 1);
    if (!s) {
        throw_java(env, "java/lang/OutOfMemoryError", "sdfs_cdc_jni scratch");
        return -1;
    }
    (*env)->GetByteArrayRegion(env, data, 0, n, (jbyte*)s->in);
    if ((*env)->ExceptionCheck(env)) return -1;
    uint8_t digest[32];
    const int rc = sdfs_cdc_get_hash(e, s->in, (uint64_t)n, digest);
    if (rc != SDFS_CDC_OK) {
        throw_java(env, "java/lang/IllegalStateException", sdfs_cdc_last_error());
        return -1;
    }
    (*env)->SetByteArrayRegion(env, out, 0, dl, (const jbyte*)digest);
    return (*env)->ExceptionCheck(env) ? -1 : 0;
}

/* Page-locks a direct ByteBuffer (ByteBuffer.allocateDirect) for in-place H2D copies by
 * sdfs_cdc_get_chunks_batch; 0, or -1 with a pending IOException. */
JNIEXPORT jint JNICALL CLS(nativeRegister)(JNIEnv* env, jclass cls, jobject direct_buffer) {
    (void)cls;
    void* p = (*env)->GetDirectBufferAddress(env, direct_buffer);
    const jlong n = (*env)->GetDirectBufferCapacity(env, direct_buffer);
    if (!p || n <= 0 || sdfs_cdc_host_register(p, (uint64_t)n) != SDFS_CDC_OK) {
        throw_java(env, "java/io/IOException", p ? sdfs_cdc_last_error() : "not a direct buffer");
        return -1;
    }
    return 0;
}

JNIEXPORT jstring JNICALL CLS(nativeLastError)(JNIEnv* env, jclass cls) {
    (void)cls;
    return (*env)->NewStringUTF(env, sdfs_cdc_last_error());
}
