/*
 * org.opendedup.hashing.HipVariableSha256HashEngine — AbstractHashEngine backed by the MI355X
 * engine (libsdfs_cdc.so) through the JNI glue in jni/sdfs_cdc_jni.c.  Source for the SDFS tree
 * (src/org/opendedup/hashing/); this image has no JDK, so it is not compiled here — the glue's
 * native side is compiled and tested against a stub JNIEnv (tests/test_jni.py).
 *
 * Surface: AbstractHashEngine.java:24-39; behaviour: VariableSha256HashEngine.java:41-121
 * (VARIABLE_SHA256 / VARIABLE_SHA256_160) and VariableMD5HashEngine.java:37-108 (VARIABLE_MD5).
 * Selected in HashFunctionPool.getHashEngine() (HashFunctionPool.java:102-121), INTEGRATION.md §1.
 */
package org.opendedup.hashing;

import java.io.IOException;
import java.util.ArrayList;
import java.util.Arrays;
import java.util.List;
import java.util.concurrent.locks.ReentrantReadWriteLock;

import org.opendedup.sdfs.Main;

public final class HipVariableSha256HashEngine implements AbstractHashEngine {
    public static enum HASHTYPE { HASH160, HASH256, MD5 }

    static { System.loadLibrary("sdfs_cdc_jni"); }   // links libsdfs_cdc.so

    private static final long POLY = 10923124345206883L;  // VariableSha256HashEngine.java:41
    private long handle;                                   // sdfs_cdc_engine handle (guarded by lock)
    private final int hashLen;                             // 32, 20 or 16
    // calls hold the read lock, destroy() the write lock: no call ever uses a destroyed handle
    // (HashFunctionPool.destroyObject, HashFunctionPool.java:98-100, may race a borrower)
    private final ReentrantReadWriteLock lock = new ReentrantReadWriteLock();

    /** Every instance with the same parameters shares ONE native engine (all GPUs of the
     *  "sdfs.hip.device" set: -1 = every gfx950 device, the default; an ordinal = that GPU). */
    public HipVariableSha256HashEngine(HASHTYPE ht) throws IOException {
        int algo = ht == HASHTYPE.HASH256 ? 0 : (ht == HASHTYPE.HASH160 ? 1 : 2);  // SDFS_CDC_*
        long[] det = boundaryDetector(System.getProperty("sdfs.hip.boundary", "mask:0xfff:0"));
        handle = nativeCreate(POLY, HashFunctionPool.bytesPerWindow, HashFunctionPool.minLen,
                HashFunctionPool.maxLen, Main.CHUNK_LENGTH, algo, Integer.getInteger("sdfs.hip.device", -1),
                (int) det[0], det[1], det[2]);
        hashLen = nativeDigestLen(handle);
    }

    /** The form of BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR (VariableSha256HashEngine.java:42),
     *  which the rabinwindow jar fixes and SDFS does not configure: "mask:M:V" is the bitmask
     *  detector (fp &amp; M) == V, "div:D:R" the divisor detector fp % D == R (numbers decimal or 0x hex).
     *  tools/java/JarParity.java tells which one (and which constants) a given jar uses. */
    static long[] boundaryDetector(String spec) throws IOException {
        String[] f = spec.trim().split(":");
        if (f.length != 3 || !(f[0].equals("mask") || f[0].equals("div")))
            throw new IOException("sdfs.hip.boundary must be mask:M:V or div:D:R, got " + spec);
        return new long[] {f[0].equals("div") ? 1 : 0, unsigned(f[1], spec), unsigned(f[2], spec)};
    }

    /** A 64-bit unsigned field (decimal or 0x hex, e.g. 0xFFFFFFFFFFFFFFFF); a malformed one is an
     *  IOException naming the property, as the constructor declares. */
    static long unsigned(String v, String spec) throws IOException {
        String t = v.trim();
        try {
            if (t.startsWith("0x") || t.startsWith("0X")) return Long.parseUnsignedLong(t.substring(2), 16);
            return Long.parseUnsignedLong(t);
        } catch (NumberFormatException ex) {
            throw new IOException("sdfs.hip.boundary: bad number '" + v + "' in " + spec, ex);
        }
    }

    @Override public boolean isVariableLength() { return true; }
    @Override public int getMaxLen() { return Main.CHUNK_LENGTH; }                 // :106-109
    @Override public int getMinLen() { return HashFunctionPool.minLen; }           // :111-114
    @Override public void setSeed(int seed) { }                                     // :116-120
    @Override public void destroy() {
        lock.writeLock().lock();
        try {
            if (handle != 0) { nativeDestroy(handle); handle = 0; }
        } finally { lock.writeLock().unlock(); }
    }

    @Override public byte[] getHash(byte[] data) {                                  // :58-67
        byte[] out = new byte[hashLen];
        lock.readLock().lock();
        try {
            if (handle == 0) throw new IllegalStateException("engine destroyed");
            nativeGetHash(handle, data, out);   // throws IllegalStateException on a device error
        } finally { lock.readLock().unlock(); }
        return out;
    }

    /** Thread-safe: SDFS's flush threads share one engine (SparseDedupFile.java:100); concurrent
     *  calls are coalesced into shared GPU passes inside the library. */
    @Override public List<Finger> getChunks(byte[] data, String uuid) throws IOException {  // :71-86
        int[] starts, lens;
        byte[] digests;
        int n;
        long key = uuid == null ? -1L : (uuid.hashCode() & 0xffffffffL);  // write-stream key
        lock.readLock().lock();
        try {
            if (handle == 0) throw new IOException("engine destroyed");
            int cap = nativeSlotCap(handle, data.length);
            starts = new int[cap];
            lens = new int[cap];
            digests = new byte[cap * hashLen];
            n = nativeGetChunks(handle, data, key, starts, lens, digests);  // IOException on failure
        } finally { lock.readLock().unlock(); }
        ArrayList<Finger> al = new ArrayList<Finger>(n);
        for (int i = 0; i < n; i++) {
            Finger f = new Finger(uuid);
            f.start = starts[i];
            f.len = lens[i];
            f.chunk = Arrays.copyOfRange(data, starts[i], starts[i] + lens[i]);  // outlives the buffer
            f.hash = Arrays.copyOfRange(digests, i * hashLen, (i + 1) * hashLen);
            al.add(f);
        }
        return al;
    }

    /** Page-locks a direct flush buffer (ByteBuffer.allocateDirect) for in-place H2D copies. */
    public static void register(java.nio.ByteBuffer direct) throws IOException { nativeRegister(direct); }

    private static native long nativeCreate(long poly, int window, int minLen, int maxLen,
                                            int chunkLength, int algo, int device, int predKind,
                                            long predA, long predB) throws IOException;
    private static native void nativeDestroy(long h);
    private static native int nativeSlotCap(long h, int len);
    private static native int nativeDigestLen(long h);
    private static native int nativeGetChunks(long h, byte[] data, long key, int[] starts, int[] lens,
                                              byte[] digests) throws IOException;
    private static native int nativeGetHash(long h, byte[] data, byte[] out);
    private static native int nativeRegister(java.nio.ByteBuffer direct) throws IOException;
    private static native String nativeLastError();
}
