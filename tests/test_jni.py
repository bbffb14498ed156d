"""The JNI glue (jni/sdfs_cdc_jni.c, compiled against jni/jni_min.h) driven through a stand-in
JNIEnv (tests/jni/jni_stub.c): the native methods a JVM would call for
org.opendedup.hashing.HipVariableSha256HashEngine (jni/HipVariableSha256HashEngine.java), i.e.
AbstractHashEngine.getChunks / getHash (AbstractHashEngine.java:24-39,
VariableSha256HashEngine.java:58-86).  CPU tests: symbols and the no-device error path; GPU
tests: results against the oracle, and the error convention (IOException from getChunks,
SparseDedupFile.java:578-580)."""
import ctypes
import hashlib
import os

import numpy as np
import pytest

from oracle import cdc_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GLUE = os.path.join(ROOT, "jni", "libsdfs_cdc_jni.so")
STUB = os.path.join(ROOT, "tests", "jni", "libjni_stub.so")
PFX = "Java_org_opendedup_hashing_HipVariableSha256HashEngine_"
NATIVES = ["nativeCreate", "nativeDestroy", "nativeSlotCap", "nativeDigestLen", "nativeGetChunks", "nativeGetHash",
           "nativeRegister", "nativeLastError"]
VP = ctypes.c_void_p


class Jni:
    def __init__(self):
        from sdfs_amd import _lib
        _lib.load()  # torch's HIP runtime first, then the engine (same order as the package)
        self.stub = ctypes.CDLL(STUB)
        self.glue = ctypes.CDLL(GLUE)
        s = self.stub
        s.stub_env.restype = VP
        s.stub_new_array.restype = VP
        s.stub_new_array.argtypes = [ctypes.c_int, ctypes.c_int32, VP]
        s.stub_array_data.restype = VP
        s.stub_array_data.argtypes = [VP]
        s.stub_free.argtypes = [VP]
        s.stub_take_exception.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
        g = self.glue
        f = getattr(g, PFX + "nativeCreate")
        f.restype = ctypes.c_int64
        f.argtypes = [VP, VP, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int32,
                      ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int64, ctypes.c_int64]
        getattr(g, PFX + "nativeDestroy").argtypes = [VP, VP, ctypes.c_int64]
        for n in ("nativeSlotCap",):
            getattr(g, PFX + n).argtypes = [VP, VP, ctypes.c_int64, ctypes.c_int32]
        getattr(g, PFX + "nativeDigestLen").argtypes = [VP, VP, ctypes.c_int64]
        getattr(g, PFX + "nativeGetChunks").argtypes = [VP, VP, ctypes.c_int64, VP, ctypes.c_int64, VP, VP, VP]
        getattr(g, PFX + "nativeGetHash").argtypes = [VP, VP, ctypes.c_int64, VP, VP]
        getattr(g, PFX + "nativeRegister").argtypes = [VP, VP, VP]
        self.env = s.stub_env()

    def call(self, name, *args):
        return getattr(self.glue, PFX + name)(self.env, None, *args)

    def exception(self):
        c, m = ctypes.create_string_buffer(128), ctypes.create_string_buffer(512)
        return (c.value.decode(), m.value.decode()) if self.stub.stub_take_exception(c, 128, m, 512) else None

    def byte_array(self, data: bytes):
        return self.stub.stub_new_array(1, len(data), data)

    def new(self, kind, n):
        return self.stub.stub_new_array(kind, n, None)

    def read(self, arr, dtype, n):
        return np.ctypeslib.as_array(ctypes.cast(self.stub.stub_array_data(arr), ctypes.POINTER(ctypes.c_uint8)),
                                     (n * np.dtype(dtype).itemsize,)).view(dtype).copy()


def test_glue_exports_every_native_method():
    lib = ctypes.CDLL(GLUE)
    missing = [n for n in NATIVES if not hasattr(lib, PFX + n)]
    assert not missing, missing
    # the Java source declares exactly these natives
    java = open(os.path.join(ROOT, "jni", "HipVariableSha256HashEngine.java")).read()
    for n in NATIVES:
        assert f" {n}(" in java, n


def test_create_without_device_throws_ioexception():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    j = Jni()
    h = j.call("nativeCreate", O.POLY, 48, 4095, 32768, 262144, 0, 0, 0, 0xFFF, 0)
    assert h == 0
    cls, msg = j.exception()
    assert cls == "java/io/IOException" and msg


@pytest.mark.gpu
@pytest.mark.parametrize("algo", [0, 1, 2])
def test_jni_get_chunks_and_get_hash_vs_oracle(algo):
    j = Jni()
    h = j.call("nativeCreate", O.POLY, 48, 4095, 32768, 262144, algo, 0, 0, 0xFFF, 0)
    assert h and j.exception() is None
    dl = j.call("nativeDigestLen", h)
    assert dl == (32, 20, 16)[algo]
    prm = O.Params(hash_algo=algo)
    for n in (1, 4096, 65536 + 17, 262144):
        data = O.synth(O.SYNTH_SEED, 3000 + n % 97, 0, n).tobytes()
        cap = j.call("nativeSlotCap", h, n)
        arr = j.byte_array(data)
        st, ln, dg = j.new(2, cap), j.new(2, cap), j.new(1, cap * dl)
        key = -1 if n % 2 else 0x9E3779B9  # no stream / a uuid's hashCode (unsigned)
        cnt = j.call("nativeGetChunks", h, arr, key, st, ln, dg)
        assert j.exception() is None
        es, el, ed = O.chunk(data, prm)
        assert cnt == len(es)
        assert j.read(st, np.int32, cnt).tolist() == es.tolist()
        assert j.read(ln, np.int32, cnt).tolist() == el.tolist()
        assert j.read(dg, np.uint8, cnt * dl).tobytes() == ed.tobytes()
        out = j.new(1, dl)
        assert j.call("nativeGetHash", h, arr, out) == 0
        want = (hashlib.md5 if algo == 2 else hashlib.sha256)(data).digest()[:dl]
        assert j.read(out, np.uint8, dl).tobytes() == want
        for a in (arr, st, ln, dg, out):
            j.stub.stub_free(a)
    # capacity too small for the chunk list -> IOException (getChunks' checked exception)
    data = O.synth(O.SYNTH_SEED, 77, 0, 262144).tobytes()
    arr = j.byte_array(data)
    st, ln, dg = j.new(2, 2), j.new(2, 2), j.new(1, 2 * dl)
    assert j.call("nativeGetChunks", h, arr, -1, st, ln, dg) == -1
    cls, msg = j.exception()
    assert cls == "java/io/IOException" and "cap" in msg
    # a second Java instance with the same parameters shares the native engine (one queue)
    from sdfs_amd import _lib
    lib = _lib.load()
    k = lib.sdfs_cdc_share_count(ctypes.c_void_p(h))  # (other live instances of this process count too)
    h2 = j.call("nativeCreate", O.POLY, 48, 4095, 32768, 262144, algo, 0, 0, 0xFFF, 0)
    assert h2 and h2 != h and j.exception() is None
    assert lib.sdfs_cdc_share_count(ctypes.c_void_p(h)) == k + 1 == lib.sdfs_cdc_share_count(ctypes.c_void_p(h2))
    j.call("nativeDestroy", h)
    assert lib.sdfs_cdc_share_count(ctypes.c_void_p(h2)) == k
    # the destroyed handle is refused (EINVAL: no use after free); the other still works
    assert lib.sdfs_cdc_share_count(ctypes.c_void_p(h)) == _lib.EINVAL
    st, ln, dg = j.new(2, 66), j.new(2, 66), j.new(1, 66 * dl)
    assert j.call("nativeGetChunks", h2, arr, 7, st, ln, dg) == len(O.chunk(data, prm)[0])
    j.call("nativeDestroy", h2)


@pytest.mark.gpu
def test_fill_failure_is_einval_with_its_own_message():
    """A fill callback that fails (the JNI glue's GetByteArrayRegion raising) fails that call only:
    SDFS_CDC_EINVAL with "fill callback failed" in sdfs_cdc_last_error (not an earlier, unrelated
    message), count 0, the Java exception left pending; the engine keeps serving calls."""
    from sdfs_amd import _lib
    from sdfs_amd.engine import HipVariableSha256HashEngine
    lib = _lib.load()
    eng = HipVariableSha256HashEngine(device=0)
    data = O.synth(O.SYNTH_SEED, 4242, 0, 262144).tobytes()
    es, el, ed = O.chunk(data)
    cap = eng.slot_cap(len(data))
    st, ln = np.zeros(cap, np.uint32), np.zeros(cap, np.uint32)
    dg = np.zeros((cap, 32), np.uint8)
    n = ctypes.c_uint32(99)
    cb = _lib.FILL_FN(lambda ctx, dst, ln_: -7)
    rc = lib.sdfs_cdc_get_chunks_fill(eng._h, _lib.NO_STREAM, len(data), cb, None, st.ctypes.data, ln.ctypes.data,
                                      dg.ctypes.data, cap, ctypes.byref(n))
    assert rc == _lib.EINVAL and n.value == 0
    assert "fill callback failed (-7)" in lib.sdfs_cdc_last_error().decode()
    s2, l2, d2 = eng.chunk_arrays(data, fill=True)  # the engine still serves calls
    assert s2.tolist() == es.tolist() and l2.tolist() == el.tolist() and (d2 == ed).all()
    eng.destroy()
    # through the glue: the injected ArrayIndexOutOfBoundsException stays the pending exception
    j = Jni()
    h = j.call("nativeCreate", O.POLY, 48, 4095, 32768, 262144, 0, 0, 0, 0xFFF, 0)
    assert h and j.exception() is None
    arr = j.byte_array(data)
    c = j.call("nativeSlotCap", h, len(data))
    st, ln, dg = j.new(2, c), j.new(2, c), j.new(1, c * 32)
    j.stub.stub_fail_next_region()
    assert j.call("nativeGetChunks", h, arr, -1, st, ln, dg) == -1
    cls, _ = j.exception()
    assert cls == "java/lang/ArrayIndexOutOfBoundsException"
    assert "fill callback failed" in lib.sdfs_cdc_last_error().decode()
    assert j.call("nativeGetChunks", h, arr, -1, st, ln, dg) == len(es) and j.exception() is None
    for a in (arr, st, ln, dg):
        j.stub.stub_free(a)
    j.call("nativeDestroy", h)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,a,b", [(1, 4099, 0), (1, 8192, 8191), (0, 0x7FF, 0x15)])
def test_jni_boundary_detector_forms_vs_oracle(kind, a, b):
    """The Java class passes the detector form of "sdfs.hip.boundary" (mask:M:V / div:D:R) through
    nativeCreate; every form chunks like the oracle with the same detector."""
    j = Jni()
    h = j.call("nativeCreate", O.POLY, 48, 4095, 32768, 262144, 0, 0, kind, a, b)
    assert h and j.exception() is None
    prm = (O.Params(pred_kind=O.PRED_DIV, pred_div=a, pred_rem=b) if kind == 1 else
           O.Params(pred_mask=a, pred_value=b))
    for n in (5000, 262144):
        data = O.synth(O.SYNTH_SEED, 5100 + n % 89, 0, n).tobytes()
        cap = j.call("nativeSlotCap", h, n)
        arr = j.byte_array(data)
        st, ln, dg = j.new(2, cap), j.new(2, cap), j.new(1, cap * 32)
        cnt = j.call("nativeGetChunks", h, arr, -1, st, ln, dg)
        assert j.exception() is None
        es, el, ed = O.chunk(data, prm)
        assert cnt == len(es)
        assert j.read(st, np.int32, cnt).tolist() == es.tolist()
        assert j.read(ln, np.int32, cnt).tolist() == el.tolist()
        assert j.read(dg, np.uint8, cnt * 32).tobytes() == ed.tobytes()
        for x in (arr, st, ln, dg):
            j.stub.stub_free(x)
    j.call("nativeDestroy", h)
