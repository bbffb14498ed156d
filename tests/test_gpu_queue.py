"""GPU tests of the coalescing queue behind sdfs_cdc_get_chunks / sdfs_cdc_get_hash: many threads
calling ONE shared engine one buffer at a time, as SDFS's flush threads do
(SparseDedupFile.java:100,432; WritableCacheBuffer.java:100-104,640-643).  Every call's chunk
list and digests must equal the oracle's for its own buffer (bit-exact), whatever batch it was
served in."""
import hashlib
import threading

import numpy as np
import pytest

from oracle import cdc_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from sdfs_amd import HipVariableMD5HashEngine, HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from tools import threads as T  # noqa: E402

L = 262144


def _buffers(nbuf, stream0=5000):
    return np.concatenate([O.synth(O.SYNTH_SEED, stream0 + b // 16, (b % 16) * L, L) for b in range(nbuf)])


def _check(res, exp, nbuf, dl):
    counts, st, ln, dg = res
    for b in range(nbuf):
        es, el, ed = exp[b]
        c = counts[b]
        assert st[b, :c].tolist() == list(es) and ln[b, :c].tolist() == list(el), b
        assert (dg[b, :c, :dl] == np.asarray(ed)).all(), b


def test_64_threads_x4_buffers_bit_exact():
    e = HipVariableSha256HashEngine()
    nbuf = 256
    data = _buffers(nbuf)
    b0, r0 = e.queue_stats()  # the native engine is shared with this process's other instances
    r, res = T.getchunks(e, 64, data, L, nbuf, keep=True)
    assert r.first_error == 0
    exp = [O.chunk(data[b * L:(b + 1) * L]) for b in range(nbuf)]
    _check(res, exp, nbuf, 32)
    b1, r1 = e.queue_stats()
    batches, reqs = b1 - b0, r1 - r0
    assert reqs == nbuf and batches < reqs, (batches, reqs)  # concurrent calls shared GPU passes
    # the same calls, one GPU round trip each (SDFS_CDC_FLAG_DIRECT): identical results
    d = HipVariableSha256HashEngine(config=SdfsConfig(direct=True))
    r2, res2 = T.getchunks(d, 16, data, L, nbuf, keep=True)
    assert r2.first_error == 0
    for x, y in zip(res, res2):
        assert np.array_equal(x, y)
    assert d.queue_stats() == (0, 0)
    e.destroy()
    d.destroy()


def test_threads_gethash_md5_and_sha256():
    data = _buffers(96, 6000)
    for eng, hf in ((HipVariableSha256HashEngine(), hashlib.sha256), (HipVariableMD5HashEngine(), hashlib.md5)):
        r, dg = T.gethash(eng, 32, data, L, 96, keep=True)
        assert r.first_error == 0
        for b in range(96):
            assert dg[b].tobytes() == hf(data[b * L:(b + 1) * L].tobytes()).digest(), b
        eng.destroy()


def test_mixed_lengths_chunks_and_hashes_from_python_threads():
    """Write-accelerator runs of arbitrary length (WritableCacheBuffer.java:641-643) and getHash
    calls mixed with full buffers: ragged and hash requests share slots."""
    e = HipVariableSha256HashEngine()
    rng = np.random.default_rng(11)
    jobs = []
    for i in range(120):
        kind = i % 4
        n = L if kind == 0 else int(rng.integers(1, L + 1))
        jobs.append((kind, O.synth(O.SYNTH_SEED, 7000 + i, 0, n).tobytes()))
    errors = []

    def work(k):
        try:
            for kind, data in jobs[k::12]:
                if kind == 3:
                    assert e.getHash(data) == hashlib.sha256(data).digest()
                else:
                    st, ln, dg = e.chunk_arrays(data)
                    es, el, ed = O.chunk(data)
                    assert st.tolist() == es.tolist() and ln.tolist() == el.tolist() and (dg == ed).all()
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    th = [threading.Thread(target=work, args=(k,)) for k in range(12)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:3]
    e.destroy()


def test_queue_4k_mean_mix_and_backup_buffers():
    """min-variable-segment-size=2 with an 11-bit predicate (the 4 KiB-mean mix), and 40 MiB
    BACKUP_VOLUME buffers (VolumeConfigWriter.java:298-307) through the queue."""
    prm = O.Params(min_len=2047, pred_mask=0x7FF)
    e = HipVariableSha256HashEngine(config=SdfsConfig(min_len=2047, pred_mask=0x7FF))
    data = _buffers(64, 8000)
    r, res = T.getchunks(e, 32, data, L, 64, keep=True)
    assert r.first_error == 0
    _check(res, [O.chunk(data[b * L:(b + 1) * L], prm) for b in range(64)], 64, 32)
    e.destroy()
    b = HipVariableSha256HashEngine(config=SdfsConfig.backup_volume())
    big = [O.synth(O.SYNTH_SEED, 8100 + i, 0, 40960 * 1024) for i in range(3)]
    out = [None] * 3

    def work(i):
        out[i] = b.chunk_arrays(big[i])

    th = [threading.Thread(target=work, args=(i,)) for i in range(3)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i in range(3):
        es, el, ed = O.chunk(big[i], O.Params(max_len=131072))
        st, ln, dg = out[i]
        assert st.tolist() == es.tolist() and ln.tolist() == el.tolist() and (dg == ed).all(), i
    b.destroy()


@pytest.mark.parametrize("mix", [(4095, 0xFFF), (2047, 0x7FF)], ids=["default", "mix4k"])
def test_early_completion_callers_leave_before_their_pass(mix):
    """A pass's callers return as their own buffer's last chunk is fingerprinted (the kernel sets
    the buffer's ready word in the pinned image), not when the pass's longest chunk is.  Passes
    mixing buffers of maxLen-forced chunks (0x55 bytes: no boundary candidate at all, so every
    chunk is a 32 KiB chain) with random buffers: every call's results are bit-exact, and calls
    did complete early."""
    prm = O.Params(min_len=mix[0], pred_mask=mix[1])
    e = HipVariableSha256HashEngine(config=SdfsConfig(min_len=mix[0], pred_mask=mix[1]))
    bufs = []
    for i in range(96):
        if i % 8 == 3:
            b = np.full(L, 0x55, np.uint8)
            b[:100] = O.synth(O.SYNTH_SEED, 9100 + i, 0, 100)
        else:
            b = O.synth(O.SYNTH_SEED, 9000 + i, 0, L)
        bufs.append(b)
    exp = [O.chunk(b.tobytes(), prm) for b in bufs]
    e0 = e.queue_early()
    errors = []

    def work(t):
        try:
            for k in range(3):
                i = (t * 3 + k) % len(bufs)
                st, ln, dg = e.chunk_arrays(bufs[i].tobytes())
                es, el, ed = exp[i]
                assert st.tolist() == es.tolist() and ln.tolist() == el.tolist() and (dg == ed).all(), i
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    th = [threading.Thread(target=work, args=(t,)) for t in range(32)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:3]
    # the C driver (no GIL between calls): the JNI glue's entry point at 48 threads
    data = np.concatenate(bufs[:64])
    r, res = T.getchunks(e, 48, data, L, 192, keep=True, mode="fill")
    assert r.first_error == 0
    _check(res, exp[:64], 64, 32)
    assert e.queue_early() > e0
    e.destroy()
