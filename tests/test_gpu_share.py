"""GPU tests of the process-wide engine (include/sdfs_cdc.h "Sharing" / "Devices", ABI 2).

SDFS makes many hash-engine instances — static singletons (SparseDedupFile.java:100,
HashBlobArchive.java:140, FileIOServiceImpl.java:152), a pool of one per concurrent
write-accelerator caller (HashFunctionPool.java:73-86, WritableCacheBuffer.java:640,779) and
one-shot ones (HashStore.java:68) — and the pool may destroy an instance while another thread
still calls it (HashFunctionPool.java:98-100).  Checked here on the GPU, every result against the
oracle (bit-exact):
* instances with equal parameters share ONE native engine: calls on different handles are served
  by the same GPU passes (queue statistics), and give the oracle's results;
* the JNI glue's entry point (fill callback into pinned staging) and the stream-keyed one;
* destroying a handle while other threads are in its calls;
* a device set (device = -1: every gfx950 GPU of the box) through the batched host path, the
  device-resident path (routed by the data pointer's device) and the in-process RCCL all-gather
  of the fingerprint tables;
* a 40 MiB BACKUP_VOLUME buffer through the queue (its sectioned cut walk's scratch is sized when
  the queue starts)."""
import ctypes
import threading

import numpy as np
import pytest

from oracle import cdc_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig, _lib  # noqa: E402
from sdfs_amd.device import DeviceBatch  # noqa: E402
from tools import threads as T  # noqa: E402

L = 262144


def _buffers(nbuf, stream0):
    return np.concatenate([O.synth(O.SYNTH_SEED, stream0 + b // 16, (b % 16) * L, L) for b in range(nbuf)])


def _check(res, data, nbuf, prm=None):
    counts, st, ln, dg = res
    for b in range(nbuf):
        es, el, ed = O.chunk(data[b * L:(b + 1) * L], prm or O.Params())
        c = counts[b]
        assert st[b, :c].tolist() == es.tolist() and ln[b, :c].tolist() == el.tolist(), b
        assert (dg[b, :c, :32] == ed).all(), b


def test_instances_share_one_engine_and_its_gpu_passes():
    # (other tests of this process may hold instances of the same parameters: counts are relative)
    engines = [HipVariableSha256HashEngine() for _ in range(4)]
    k = engines[0].share_count()
    assert k >= 4 and all(e.share_count() == k for e in engines)
    other = HipVariableSha256HashEngine(config=SdfsConfig(min_len=2047, pred_mask=0x7FF, max_len=32000))
    assert other.share_count() == 1 and engines[0].share_count() == k  # other parameters: its own engine
    b0, r0 = engines[0].queue_stats()
    nbuf = 192
    data = _buffers(nbuf, 9100)
    for mode in ("copy", "fill", "stream"):
        r, res = T.getchunks(None, 48, data, L, nbuf, keep=True, engines=engines, mode=mode)
        assert r.first_error == 0, mode
        _check(res, data, nbuf)
    b1, r1 = engines[0].queue_stats()
    assert r1 - r0 == 3 * nbuf  # every call of every handle went through the one shared queue
    assert b1 - b0 < r1 - r0     # ... and calls shared GPU passes
    assert engines[3].queue_stats() == (b1, r1)
    for e in engines[:3]:
        e.destroy()
    assert engines[3].share_count() == k - 3
    st, ln, dg = engines[3].chunk_arrays(data[:L], fill=True)
    es, el, ed = O.chunk(data[:L])
    assert st.tolist() == es.tolist() and ln.tolist() == el.tolist() and (dg == ed).all()
    engines[3].destroy()
    other.destroy()


def test_destroy_while_other_threads_are_in_calls():
    """A handle destroyed while threads are inside its calls: those calls finish with the right
    results, later calls on it fail with EINVAL, the other handle of the engine is unaffected."""
    a = HipVariableSha256HashEngine()
    b = HipVariableSha256HashEngine()
    k = b.share_count()
    lib = _lib.load()
    ha = a._h
    bufs = [O.synth(O.SYNTH_SEED, 9300 + i, 0, L).tobytes() for i in range(8)]
    want = [O.chunk(x) for x in bufs]
    errors, refused, done = [], [0], [0]
    stop = threading.Event()

    def work(k):
        cap = 66
        st = np.zeros(cap, np.uint32)
        ln = np.zeros(cap, np.uint32)
        dg = np.zeros((cap, 32), np.uint8)
        n = ctypes.c_uint32()
        i = k
        while not stop.is_set():
            x = bufs[i % 8]
            h = ha if k % 2 else b._h
            rc = lib.sdfs_cdc_get_chunks(h, x, L, st.ctypes.data, ln.ctypes.data, dg.ctypes.data, cap, ctypes.byref(n))
            if rc == _lib.EINVAL and h is ha:
                refused[0] += 1
            elif rc != 0:
                errors.append(rc)
            else:
                es, el, ed = want[i % 8]
                c = n.value
                if st[:c].tolist() != es.tolist() or ln[:c].tolist() != el.tolist() or not (dg[:c] == ed).all():
                    errors.append("mismatch")
                done[0] += 1
            i += 1

    th = [threading.Thread(target=work, args=(k,)) for k in range(16)]
    for t in th:
        t.start()
    import time
    time.sleep(1.0)
    a.destroy()  # threads are inside calls on ha now
    time.sleep(0.5)
    stop.set()
    for t in th:
        t.join()
    assert not errors, errors[:5]
    assert refused[0] > 0 and done[0] > 50
    assert b.share_count() == k - 1
    b.destroy()


def test_device_set_all_gpus_batch_device_and_allgather():
    """device = -1: a device set of every gfx950 GPU (one on a one-GPU box): the batched host
    path (split across the set), the device-resident path (routed by the pointer's device) and
    the in-process RCCL all-gather of the record tables, all equal to the oracle."""
    e = HipVariableSha256HashEngine(device=_lib.ALL_DEVICES)
    ords = e.device_ordinals()
    n = e.device_count()
    assert n == torch.cuda.device_count() >= 1 and ords == list(range(n))
    # host batch: nbuf buffers, split in contiguous shares over the set
    nbuf = 96 * n
    data = _buffers(nbuf, 9500)
    offs = np.arange(nbuf, dtype=np.uint64) * L
    lens = np.full(nbuf, L, np.uint32)
    _check(e.chunk_batch(data, offs, lens), data, nbuf)
    # device-resident: one batch per device, then the exchange
    per = 48
    batches, streams = [], []
    for d in range(n):
        with torch.cuda.device(d):
            bt = DeviceBatch(e, nbuf=per, buf_len=L, device=f"cuda:{d}")
            bt.fill_streams(first_stream=9600 + 3 * d, bufs_per_stream=16)
            s = torch.cuda.Stream(device=d)
            s.wait_stream(torch.cuda.current_stream(d))  # the fill ran on the current stream
            bt.run(buffer_id_base=d * per, stream=s.cuda_stream)
            batches.append(bt)
            streams.append(s)
    for d in range(n):
        torch.cuda.synchronize(d)
    gathered = []
    for d in range(n):
        cap = batches[d].recs.view(-1, 48).shape[0]
        gathered.append(torch.zeros((n * cap, 48), dtype=torch.uint8, device=f"cuda:{d}"))
    counts, stride = e.allgather_records([b.recs.view(-1, 48) for b in batches], [b.total for b in batches], gathered,
                                         streams=[s.cuda_stream for s in streams])
    for d in range(n):
        torch.cuda.synchronize(d)
    assert counts == [int(b.total.item()) for b in batches] and stride == max(counts)
    for d in range(n):
        host = batches[d].data.cpu().numpy()
        tab = batches[d].record_table().cpu().numpy()
        recs = []
        for b in range(per):
            es, el, ed = O.chunk(host[b * L:(b + 1) * L])
            for k in range(len(es)):
                recs.append(bytes(ed[k]) + int(d * per + b).to_bytes(8, "little") + int(es[k]).to_bytes(4, "little") +
                            int(el[k]).to_bytes(4, "little"))
        assert [bytes(r) for r in tab] == recs, d
        for g in range(n):  # every device received device d's table at d * stride
            got = gathered[g][d * stride: d * stride + counts[d]].cpu().numpy()
            assert np.array_equal(got, tab), (g, d)
    e.destroy()


def test_backup_buffer_through_the_queue_alone_in_its_slot():
    """A 40 MiB BACKUP_VOLUME getChunks (VolumeConfigWriter.java:298-307) next to 256 KiB calls of
    the same engine: it travels in a slot of its own (its sectioned walk's scratch was sized when
    the queue started) and every result equals the oracle's."""
    cfg = SdfsConfig.backup_volume()
    e = HipVariableSha256HashEngine(config=cfg)
    big = O.synth(O.SYNTH_SEED, 9700, 0, 40960 * 1024)
    small = [O.synth(O.SYNTH_SEED, 9701 + i, 0, L) for i in range(6)]
    out = {}

    def work(k):
        x = big if k == 0 else small[k - 1]
        out[k] = e.chunk_arrays(x)

    th = [threading.Thread(target=work, args=(k,)) for k in range(7)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    prm = O.Params(max_len=131072)
    for k in range(7):
        x = big if k == 0 else small[k - 1]
        es, el, ed = O.chunk(x, prm)
        st, ln, dg = out[k]
        assert st.tolist() == es.tolist() and ln.tolist() == el.tolist() and (dg == ed).all(), k
    e.destroy()
