"""Dedup-hit index (include/sdfs_index.h).

CPU: the oracle's per-buffer writeCache restatement (claims per buffer, one put per distinct
fingerprint) against the flat rule the GPU implements (first record of a new fingerprint in
record order is inserted, every other record is a duplicate), and the loud failure without a GPU.
GPU: the HIP index, through the C-ABI, against the oracle — random record batches with
duplicates inside a buffer, across buffers and across batches; the engine's own fingerprint
table of a 50 %-duplicate workload; the device-count path; a full index; lookups.
Parity status: pinned by the reference's control flow (SparseDedupFile.java:435-446,541-560,
RocksDBMap.java:785-870); the reference holds no fixtures for this step."""
import ctypes
import random

import numpy as np
import pytest

from oracle import dedup_oracle as D
from sdfs_amd import _lib


def _random_batch(rng, nbuf, per_buf, pool, dup_rate):
    """Digests for nbuf buffers (buffer ids ascending); some repeat within/between buffers."""
    digests, bids = [], []
    for b in range(nbuf):
        for _ in range(rng.randint(0, per_buf)):
            if pool and rng.random() < dup_rate:
                d = rng.choice(pool)
            else:
                d = bytes(rng.getrandbits(8) for _ in range(32))
                pool.append(d)
            digests.append(d)
            bids.append(b)
    return digests, bids


def _flat_rule(m, digests, pos_base):
    dup, loc, new = [], [], []
    for i, d in enumerate(digests):
        e = m.get(d)
        if e is None:
            m[d] = [pos_base + len(new), 1]
            new.append(i)
            dup.append(0)
        else:
            e[1] += 1
            dup.append(1)
        loc.append(m[d][0])
    return dup, loc, new


def test_oracle_per_buffer_claims_equal_flat_rule():
    rng = random.Random(7)
    m = D.HashesMap()
    flat = {}
    pool = []
    base = 1000
    for batch in range(5):
        digests, bids = _random_batch(rng, 40, 30, pool, 0.4)
        dup, loc, new = D.write_buffers(m, digests, bids, base)
        fdup, floc, fnew = _flat_rule(flat, digests, base)
        assert (dup, loc, new) == (fdup, floc, fnew)
        base += len(new)
    assert {k: (e.pos, e.refcount) for k, e in m.entries.items()} == {k: tuple(v) for k, v in flat.items()}


def test_oracle_claims_counted_per_buffer():
    # one buffer with the same chunk three times: inserted once with refcount 3
    # (SparseDedupFile.java:435-446 claims, RocksDBMap.java:857-864 ct = references)
    m = D.HashesMap()
    dup, loc, new = D.write_buffers(m, [b"a" * 32, b"a" * 32, b"b" * 32, b"a" * 32], [0, 0, 0, 0], 5)
    assert dup == [0, 1, 0, 1] and loc == [5, 5, 6, 5] and new == [0, 2]
    assert m.entries[b"a" * 32].refcount == 3
    # a later buffer hits: refcount += claims, every record a duplicate
    dup, loc, new = D.write_buffers(m, [b"a" * 32, b"a" * 32], [1, 1], 7)
    assert dup == [1, 1] and loc == [5, 5] and new == []
    assert m.entries[b"a" * 32].refcount == 5


def test_index_create_fails_loudly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    h = ctypes.c_void_p()
    assert _lib.load().sdfs_cdc_index_create(0, 1024, ctypes.byref(h)) == _lib.ENODEV and not h.value
    from sdfs_amd.index import HipHashesMap
    with pytest.raises(_lib.SdfsCdcError):
        HipHashesMap(1024)


# ------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------
def _records(digests, bids):
    n = len(digests)
    rec = np.zeros((n, 48), dtype=np.uint8)
    for i, (d, b) in enumerate(zip(digests, bids)):
        rec[i, :32] = np.frombuffer(d.ljust(32, b"\0"), dtype=np.uint8)
        rec[i, 32:40] = np.frombuffer(int(b).to_bytes(8, "little"), dtype=np.uint8)
        rec[i, 40:48] = np.frombuffer((i * 4096).to_bytes(4, "little") + (4096).to_bytes(4, "little"),
                                      dtype=np.uint8)
    return rec


def _put(ix, torch, rec_np, pos_base, count=None):
    rec = torch.from_numpy(rec_np).cuda()
    cnt = None if count is None else torch.tensor([count], dtype=torch.int32, device="cuda")
    dup, loc, new, nc = ix.put_records(rec, cnt, pos_base)
    torch.cuda.synchronize()
    k = int(nc.item())
    n = rec_np.shape[0] if count is None else count
    return dup.cpu().numpy()[:n].tolist(), loc.cpu().numpy()[:n].tolist(), new.cpu().numpy()[:k].tolist()


@pytest.mark.gpu
def test_index_random_batches_vs_oracle():
    torch = pytest.importorskip("torch")
    from sdfs_amd.index import HipHashesMap
    rng = random.Random(11)
    ix = HipHashesMap(1 << 16)
    m = D.HashesMap()
    pool = []
    base = 1 << 40
    for batch in range(6):
        digests, bids = _random_batch(rng, 200, 40, pool, 0.35 if batch else 0.1)
        # short fingerprints (HASH160 / MD5 records are zero-padded) collide only when equal
        if batch == 3:
            digests = [d[:20] for d in digests]
        dup, loc, new = _put(ix, torch, _records(digests, bids), base)
        edup, eloc, enew = D.write_buffers(m, [d.ljust(32, b"\0") for d in digests], bids, base)
        assert dup == edup, batch
        assert loc == eloc, batch
        assert new == enew, batch
        base += len(new)
    assert ix.getSize() == len(m.entries)
    keys = list(m.entries)[:500]
    pos, ref = ix.get_digests(ix._digest_tensor(keys))
    assert pos.cpu().tolist() == [m.entries[k].pos for k in keys]
    assert ref.cpu().tolist() == [m.entries[k].refcount for k in keys]
    assert ix.get(b"\x01" * 32) == -1 and not ix.containsKey(b"\x02" * 32)
    ix.destroy()


@pytest.mark.gpu
def test_index_batches_from_two_streams_apply_in_call_order():
    """Batches enqueued back to back on different streams (flush threads with their own
    streams) apply in call order: the second sees every fingerprint the first inserted."""
    torch = pytest.importorskip("torch")
    from sdfs_amd.index import HipHashesMap
    rng = random.Random(21)
    ix = HipHashesMap(1 << 18)
    digests, bids = _random_batch(rng, 6000, 20, [], 0.0)
    rec = torch.from_numpy(_records(digests, bids)).cuda()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(s1):
        d1, l1, _, n1 = ix.put_records(rec, None, 0, stream=s1.cuda_stream)
    with torch.cuda.stream(s2):
        d2, l2, _, n2 = ix.put_records(rec, None, 1 << 30, stream=s2.cuda_stream)
    torch.cuda.synchronize()
    m = D.HashesMap()
    edup, eloc, _ = D.write_buffers(m, [d.ljust(32, b"\0") for d in digests], bids, 0)
    assert d1.cpu().tolist() == edup and l1.cpu().tolist() == eloc
    assert int(n2.item()) == 0 and all(d2.cpu().tolist()) and l2.cpu().tolist() == l1.cpu().tolist()
    ix.destroy()


@pytest.mark.gpu
def test_index_device_count_and_empty_batch():
    torch = pytest.importorskip("torch")
    from sdfs_amd.index import HipHashesMap
    rng = random.Random(3)
    ix = HipHashesMap(4096)
    digests, bids = _random_batch(rng, 20, 20, [], 0.3)
    rec = _records(digests, bids)
    half = len(digests) // 2
    dup, loc, new = _put(ix, torch, rec, 0, count=half)  # only the first `half` records are valid
    m = D.HashesMap()
    edup, eloc, enew = D.write_buffers(m, digests[:half], bids[:half], 0)
    assert (dup, loc, new) == (edup, eloc, enew)
    assert ix.getSize() == len(m.entries)
    d0, l0, n0 = _put(ix, torch, rec[:0], 0)
    assert d0 == [] and n0 == []
    ix.destroy()


@pytest.mark.gpu
def test_index_epoch_wrap_keeps_dedup():
    """A batch's insertion stamp must not outlive the batch: with the epoch counter wrapped so that
    a later batch reuses an earlier batch's stamp, re-putting the same fingerprints finds every
    one of them (a surviving stamp made the probe skip the slot and insert twice)."""
    torch = pytest.importorskip("torch")
    from sdfs_amd.index import HipHashesMap
    rng = random.Random(17)
    ix = HipHashesMap(4096)
    lib = _lib.load()
    digests = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(300)]
    rec = _records(digests, list(range(300)))
    _lib.check(lib.sdfs_cdc_index_set_epoch(ix._h, 0x7FFFFFFE))  # next batch: the last epoch
    dup, loc, new = _put(ix, torch, rec, 1000)
    assert sum(dup) == 0 and len(new) == 300
    _lib.check(lib.sdfs_cdc_index_set_epoch(ix._h, 0x7FFFFFFE))  # the same stamp again
    dup2, loc2, new2 = _put(ix, torch, rec, 5000)
    assert all(d == 1 for d in dup2) and new2 == [] and loc2 == loc
    dup3, _, new3 = _put(ix, torch, rec, 9000)  # epoch wraps to 1 here
    assert all(d == 1 for d in dup3) and new3 == []
    assert ix.getSize() == 300
    pos, ref = ix.get_digests(ix._digest_tensor(digests[:10]))
    assert ref.cpu().tolist() == [3] * 10
    ix.destroy()


@pytest.mark.gpu
def test_index_full_raises():
    torch = pytest.importorskip("torch")
    from sdfs_amd.index import HipHashesMap
    ix = HipHashesMap(100)  # 128 slots, 112 usable
    cap = ix.getMaxSize()
    rng = random.Random(5)
    digests = [bytes(rng.getrandbits(8) for _ in range(32)) for _ in range(cap)]
    _put(ix, torch, _records(digests, [0] * cap), 0)
    assert ix.getSize() == cap
    with pytest.raises(_lib.SdfsCdcError) as ei:
        _put(ix, torch, _records([b"\x07" * 32], [1]), 0)
    assert ei.value.code == _lib.ECAP
    # a batch of pure duplicates still fits once the bound is refreshed? no: the bound is the
    # batch size, so any non-empty batch is refused on a full index (HashtableFullException)
    ix.destroy()


@pytest.mark.gpu
def test_index_on_engine_records_50pct_duplicate_buffers():
    """configs[2] shape end to end: CDC + fingerprints on the GPU, then the index on the
    engine's own record table; duplicate buffers must be pure hits."""
    torch = pytest.importorskip("torch")
    from sdfs_amd import HipVariableSha256HashEngine
    from sdfs_amd.device import DeviceBatch
    from sdfs_amd.index import HipHashesMap
    e = HipVariableSha256HashEngine()
    nbuf = 256
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=262144)
    batch.fill_streams(first_stream=300, bufs_per_stream=64)
    rng = np.random.default_rng(9)
    v = batch.data.view(nbuf, 262144)
    fresh, copies = [0], {}
    for b in range(1, nbuf):
        if rng.random() < 0.5:
            fresh.append(b)
        else:
            s = int(rng.choice(fresh))
            v[b].copy_(v[s])
            copies[b] = s
    batch.run()
    torch.cuda.synchronize()
    recs = batch.record_table()
    n = recs.shape[0]
    ix = HipHashesMap(1 << 20)
    dup, loc, new, nc = ix.put_records(recs, batch.total, pos_base=0)
    torch.cuda.synchronize()
    host = recs.cpu().numpy()
    digests = [bytes(r[:32]) for r in host]
    bids = [int.from_bytes(bytes(r[32:40]), "little") for r in host]
    m = D.HashesMap()
    edup, eloc, enew = D.write_buffers(m, digests, bids, 0)
    assert dup.cpu().numpy()[:n].tolist() == edup
    assert loc.cpu().numpy()[:n].tolist() == eloc
    assert new.cpu().numpy()[:int(nc.item())].tolist() == enew
    dupm = np.array(edup, dtype=bool)
    bid = np.array(bids)
    for b in copies:
        assert dupm[bid == b].all()  # a copied buffer is all hits
    assert ix.getSize() == len(m.entries)
    ix.destroy()
    e.destroy()
