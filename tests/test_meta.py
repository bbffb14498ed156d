"""Per-buffer metadata images (include/sdfs_meta.h).

CPU: the restatement (oracle/meta_oracle.py) of HashLocPair.asArray / SparseDataChunk.getBytes /
the LongByteArrayMap slot length, and the C-ABI's slot length.  GPU: the device images of a
whole batch (duplicate buffers, intra-buffer duplicate chunks, MD5 engine, overflow) against the
restatement fed with the same chunk lists and index outputs.
Parity status: pinned by the reference's own serialisation code (no reference fixtures)."""
import struct

import numpy as np
import pytest

from oracle import dedup_oracle as D
from oracle import meta_oracle as M
from sdfs_amd import _lib


def test_slot_length_matches_longbytearraymap():
    # defaults: hashLength 32, CHUNK_LENGTH 256 KiB, minLen 4095 -> max_hash_cluster 64,
    # MAX_ELEMENTS_PER_AR 128, BAL 56 -> 13 + 56 * 128
    assert M.slot_bytes(32, 262144, 4095) == 7181
    lib = _lib.load()
    for h, cl, mn in [(32, 262144, 4095), (16, 262144, 4095), (32, 40960 * 1024, 4095), (32, 262144, 2047)]:
        assert lib.sdfs_cdc_map_slot_bytes(h, cl, mn) == M.slot_bytes(h, cl, mn)


def test_hashlocpair_and_sparse_chunk_layout():
    d = bytes(range(32))
    rec = M.hashlocpair_as_array(d, 0x0102030405060708, 4096, 8192)
    assert len(rec) == M.bal(32) == 56
    assert rec[:32] == d and rec[32:40] == bytes([1, 2, 3, 4, 5, 6, 7, 8])
    assert struct.unpack(">iiii", rec[40:]) == (4096, 8192, 0, 4096)
    img = M.sparse_data_chunk_bytes([(d, 7, 100, 4096, True), (d, 7, 4096, 0, False)])
    assert img[0] == 0 and struct.unpack(">II", img[1:9]) == (13 + 112, 2)
    assert struct.unpack(">i", img[9 + 44:9 + 48])[0] == 0  # first record is pos 0 (TreeMap order)
    assert struct.unpack(">I", img[-4:])[0] == 100  # doop: bytes of duplicate chunks
    with pytest.raises(IOError):
        M.hashlocpair_as_array(d, 0, -1, 0)


def _host_images(counts, st, ln, dg, dup, loc, hash_len):
    out, r = [], 0
    for b in range(len(counts)):
        pairs = []
        for i in range(int(counts[b])):
            pairs.append((bytes(dg[b, i, :hash_len]), int(loc[r]), int(ln[b, i]), int(st[b, i]), bool(dup[r])))
            r += 1
        out.append(M.sparse_data_chunk_bytes(pairs))
    return out


def _run(engine, nbuf, hash_len, slot_len=None, holes=True):
    import torch

    from sdfs_amd.device import DeviceBatch
    from sdfs_amd.index import HipHashesMap
    from sdfs_amd.meta import emit_map_slots

    batch = DeviceBatch(engine, nbuf=nbuf, buf_len=262144)
    batch.fill_streams(first_stream=77, bufs_per_stream=8)
    v = batch.data.view(nbuf, 262144)
    if holes:
        v[1, 20000:120000] = 0  # zero chunks repeat inside the buffer (claims > 1)
    for b in range(nbuf // 2, nbuf):
        v[b].copy_(v[b - nbuf // 2])
    batch.run(buffer_id_base=0)
    recs = batch.record_table()
    ix = HipHashesMap(1 << 16)
    dup, loc, new, nc = ix.put_records(recs, batch.total, pos_base=1 << 33)
    m, doop, ovf = emit_map_slots(batch, dup, loc, hash_len=hash_len, slot_len=slot_len)
    torch.cuda.synchronize()
    counts, st, ln, dg, total = batch.host_results()
    res = (m.cpu().numpy(), doop.cpu().numpy(), int(ovf.item()), counts, st, ln, dg,
           dup.cpu().numpy()[:total], loc.cpu().numpy()[:total])
    ix.destroy()
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["sha256", "md5"])
def test_gpu_map_images_vs_restatement(algo):
    from sdfs_amd import HipVariableMD5HashEngine, HipVariableSha256HashEngine
    e = HipVariableMD5HashEngine() if algo == "md5" else HipVariableSha256HashEngine()
    hl = 16 if algo == "md5" else 32
    nbuf = 32
    m, doop, ovf, counts, st, ln, dg, dup, loc = _run(e, nbuf, hl)
    assert ovf == 0
    sb = M.slot_bytes(hl, 262144, 4095)
    want = _host_images(counts, st, ln, dg, dup, loc, hl)
    for b in range(nbuf):
        img = m[b * sb:(b + 1) * sb]
        assert img[:len(want[b])].tobytes() == want[b], b
        assert not img[len(want[b]):].any()  # the rest of the slot is untouched (zero here)
        assert doop[b] == struct.unpack(">I", want[b][-4:])[0]
    # copied buffers are all duplicates: doop = the whole buffer
    assert (doop[nbuf // 2:] == 262144).all()
    e.destroy()


@pytest.mark.gpu
def test_gpu_map_overflow_flagged():
    from sdfs_amd import HipVariableSha256HashEngine
    e = HipVariableSha256HashEngine()
    m, doop, ovf, counts, *_ = _run(e, 8, 32, slot_len=13 + 56 * 8, holes=False)  # room for 8 records only
    assert ovf == 1 and (counts > 8).any()
    e.destroy()
