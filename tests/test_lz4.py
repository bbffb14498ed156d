"""LZ4 compression of unique chunks (include/sdfs_lz4.h).

CPU: the oracle restatement (oracle/lz4_ref.c) is pinned byte for byte against the image's
liblz4 1.9.x in its V19 mode; both modes (R123 = lz4-java 1.3.0's bundled r123, the reference;
V19) decode back to the input with the oracle's decoder and with liblz4; the committed fixtures
(tests/golden/lz4.json) are reproduced; the putChunk framing (HashBlobArchive.java:1281-1289) is
[big-endian length][block]; the library fails loudly without a GPU.
GPU: the HIP compressor, through the C-ABI, against the oracle — single chunks, host batches of
mixed kinds and lengths (incl. the 64 KiB + 11 table switch), the golden fixtures, and the
device path fed by the dedup index's new-chunk list.
Parity status: V19 pinned (liblz4); R123 differs from V19 only in the two rules lz4_ref.c names
(where the match search stops; 4- vs 5-byte hash of 32-bit tables): those are unpinned."""
import ctypes
import hashlib

import numpy as np
import pytest

from oracle import cdc_oracle as C
from oracle import lz4_oracle as Z
from sdfs_amd import _lib
from tests import golden_util as G
from tests.golden.make_lz4_golden import make_input

LENS = [0, 1, 4, 11, 12, 13, 14, 15, 16, 17, 31, 64, 100, 1000, 4095, 4096, 4097, 8192, 32768, 65535, 65536,
        65546, 65547, 65548, 100000, 131072]


def _gen(kind, n, stream=1):
    if kind == "rand":
        return C.synth(1, stream, 0, n).tobytes()
    if kind == "zeros":
        return bytes(n)
    if kind == "text":
        return Z.text_like(1, stream, n).tobytes()
    if kind == "mixed":
        return Z.mixed(1, stream, n).tobytes()
    if kind == "ramp":
        return (np.arange(n) % 251).astype(np.uint8).tobytes()
    raise ValueError(kind)


KINDS = ["rand", "zeros", "text", "mixed", "ramp"]
needs_liblz4 = pytest.mark.skipif(Z.system_lz4() is None, reason="no system liblz4 to pin against")


@needs_liblz4
def test_liblz4_batch_baseline_matches_v19_and_round_trips():
    """The LZ4 bench's liblz4 CPU leg (oracle/lz4_sys.c) makes the V19 oracle's blocks and
    decodes them back."""
    parts = [_gen(k, n, stream=60 + i) for i, (k, n) in enumerate((k, n) for k in KINDS for n in (0, 13, 5000, 70000))]
    lens = np.array([len(p) for p in parts], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    base = np.frombuffer(b"".join(parts) + bytes(8), np.uint8)
    out, oo, ol, _ = Z.system_batch(False, base, offs, lens, lens + lens // 255 + 16, 4)
    for i, p in enumerate(parts):
        assert out[int(oo[i]): int(oo[i]) + int(ol[i])].tobytes() == Z.compress(p, Z.V19), i
    back, bo, bl, _ = Z.system_batch(True, out, oo, ol, lens, 4)
    assert (bl == lens).all()
    for i, p in enumerate(parts):
        assert back[int(bo[i]): int(bo[i]) + len(p)].tobytes() == p, i


@needs_liblz4
@pytest.mark.parametrize("kind", KINDS)
def test_oracle_v19_equals_system_liblz4(kind):
    for n in LENS:
        d = _gen(kind, n)
        assert Z.compress(d, Z.V19) == Z.system_compress(d), (kind, n)


@needs_liblz4
@pytest.mark.parametrize("kind", KINDS)
def test_both_modes_decode_with_both_decoders(kind):
    for n in LENS:
        d = _gen(kind, n, stream=7)
        for mode in (Z.R123, Z.V19):
            blk = Z.compress(d, mode)
            assert len(blk) <= Z.bound(n)
            assert Z.decompress(blk, n) == d and Z.system_decompress(blk, n) == d, (kind, n, mode)


def test_oracle_reproduces_lz4_golden_fixtures():
    fx = G.load("lz4.json")["fixtures"]
    assert len(fx) >= 100
    for f in fx:
        d = make_input(f["input"])
        assert hashlib.sha256(d).hexdigest() == f["input_sha256"]
        for name, mode in Z.MODES.items():
            blk = Z.compress(d, mode)
            assert len(blk) == f[name]["len"] and hashlib.sha256(blk).hexdigest() == f[name]["sha256"], (f, name)


def test_putchunk_framing_and_known_blocks():
    # HashBlobArchive.putChunk: bf.putInt(nz = chunk.length) (big-endian) then the block
    d = b"abcabcabcabcabcabcabcabcabcabcabcabc"
    fr = Z.compress_framed(d)
    assert fr[:4] == len(d).to_bytes(4, "big") and fr[4:] == Z.compress(d)
    # LZ4 block of an empty input is one zero token; of < 13 bytes, literals only
    assert Z.compress(b"") == b"\x00"
    assert Z.compress(b"hello") == b"\x50hello"


def test_lz4_fails_loudly_without_gpu():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    h = ctypes.c_void_p()
    assert _lib.load().sdfs_cdc_lz4_create(0, 0, ctypes.byref(h)) == _lib.ENODEV and not h.value
    assert _lib.load().sdfs_cdc_lz4_create(0, 7, ctypes.byref(h)) == _lib.EINVAL
    assert _lib.load().sdfs_cdc_lz4_bound(65536) == 65536 + 257 + 16
    from sdfs_amd.lz4 import HipLz4Compressor
    with pytest.raises(_lib.SdfsCdcError):
        HipLz4Compressor()


# ------------------------------------------------------------------------------------------
# GPU
# ------------------------------------------------------------------------------------------
_COMP = {}


def comp(mode):
    from sdfs_amd.lz4 import HipLz4Compressor
    if mode not in _COMP:
        _COMP[mode] = HipLz4Compressor(mode)
    return _COMP[mode]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [Z.R123, Z.V19], ids=["r123", "v19"])
def test_gpu_single_chunks_vs_oracle(mode):
    c = comp(mode)
    for kind in KINDS:
        for n in LENS:
            d = _gen(kind, n, stream=3)
            assert c.compress(d) == Z.compress(d, mode), (kind, n)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [Z.R123, Z.V19], ids=["r123", "v19"])
def test_gpu_batch_mixed_chunks_vs_oracle(mode):
    rng = np.random.default_rng(4 + mode)
    parts, lens = [], []
    for i in range(300):
        kind = KINDS[i % len(KINDS)]
        n = int(rng.choice([0, 1, 13, 4096, 8000, 20000, 32768, 65546, 65547, 131072])) if i % 7 == 0 else \
            int(rng.integers(4096, 33000))
        parts.append(_gen(kind, n, stream=100 + i))
        lens.append(n)
    offs = np.concatenate([[0], np.cumsum([len(p) + 3 for p in parts[:-1]])]).astype(np.uint64)  # unaligned
    base = np.zeros(int(offs[-1]) + len(parts[-1]) + 8, np.uint8)
    for o, p in zip(offs, parts):
        base[int(o): int(o) + len(p)] = np.frombuffer(p, np.uint8)
    got = comp(mode).compress_chunks(base, offs, np.array(lens, np.uint32), framed=True)
    for i, p in enumerate(parts):
        assert got[i] == Z.compress_framed(p, mode), (i, lens[i])


@pytest.mark.gpu
def test_gpu_golden_fixtures():
    fx = G.load("lz4.json")["fixtures"]
    for name, mode in Z.MODES.items():
        datas = [make_input(f["input"]) for f in fx]
        offs = np.concatenate([[0], np.cumsum([len(d) for d in datas[:-1]])]).astype(np.uint64)
        base = np.frombuffer(b"".join(datas) + b"\0" * 8, np.uint8)
        got = comp(mode).compress_chunks(base, offs, np.array([len(d) for d in datas], np.uint32), framed=False)
        for f, blk in zip(fx, got):
            assert len(blk) == f[name]["len"] and hashlib.sha256(blk).hexdigest() == f[name]["sha256"], f["input"]


@pytest.mark.gpu
def test_gpu_device_path_new_chunks_from_the_index():
    """Write path on the device: getChunks batch (50 % duplicate buffers) -> dedup index ->
    extents of the NEW chunks -> LZ4 putChunk records; each record equals the oracle's."""
    torch = pytest.importorskip("torch")
    from sdfs_amd import HipVariableSha256HashEngine
    from sdfs_amd.device import DeviceBatch
    from sdfs_amd.index import HipHashesMap
    e = HipVariableSha256HashEngine()
    nbuf, L = 64, 262144
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=L)
    batch.fill_streams(first_stream=900, bufs_per_stream=16)
    v = batch.data.view(nbuf, L)
    v[3, 100000:180000] = 0  # a zero hole: compressible chunks
    for b in range(32, nbuf):
        v[b].copy_(v[b - 32])
    batch.run(buffer_id_base=5000)
    recs = batch.record_table()
    ix = HipHashesMap(1 << 16)
    dup, loc, new, nc = ix.put_records(recs, batch.total, pos_base=0)
    for mode in (Z.R123, Z.V19):
        c = comp(mode)
        src_off, src_len, dst_off, total = c.plan_records(recs, sel=new[: recs.shape[0]], count=nc.view(torch.int32),
                                                          buffer_id_base=5000, uniform_len=L)
        out = torch.zeros(int(total.item()) + 16, dtype=torch.uint8, device="cuda")
        dst_len = torch.zeros(src_len.shape[0], dtype=torch.int32, device="cuda")
        c.compress_device(batch.data, src_off, src_len, out, dst_off, dst_len, count=nc.view(torch.int32))
        torch.cuda.synchronize()
        k = int(nc.item())
        host = batch.data.cpu().numpy()
        so, sl, do, dl = (t.cpu().numpy()[:k] for t in (src_off, src_len, dst_off, dst_len))
        ob = out.cpu().numpy()
        distinct = {bytes(r[:32]) for r in recs.cpu().numpy()}
        assert k == len(distinct) <= int(recs.shape[0]) // 2  # buffers 32..63 repeat 0..31
        for i in range(k):
            chunk = host[int(so[i]): int(so[i]) + int(sl[i])].tobytes()
            rec = ob[int(do[i]): int(do[i]) + int(dl[i])].tobytes()
            assert rec == Z.compress_framed(chunk, mode), i
    ix.destroy()
    e.destroy()


@pytest.mark.gpu
def test_gpu_decompress_single_and_malformed():
    """Read side: the GPU decoder restores every oracle block (both modes, all kinds/lengths)."""
    c = comp(Z.R123)
    for kind in KINDS:
        for n in LENS:
            d = _gen(kind, n, stream=5)
            for mode in (Z.R123, Z.V19):
                assert c.decompress(Z.compress(d, mode), n) == d, (kind, n, mode)
    blk = bytearray(Z.compress(_gen("text", 5000, 9)))
    with pytest.raises(_lib.SdfsCdcError):
        c.decompress(bytes(blk), 4999)  # wrong length
    bad = bytearray(blk)
    bad[-3] = 0xF0  # a literal run past the end of the block
    with pytest.raises(_lib.SdfsCdcError):
        c.decompress(bytes(bad[:-1]), 5000)


@pytest.mark.gpu
def test_gpu_decompress_device_framed_records():
    """putChunk records ([BE32 nz][LZ4 block], or nz = -1 with the raw chunk) decoded on the device."""
    import struct

    import torch

    rng = np.random.default_rng(44)
    recs, datas = [], []
    for i in range(400):
        kind = KINDS[i % len(KINDS)]
        n = int(rng.integers(0, 40000))
        d = _gen(kind, n, stream=300 + i)
        datas.append(d)
        recs.append(struct.pack(">i", -1) + d if i % 11 == 0 else Z.compress_framed(d))
    # malformed records (decoded length -1): truncated block, nz larger than the block decodes
    # to, a match offset reaching before the output start, a literal run past the block end,
    # a zero offset, and a header-only record
    good = Z.compress(_gen("text", 3000, 17))
    bad = [struct.pack(">i", 3000) + good[:-7], struct.pack(">i", 3001) + good,
           struct.pack(">i", 24) + bytes([0x40]) + b"abcd" + bytes([0x10, 0x00]) + bytes([0x50]) + b"abcde",
           struct.pack(">i", 3000) + bytes([0xF0, 0x20]) + good[:30],
           struct.pack(">i", 12) + bytes([0x40]) + b"abcd" + bytes([0x00, 0x00]) + bytes([0x40]) + b"wxyz",
           b"\x00\x00"]
    nbad = len(bad)
    for i, r in enumerate(bad):
        recs.append(r)
        datas.append(None)
    src_off = np.concatenate([[0], np.cumsum([len(r) + 1 for r in recs[:-1]])]).astype(np.int64)
    base = np.zeros(int(src_off[-1]) + len(recs[-1]) + 16, np.uint8)
    for o, r in zip(src_off, recs):
        base[int(o): int(o) + len(r)] = np.frombuffer(r, np.uint8)
    caps = np.array([len(d) if d is not None else 4000 for d in datas], np.int32)
    dst_off = np.concatenate([[3], 3 + np.cumsum(caps[:-1].astype(np.int64) + 5)]).astype(np.int64)
    dev = torch.device("cuda:0")
    t = lambda a, dt: torch.from_numpy(np.ascontiguousarray(a)).to(dev, dt)  # noqa: E731
    out = torch.zeros(int(dst_off[-1] + caps[-1] + 16), dtype=torch.uint8, device=dev)
    dl = torch.zeros(len(recs), dtype=torch.int32, device=dev)
    comp(Z.R123).decompress_device(t(base, torch.uint8), t(src_off, torch.int64),
                                   t([len(r) for r in recs], torch.int32), out, t(dst_off, torch.int64),
                                   t(caps, torch.int32), dl, framed=True)
    torch.cuda.synchronize()
    o, dln = out.cpu().numpy(), dl.cpu().numpy()
    for i, d in enumerate(datas):
        if d is None:
            assert dln[i] == -1, i
        else:
            assert dln[i] == len(d) and o[dst_off[i]: dst_off[i] + len(d)].tobytes() == d, i
    assert nbad == 6


@pytest.mark.gpu
def test_gpu_hybrid_batch_with_records_over_128k_vs_oracle():
    """A hybrid-size batch (>= 192 chunks per CU, so lanes compress the compressible chunks) that
    also holds compressible records of 128 KiB + 1 .. 1 MiB: a lane's table entry keeps positions
    in 17 bits, so those must go to the wave kernel; every record equals the oracle's."""
    torch = pytest.importorskip("torch")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    n_small = 192 * ncu + 64
    rng = np.random.default_rng(128)
    src = Z.text_like(1, 91, 8 << 20)
    longs = [131072, 131073, 200000, 262144, 524288 + 17, 1 << 20]
    lens = [int(x) for x in rng.integers(600, 2600, n_small)]
    where = sorted(int(x) for x in rng.choice(n_small, len(longs), replace=False))
    for w, n in zip(where, longs):
        lens[w] = n
    lens = np.array(lens, np.uint32)
    # text windows (compressible: the lane path takes them unless they are too long); one long
    # record is mostly zeros (long match runs)
    starts = rng.integers(0, len(src) - (1 << 20) - 1, len(lens))
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 5)]).astype(np.uint64)
    base = np.zeros(int(offs[-1]) + int(lens[-1]) + 16, np.uint8)
    for i, (o, n) in enumerate(zip(offs, lens)):
        base[int(o): int(o) + int(n)] = src[int(starts[i]): int(starts[i]) + int(n)]
    zo = int(offs[where[3]])
    base[zo + 1000: zo + 250000] = 0
    for mode in (Z.R123, Z.V19):
        got = comp(mode).compress_chunks(base, offs, lens, framed=True)
        want, _ = Z.compress_batch(base, offs, lens, mode, 16)
        for i in where:
            assert got[i] == want[i], (mode, int(lens[i]))
        bad = [i for i in range(len(lens)) if got[i] != want[i]]
        assert not bad, (mode, len(bad), bad[:8])


@pytest.mark.gpu
def test_gpu_large_batch_hybrid_vs_oracle():
    """A batch large enough for the product library's hybrid (one lane per chunk, bailed
    incompressible chunks re-run one wave each: >= 192 chunks per CU): every record of a
    half-random, half-text 512 MiB batch equals the oracle's, in both modes, and decodes back."""
    torch = pytest.importorskip("torch")
    from sdfs_amd import HipVariableSha256HashEngine
    from sdfs_amd.device import DeviceBatch
    e = HipVariableSha256HashEngine()
    nbuf, L = 2048, 262144
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=L)
    batch.fill_streams(first_stream=700, bufs_per_stream=64)
    v = batch.data.view(nbuf, L)
    src = Z.text_like(1, 77, 4 << 20)
    txt = np.stack([src[(b * 12347) % (len(src) - L):][:L] for b in range(nbuf // 2)])
    v[1::2].copy_(torch.from_numpy(txt).to(v.device))
    v[6, 1000:90000] = 0  # long zero runs: 255-runs in the match lengths
    batch.run()
    recs = batch.record_table()
    n = int(recs.shape[0])
    assert n >= 192 * torch.cuda.get_device_properties(0).multi_processor_count
    host = batch.data.cpu().numpy()
    for mode in (Z.R123, Z.V19):
        c = comp(mode)
        src_off, src_len, dst_off, total = c.plan_records(recs, uniform_len=L)
        out = torch.zeros(int(total.item()) + 16, dtype=torch.uint8, device="cuda")
        dst_len = torch.zeros(n, dtype=torch.int32, device="cuda")
        c.compress_device(batch.data, src_off, src_len, out, dst_off, dst_len)
        torch.cuda.synchronize()
        so, sl, do, dl = (t.cpu().numpy() for t in (src_off, src_len, dst_off, dst_len))
        ob = out.cpu().numpy()
        want, _ = Z.compress_batch(host, so, sl, mode, 16)
        bad = [i for i in range(n) if ob[int(do[i]): int(do[i]) + int(dl[i])].tobytes() != want[i]]
        assert not bad, (len(bad), bad[:8])
        # the same compressor from two streams at once (its lane tables and bail list are shared:
        # the second launch must wait for the first): both outputs equal the checked one
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        outs = [torch.zeros_like(out) for _ in range(2)]
        lens2 = [torch.zeros_like(dst_len) for _ in range(2)]
        torch.cuda.synchronize()
        for st_, o_, l_ in zip((s1, s2), outs, lens2):
            with torch.cuda.stream(st_):
                c.compress_device(batch.data, src_off, src_len, o_, dst_off, l_, stream=st_.cuda_stream)
        torch.cuda.synchronize()
        for o_, l_ in zip(outs, lens2):
            assert torch.equal(l_, dst_len) and torch.equal(o_, out)
        # read side at the same size (the split decode: lanes for compressible records, waves
        # for the rest): every record back to its chunk
        back = torch.zeros_like(batch.data)
        blen = torch.zeros(n, dtype=torch.int32, device="cuda")
        c.decompress_device(out, dst_off, dst_len, back, src_off, src_len, blen)
        torch.cuda.synchronize()
        assert torch.equal(blen, src_len) and torch.equal(back, batch.data)
    e.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", [Z.R123, Z.V19], ids=["r123", "v19"])
def test_gpu_literal_screen_edges_vs_oracle(mode):
    """The literal screen (lz4_kernels.hip: a chunk whose words at position 0 and at every search
    probe are pairwise distinct is one literal run) against the oracle's parse on its edges: random
    chunks (screened), random chunks with one 4-byte word planted again at a probe position or at a
    position the search skips (a repeat the screen must send to the exact kernels, or need not),
    a repeat of position 0's word, zero words (the set's empty mark), chunks right at the search's
    end (13 .. 16 bytes) and long ones (u32 tables, more probes than the LDS set holds)."""
    rng = np.random.default_rng(55 + mode)
    parts = []
    for i in range(400):
        n = int(rng.choice([13, 14, 15, 16, 17, 64, 100, 4096, 8192, 20000, 32768, 65547, 131072]))
        d = bytearray(C.synth(9, 2000 + i, 0, n).tobytes())
        kind = i % 5
        if kind == 1 and n > 40:  # a word planted again further on (at a probe or a skipped position)
            a = int(rng.integers(0, n // 2))
            b = int(rng.integers(a + 4, n - 4))
            d[b:b + 4] = d[a:a + 4]
        elif kind == 2 and n > 40:  # position 0's word again
            b = int(rng.integers(1, n - 4))
            d[b:b + 4] = d[0:4]
        elif kind == 3 and n > 40:  # a zero word, or two
            for _ in range(int(rng.integers(1, 3))):
                b = int(rng.integers(0, n - 4))
                d[b:b + 4] = b"\0\0\0\0"
        parts.append(bytes(d))
    lens = np.array([len(p) for p in parts], np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 1)]).astype(np.uint64)
    base = np.zeros(int(offs[-1]) + int(lens[-1]) + 8, np.uint8)
    for o, p in zip(offs, parts):
        base[int(o): int(o) + len(p)] = np.frombuffer(p, np.uint8)
    got = comp(mode).compress_chunks(base, offs, lens, framed=True)
    for i, p in enumerate(parts):
        assert got[i] == Z.compress_framed(p, mode), (i, len(p), i % 5)
