"""GPU parity tests: the MI355X kernels, called through the C-ABI, against the CPU oracle and the
committed golden fixtures.  Bar: bit-exact chunk starts, lengths and digests (integer work).

Boundary parity is against the oracle restatement (the Java engine's jar is absent: parity vs the
Java reference UNPINNED for the A.3 knobs); digests are additionally pinned by FIPS/RFC vectors.
At BASELINE.json's full size (64 x 64 MiB, 4 GiB) the tests check size-independent properties
(exact cover, min/max bounds, record table == slots, duplicate buffers -> identical lists) plus a
random sample of buffers against the oracle."""
import hashlib
import threading

import numpy as np
import pytest

from oracle import cdc_oracle as O
from tests import golden_util as G

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from sdfs_amd import HipVariableMD5HashEngine, HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd import _lib  # noqa: E402
from sdfs_amd.device import SYNTH_SEED, DeviceBatch  # noqa: E402

_ENGINES = {}


def engine_for(prm: dict):
    key = tuple(sorted(prm.items()))
    if key not in _ENGINES:
        cfg = SdfsConfig(min_len=prm["min_len"], max_len=prm["max_len"], window=prm["window"], poly=prm["poly"],
                         pred_mask=prm["pred_mask"], pred_value=prm["pred_value"], min_cmp=prm["min_cmp"],
                         pred_kind=prm.get("pred_kind", 0), pred_div=prm.get("pred_div", 0),
                         pred_rem=prm.get("pred_rem", 0))
        algo = prm["hash_algo"]
        if algo == O.MD5:
            e = HipVariableMD5HashEngine(cfg)
        else:
            e = HipVariableSha256HashEngine(
                HipVariableSha256HashEngine.HASH160 if algo == O.SHA256_160 else HipVariableSha256HashEngine.HASH256,
                cfg)
        _ENGINES[key] = e
    return _ENGINES[key]


DEFAULT = dict(poly=O.POLY, window=48, min_len=4095, max_len=32768, min_cmp=O.MIN_GT, pred_mask=0xFFF, pred_value=0,
               hash_algo=O.SHA256)


def P(**kw):
    d = dict(DEFAULT)
    d.update(kw)
    return d


def assert_same(got, exp, what=""):
    st, ln, dg = got
    es, el, ed = exp
    assert st.tolist() == list(es), what
    assert ln.tolist() == list(el), what
    assert [bytes(d) for d in dg] == [bytes(d) for d in ed], what


# ---------------------------------------------------------------- getHash
def test_get_hash_known_answers():
    kat = G.load("kat.json")
    e = engine_for(P())
    for msg, h in kat["sha256"]:
        assert e.getHash(msg.encode()).hex() == h
    assert e.getHash(b"a" * 1000000).hex() == kat["sha256_million_a"]
    m = engine_for(P(hash_algo=O.MD5))
    for msg, h in kat["md5"]:
        assert m.getHash(msg.encode()).hex() == h
    assert engine_for(P(hash_algo=O.SHA256_160)).getHash(b"abc").hex() == kat["sha256"][1][1][:40]


def test_get_hash_blank_chunks_and_lengths():
    kat = G.load("kat.json")["blank"]
    e = engine_for(P())
    assert e.getHash(bytes(4096)).hex() == kat["sha256_zero_4096"]  # WritableCacheBuffer.bk
    assert e.getHash(bytes(262144)).hex() == kat["sha256_zero_262144"]  # HashStore.blankHash
    for n in [1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 129, 1000, 4097]:
        d = O.synth(3, 77, 5, n).tobytes()
        assert e.getHash(d) == hashlib.sha256(d).digest(), n


# ---------------------------------------------------------------- golden fixtures
@pytest.mark.parametrize("fx", G.fixtures(), ids=lambda f: f["name"])
def test_golden_fixture_bit_exact(fx):
    data = G.fixture_input(fx)
    e = engine_for(fx["params"])
    got = e.chunk_arrays(data)
    exp = (fx["starts"], fx["lens"], [bytes.fromhex(h) for h in fx["digests"]])
    assert_same(got, exp, fx["name"])


@pytest.mark.parametrize("window", [16, 32, 48, 64])
def test_every_window_through_the_small_pass_scan(window):
    """Every supported window through the queue's lone-pass scan (64-byte segments, ScanTiny) and a
    ragged small batch, random and zero-run buffers, against the oracle."""
    prm = P(window=window)
    e = engine_for(prm)
    rng = np.random.default_rng(window)
    bufs = [O.synth(SYNTH_SEED, 60 + window, 0, 262144), rng.integers(0, 256, 200003, dtype=np.uint8)]
    bufs[1][5000:9000] = 0
    bufs[1][150000:151000] = 0
    for buf in bufs:
        assert_same(e.chunk_arrays(buf.tobytes()), O.chunk(buf.tobytes(), O.Params(**prm)), (window, len(buf)))
    lens = np.array([len(b) for b in bufs] + [0, 777], dtype=np.uint32)
    base = np.concatenate(bufs + [rng.integers(0, 256, 777, dtype=np.uint8)])
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    counts, st, ln, dg = e.chunk_batch(base, offs, lens)
    for b in range(len(lens)):
        buf = base[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
        exp = O.chunk(buf, O.Params(**prm)) if lens[b] else ([], [], [])
        assert_same((st[b, :counts[b]], ln[b, :counts[b]], dg[b, :counts[b]]), exp, (window, b))


def test_get_chunks_fingers():
    data = O.synth(SYNTH_SEED, 0, 0, 262144).tobytes()
    fingers = engine_for(P()).getChunks(data, "uuid-1")
    st, ln, dg = O.chunk(data)
    assert [f.start for f in fingers] == st.tolist() and [f.len for f in fingers] == ln.tolist()
    for f, d in zip(fingers, dg):
        assert f.chunk == data[f.start: f.start + f.len] and f.hash == d.tobytes() and f.uuid == "uuid-1"


@pytest.mark.parametrize("n", [0, 1, 47, 48, 49, 63, 64, 65, 127, 4095, 4096, 4097, 8191, 8192, 32767, 32768, 32769,
                               65536 + 5, 262143, 262144])
def test_edge_lengths(n):
    data = O.synth(SYNTH_SEED, 21, 3, n).tobytes()
    for prm in (P(), P(min_len=0, max_len=100, pred_mask=0xF)):
        got = engine_for(prm).chunk_arrays(data)
        exp = O.chunk(data, O.Params(**prm)) if n else ([], [], [])
        assert_same(got, exp, (n, prm["min_len"]))


def test_ragged_batch_vs_oracle():
    rng = np.random.default_rng(5)
    lens = rng.integers(1, 300000, 40).astype(np.uint32)
    lens[3] = 0
    lens[7] = 64
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 13)]).astype(np.uint64)  # unaligned
    base = O.synth(SYNTH_SEED, 30, 0, int(offs[-1] + lens[-1]))
    for prm in (P(), P(hash_algo=O.MD5), P(min_len=511, max_len=4096, pred_mask=0x1FF)):
        counts, st, ln, dg = engine_for(prm).chunk_batch(base, offs, lens)
        for b in range(len(lens)):
            buf = base[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
            exp = O.chunk(buf, O.Params(**prm)) if lens[b] else ([], [], [])
            c = counts[b]
            assert_same((st[b, :c], ln[b, :c], dg[b, :c]), exp, (b, prm))


def test_small_batch_walk_routes_at_the_lds_limit():
    """Small batches resolve their cuts from LDS (cdc_resolve_small_kernel: a buffer's whole bitmap,
    up to 512 KiB = 16 Ki words); a batch whose longest buffer is past that takes the global walk.
    Both sides of the limit, ragged (empty, 64 B, exactly 512 KiB, one byte over) and uniform
    device-resident 512 KiB buffers, single queue calls of exactly 512 KiB, all vs the oracle."""
    lim = 32 * 16384
    for lens in ([lim, 0, 64, 300001, lim - 1, 4096], [lim + 1, 0, 64, lim, 77777]):
        lens = np.array(lens, dtype=np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
        base = O.synth(SYNTH_SEED, 44, 0, int(offs[-1] + lens[-1]))
        for prm in (P(), P(min_len=2047, pred_mask=0x7FF)):
            counts, st, ln, dg = engine_for(prm).chunk_batch(base, offs, lens)
            for b in range(len(lens)):
                buf = base[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
                exp = O.chunk(buf, O.Params(**prm)) if lens[b] else ([], [], [])
                assert_same((st[b, :counts[b]], ln[b, :counts[b]], dg[b, :counts[b]]), exp, (b, int(lens[b])))
    e = engine_for(P(min_len=2047, pred_mask=0x7FF))
    one = O.synth(SYNTH_SEED, 45, 0, lim).tobytes()
    assert_same(e.chunk_arrays(one), O.chunk(one, O.Params(**P(min_len=2047, pred_mask=0x7FF))), "queue call")
    batch = DeviceBatch(e, nbuf=6, buf_len=lim)
    batch.fill_streams(first_stream=46, bufs_per_stream=2)
    batch.run()
    counts, st, ln, dg, _ = batch.host_results()
    _check_batch_against_oracle(batch, counts, st, ln, dg, P(min_len=2047, pred_mask=0x7FF), 2, 46, None)


def test_small_batch_walk_list_and_ballot_forms():
    """cdc_resolve_small_kernel walks a buffer's cuts through its LDS candidate list (successor
    pointers) while the buffer holds at most 2048 candidates, and by 64-word ballots past that.
    Ragged batches and single queue calls on both sides: random data, zero runs just under and
    over the list's capacity, runs straddling forced (maxLen) cuts, all-zero and candidate-free
    buffers, each vs the oracle."""
    rng = np.random.default_rng(5150)
    L = 262144
    bufs = []
    for run in (0, 1500, 2040, 2100, 6000, L):
        h = rng.integers(0, 256, L, dtype=np.uint8)
        o = int(rng.integers(0, L - run)) if run < L else 0
        h[o:o + run] = 0
        bufs.append(h)
    h = rng.integers(0, 256, L, dtype=np.uint8)
    h[70000:140000] = 0x55  # a candidate-free stretch: forced cuts, then the chain resumes
    h[140000:141900] = 0
    bufs.append(h)
    bufs.append(np.full(L - 333, 0xFF, np.uint8))  # no candidate at all
    lens = np.array([len(b) for b in bufs], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    base = np.concatenate(bufs)
    for prm in (P(), P(min_len=2047, pred_mask=0x7FF), P(min_len=0, pred_mask=0x3FF)):
        e = engine_for(prm)
        counts, st, ln, dg = e.chunk_batch(base, offs, lens)
        for b, buf in enumerate(bufs):
            exp = O.chunk(buf.tobytes(), O.Params(**prm))
            assert_same((st[b, :counts[b]], ln[b, :counts[b]], dg[b, :counts[b]]), exp, (b, prm))
        for b in (2, 3, 6):
            assert_same(e.chunk_arrays(bufs[b].tobytes()), O.chunk(bufs[b].tobytes(), O.Params(**prm)), ("queue", b))


@pytest.mark.parametrize("buf_len", [4096, 8192, 16384])
@pytest.mark.parametrize("mix", [(4095, 0xFFF), (2047, 0x7FF)], ids=["default", "mix4k"])
def test_uniform_small_buffers_every_segment_route(buf_len, mix):
    """Uniform batches of 4, 8 and 16 KiB buffers: a wave's 64 segments are one buffer when the
    segment is buf_len / 64 (64, 128 or 256 bytes), which only the 256-byte segment may take as
    the scan's fused walk (whole ScanProd blocks); 64/128-byte segments take ScanTiny + the walk.
    Small (lone-pass) and 16 MiB device batches, a uniform host batch and concurrent single calls
    of one buffer each, all vs the oracle."""
    prm = P(min_len=mix[0], pred_mask=mix[1])
    e = engine_for(prm)
    for nbuf in (64, (16 << 20) // buf_len):
        bps = 16
        batch = DeviceBatch(e, nbuf=nbuf, buf_len=buf_len)
        batch.fill_streams(first_stream=70, bufs_per_stream=bps)
        batch.run()
        counts, st, ln, dg, total = batch.host_results()
        assert total == counts.sum()
        sample = None if nbuf <= 64 else sorted(set(np.random.default_rng(buf_len).integers(0, nbuf, 48).tolist()))
        _check_batch_against_oracle(batch, counts, st, ln, dg, prm, bps, 70, sample)
    n = 96
    base = O.synth(SYNTH_SEED, 71, 0, n * buf_len)
    offs = np.arange(n, dtype=np.uint64) * buf_len
    lens = np.full(n, buf_len, np.uint32)
    counts, st, ln, dg = e.chunk_batch(base, offs, lens)
    exp = [O.chunk(base[b * buf_len:(b + 1) * buf_len].tobytes(), O.Params(**prm)) for b in range(n)]
    for b in range(n):
        assert_same((st[b, :counts[b]], ln[b, :counts[b]], dg[b, :counts[b]]), exp[b], b)
    errors = []

    def work(t):
        try:
            for k in range(4):
                b = (t * 4 + k) % n
                assert_same(e.chunk_arrays(base[b * buf_len:(b + 1) * buf_len].tobytes()), exp[b], b)
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    th = [threading.Thread(target=work, args=(t,)) for t in range(16)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


def test_concurrent_callers_share_one_engine():
    """SparseDedupFile.eng is one static engine used by every flush thread (SparseDedupFile.java:100)."""
    e = engine_for(P())
    bufs = [O.synth(SYNTH_SEED, 40 + i, 0, 262144).tobytes() for i in range(8)]
    exp = [O.chunk(b) for b in bufs]
    errors = []

    def work(i):
        try:
            for _ in range(3):
                assert_same(e.chunk_arrays(bufs[i]), exp[i], i)
        except Exception as ex:  # pragma: no cover
            errors.append(ex)

    th = [threading.Thread(target=work, args=(i,)) for i in range(8)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors


# ---------------------------------------------------------------- device-resident batches
def _check_batch_against_oracle(batch, counts, st, ln, dg, prm, bufs_per_stream, first_stream, sample):
    host = batch.data.cpu().numpy() if sample is None else None
    idx = range(batch.nbuf) if sample is None else sample
    dl = O.Params(**prm).digest_len
    for b in idx:
        stream = first_stream + b // bufs_per_stream
        off = (b % bufs_per_stream) * batch.buf_len
        buf = O.synth(SYNTH_SEED, stream, off, batch.buf_len)
        if host is not None:
            assert (host[b * batch.buf_len:(b + 1) * batch.buf_len] == buf).all()
        es, el, ed = O.chunk(buf, O.Params(**prm))
        c = counts[b]
        assert st[b, :c].tolist() == es.tolist() and ln[b, :c].tolist() == el.tolist(), b
        assert (dg[b, :c, :dl] == ed).all(), b


def _check_cover(counts, st, ln, buf_len, prm):
    cap = st.shape[1]
    k = np.arange(cap)[None, :]
    valid = k < counts[:, None]
    assert (counts > 0).all()
    assert (st[:, 0] == 0).all()
    nxt = np.where(k[:, :-1] + 1 < counts[:, None], st[:, 1:], 0)
    ends = st[:, :-1].astype(np.int64) + ln[:, :-1]
    inner = (k[:, :-1] + 1) < counts[:, None]
    assert (np.where(inner, ends == nxt, True)).all()
    last = counts - 1
    r = np.arange(len(counts))
    assert (st[r, last].astype(np.int64) + ln[r, last] == buf_len).all()
    assert (np.where(valid, ln <= prm["max_len"], True)).all()
    assert (np.where(inner, ln[:, :-1] > prm["min_len"], True)).all()


def test_device_b1_sample_full_compare():
    """256 write buffers (1 GiB/4 of configs[1]) on the device path, every buffer vs the oracle."""
    prm = P()
    e = engine_for(prm)
    batch = DeviceBatch(e, nbuf=256, buf_len=262144)
    batch.fill_streams(first_stream=0, bufs_per_stream=64)
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == counts.sum()
    _check_batch_against_oracle(batch, counts, st, ln, dg, prm, 64, 0, None)


def _dense_candidate_buffers(nbuf: int, buf_len: int) -> np.ndarray:
    """Random buffers with zero runs: an all-zero window fingerprints to 0, so every position in
    a run is a candidate and the 4 KiB scan segments it covers hold far more than the 8
    candidates a lane keeps in registers (the fused resolve then reads the bitmap blocks stored
    from the overflow on).  Runs start mid-segment, cross segment boundaries, cover whole
    buffers, and sit inside and beyond the minLen/maxLen windows."""
    rng = np.random.default_rng(20261016)
    host = rng.integers(0, 256, nbuf * buf_len, dtype=np.uint8).reshape(nbuf, buf_len)
    for b in range(nbuf):
        kind = b % 4
        if kind == 0:
            host[b] = 0
        elif kind == 1:
            for _ in range(12):
                o = int(rng.integers(0, buf_len - 4096))
                host[b, o:o + int(rng.integers(60, 4000))] = 0
        elif kind == 2:
            o = int(rng.integers(0, 64)) * 4096 + int(rng.integers(1000, 3000))
            host[b, o:o + int(rng.integers(20000, 70000))] = 0
        else:
            host[b, : int(rng.integers(4000, 9000))] = 0  # dense from the buffer start
            o = buf_len - int(rng.integers(100, 5000))
            host[b, o:] = 0  # and up to the end
    return host


def test_device_dense_candidates_segment_overflow():
    """Uniform 256 KiB batch (fused resolve) where many segments overflow the register summary."""
    prm = P()
    e = engine_for(prm)
    nbuf, buf_len = 64, 262144
    host = _dense_candidate_buffers(nbuf, buf_len)
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=buf_len)
    batch.data.copy_(torch.from_numpy(host.reshape(-1)))
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == counts.sum()
    dl = O.Params(**prm).digest_len
    for b in range(nbuf):
        es, el, ed = O.chunk(host[b].tobytes(), O.Params(**prm))
        c = counts[b]
        assert st[b, :c].tolist() == es.tolist() and ln[b, :c].tolist() == el.tolist(), b
        assert (dg[b, :c, :dl] == ed).all(), b


def test_device_b1_full_size_properties():
    """BASELINE configs[1] at full size: 64 streams x 64 MiB = 16384 buffers of 256 KiB."""
    prm = P()
    e = engine_for(prm)
    batch = DeviceBatch(e, nbuf=16384, buf_len=262144)
    batch.fill_streams(first_stream=0, bufs_per_stream=256)
    batch.run(buffer_id_base=1000)
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    _check_cover(counts, st, ln, 262144, prm)
    rng = np.random.default_rng(1)
    sample = sorted(set(rng.integers(0, 16384, 48).tolist()) | {0, 255, 256, 16383})
    _check_batch_against_oracle(batch, counts, st, ln, dg, prm, 256, 0, sample)
    # dense record table == per-buffer slots, in (buffer, chunk) order
    rec = batch.record_table().cpu().numpy()
    assert rec.shape[0] == total
    base = np.concatenate([[0], np.cumsum(counts.astype(np.int64))[:-1]]).astype(np.int64)
    for b in sample:
        for i in range(counts[b]):
            r = rec[base[b] + i]
            assert bytes(r[:32]) == bytes(dg[b, i])
            assert int.from_bytes(bytes(r[32:40]), "little") == 1000 + b
            assert int.from_bytes(bytes(r[40:44]), "little") == st[b, i]
            assert int.from_bytes(bytes(r[44:48]), "little") == ln[b, i]
    mean = 262144 * 16384 / total
    assert 7000 < mean < 9500, mean  # ~8.2 KiB for a 12-bit predicate, min 4095


def test_device_two_streams_in_flight_one_engine():
    """One engine, runs alternating between two streams (two batches in flight: the workspace
    ring lets one batch's scan overlap the other's fingerprinting).  Every run equals the
    single-stream result and the oracle."""
    prm = P()
    e = HipVariableSha256HashEngine()
    batches = [DeviceBatch(e, nbuf=300, buf_len=262144) for _ in range(2)]
    batches[0].fill_streams(first_stream=200, bufs_per_stream=100)
    batches[1].data = batches[0].data
    batches[0].run(buffer_id_base=7)
    ref = batches[0].host_results()
    ref_rec = batches[0].record_table().cpu().numpy()
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    for _ in range(3):
        for k in range(6):
            batches[k % 2].run(buffer_id_base=7, stream=streams[k % 2].cuda_stream)
    torch.cuda.synchronize()
    for bt in batches:
        got = bt.host_results()
        for x, y in zip(got[:4], ref[:4]):
            assert np.array_equal(x, y)
        assert got[4] == ref[4]
        assert np.array_equal(bt.record_table().cpu().numpy(), ref_rec)
    counts, st, ln, dg, total = ref
    _check_cover(counts, st, ln, 262144, prm)
    _check_batch_against_oracle(batches[0], counts, st, ln, dg, prm, 100, 200, [0, 1, 99, 100, 150, 299])
    e.destroy()


def test_device_4k_mean_mix_full_size():
    """The metric's 4 KiB-mean mix at BASELINE configs[1] size: min-variable-segment-size=2
    (minLen 2047, Config.java:145-148) and an 11-bit predicate; 4 GiB of 256 KiB buffers.  At
    ~2 candidates per 4 KiB scan segment a few hundred segments overflow the 8-entry register
    summary, so the fused walk's bitmap path runs at full size too."""
    prm = P(min_len=2047, pred_mask=0x7FF)
    e = engine_for(prm)
    batch = DeviceBatch(e, nbuf=16384, buf_len=262144)
    batch.fill_streams(first_stream=0, bufs_per_stream=256)
    batch.run(buffer_id_base=0)
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    _check_cover(counts, st, ln, 262144, prm)
    rng = np.random.default_rng(4)
    sample = sorted(set(rng.integers(0, 16384, 40).tolist()) | {0, 16383})
    _check_batch_against_oracle(batch, counts, st, ln, dg, prm, 256, 0, sample)
    mean = 262144 * 16384 / total
    assert 3800 < mean < 4300, mean  # 4 095 B expected (minus the buffer-end truncation)


@pytest.mark.parametrize("mask,min_len", [(0x7FF, 2047), (0x7FF, 1023)])
def test_device_dense_candidates_11bit(mask, min_len):
    """Zero runs (every position a candidate) under the 4 KiB-mean parameters: summary overflow
    mid-segment, across segments, whole buffers and both buffer ends."""
    prm = P(min_len=min_len, pred_mask=mask)
    e = engine_for(prm)
    nbuf, buf_len = 32, 262144
    host = _dense_candidate_buffers(nbuf, buf_len)
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=buf_len)
    batch.data.copy_(torch.from_numpy(host.reshape(-1)))
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    for b in range(nbuf):
        es, el, ed = O.chunk(host[b].tobytes(), O.Params(**prm))
        c = counts[b]
        assert st[b, :c].tolist() == es.tolist() and ln[b, :c].tolist() == el.tolist(), b
        assert (dg[b, :c] == ed).all(), b


def test_device_dedup_50pct_copies_are_identical():
    """configs[2] shape: half the buffers are byte copies of earlier fresh ones (dedup-hit path)."""
    e = engine_for(P())
    nbuf = 512
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=262144, records=False)
    batch.fill_streams(first_stream=100, bufs_per_stream=64)
    rng = np.random.default_rng(2)
    fresh = [0]
    src = {}
    v = batch.data.view(nbuf, 262144)
    for b in range(1, nbuf):
        if rng.random() < 0.5:
            fresh.append(b)
        else:
            s = int(rng.choice(fresh))
            v[b].copy_(v[s])
            src[b] = s
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    for b, s in src.items():
        c = counts[s]
        assert counts[b] == c and (st[b, :c] == st[s, :c]).all() and (dg[b, :c] == dg[s, :c]).all()
    _check_batch_against_oracle(batch, counts, st, ln, dg, P(), 64, 100, fresh[:16])


def test_backup_volume_profile_40mib_buffer():
    """BACKUP_VOLUME=true: CHUNK_LENGTH 40 MiB, maxLen 128 KiB (VolumeConfigWriter.java:298-307)."""
    prm = P(max_len=131072)
    cfg = SdfsConfig.backup_volume()
    e = HipVariableSha256HashEngine(config=cfg)
    assert e.getMaxLen() == 40960 * 1024
    buf = O.synth(SYNTH_SEED, 500, 0, 40960 * 1024)
    assert_same(e.chunk_arrays(buf), O.chunk(buf, O.Params(**prm)), "backup")
    e.destroy()


@pytest.mark.parametrize("prm", [P(max_len=131072), P(), P(max_len=131072, pred_mask=0xFFFFFF)],
                         ids=["backup", "default", "forced-cuts"])
def test_long_ragged_buffers_lds_walk(prm):
    """Buffers longer than one 256 Ki-position LDS window take the LDS-staged cut walk; lengths
    are unaligned so windows restage mid-buffer and the tail chunk ends inside a window."""
    lens = np.array([5 * 2**20 + 13, 300 * 1024 - 7, 2**20, 33, 2 * 2**20 + 1000], dtype=np.uint32)
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
    base = O.synth(SYNTH_SEED, 41, 0, int(offs[-1] + lens[-1]))
    counts, st, ln, dg = engine_for(prm).chunk_batch(base, offs, lens)
    for b in range(len(lens)):
        buf = base[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
        exp = O.chunk(buf, O.Params(**prm))
        c = counts[b]
        assert_same((st[b, :c], ln[b, :c], dg[b, :c]), exp, b)


def test_sectioned_walk_chains_that_never_meet():
    """All-zero data cuts at every min_len+1 bytes; with min_len+1 not dividing the 1 Mi-position
    section length the speculative chains never meet the true one, so the stitch pass walks every
    cut itself (slow path) and must still be exact."""
    prm = P(min_len=2999, max_len=131072)
    lens = np.array([6 * 2**20 + 5, 4 * 2**20], dtype=np.uint32)
    offs = np.array([0, int(lens[0]) + 59], dtype=np.uint64)
    base = np.zeros(int(offs[-1] + lens[-1]), dtype=np.uint8)
    base[int(offs[1]) + 1_500_000:int(offs[1]) + 1_600_000] = 7  # a patch of other bytes
    counts, st, ln, dg = engine_for(prm).chunk_batch(base, offs, lens)
    for b in range(len(lens)):
        buf = base[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
        c = counts[b]
        assert_same((st[b, :c], ln[b, :c], dg[b, :c]), O.chunk(buf, O.Params(**prm)), b)


def test_device_backup_uniform_40mib_batch():
    """configs[4] shape on the device path: uniform 40 MiB buffers (LDS-staged cut walk)."""
    prm = P(max_len=131072)
    e = engine_for(prm)
    nbuf = 3
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=40960 * 1024, records=False)
    batch.fill_streams(first_stream=700, bufs_per_stream=1)
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    _check_batch_against_oracle(batch, counts, st, ln, dg, prm, 1, 700, [0, 1, 2])


def test_device_error_paths_raise():
    e = engine_for(P())
    batch = DeviceBatch(e, nbuf=2, buf_len=262144, records=False)
    bad = _lib.DevOut.from_buffer_copy(batch.out)
    bad.cap = 3
    with pytest.raises(_lib.SdfsCdcError):
        e.run_device(batch.data.data_ptr(), 2, 262144, bad)
    with pytest.raises(_lib.SdfsCdcError):
        e.run_device(batch.data.data_ptr() + 1, 2, 262144, batch.out)


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["sha256", "sha256_160", "md5"])
def test_get_hash_batch_and_device_extents(algo):
    """getHash in bulk (sdfs_cdc_get_hash_batch / sdfs_cdc_hash_device) == hashlib, order kept."""
    import hashlib

    import numpy as np
    import torch

    from sdfs_amd import HipVariableMD5HashEngine, HipVariableSha256HashEngine
    e = (HipVariableMD5HashEngine() if algo == "md5" else
         HipVariableSha256HashEngine(HipVariableSha256HashEngine.HASH160 if algo == "sha256_160"
                                     else HipVariableSha256HashEngine.HASH256))
    hf = (lambda b: hashlib.md5(b).digest()) if algo == "md5" else (lambda b: hashlib.sha256(b).digest())
    dl = 16 if algo == "md5" else (20 if algo == "sha256_160" else 32)
    rng = np.random.default_rng(31)
    lens = [int(x) for x in rng.integers(0, 40000, 500)] + [0, 1, 55, 56, 63, 64, 65, 119, 120, 131072, 300000]
    chunks = [O.synth(12, i, 0, n).tobytes() for i, n in enumerate(lens)]
    got = e.getHashes(chunks)
    assert [g for g in got] == [hf(c)[:dl] for c in chunks]
    # device form, unaligned offsets, device count
    offs = np.concatenate([[1], 1 + np.cumsum([len(c) + 3 for c in chunks[:-1]])]).astype(np.int64)
    base = np.zeros(int(offs[-1]) + len(chunks[-1]) + 8, np.uint8)
    for o, c in zip(offs, chunks):
        base[int(o): int(o) + len(c)] = np.frombuffer(c, np.uint8)
    dev = torch.device("cuda:0")
    d = torch.from_numpy(base).to(dev)
    dg = torch.zeros(len(chunks), 32, dtype=torch.uint8, device=dev)
    k = len(chunks) - 7
    e.hash_device(d, torch.from_numpy(offs).to(dev), torch.tensor(lens, dtype=torch.int32, device=dev), dg,
                  count=torch.tensor([k], dtype=torch.int32, device=dev))
    torch.cuda.synchronize()
    out = dg.cpu().numpy()
    for i in range(k):
        assert out[i, :dl].tobytes() == hf(chunks[i])[:dl], i
    assert not out[k:].any()
    e.destroy()


@pytest.mark.gpu
def test_pinned_host_batch_direct_copy_matches_pageable():
    """Pinned caller memory takes the no-staging H2D path; results equal the pageable path's."""
    import torch

    e = HipVariableSha256HashEngine()
    nb, L = 96, 262144
    data = np.concatenate([O.synth(SYNTH_SEED, 900 + i, 0, L) for i in range(nb)])
    pin = torch.empty(nb * L, dtype=torch.uint8, pin_memory=True)
    pin.copy_(torch.from_numpy(data))
    offs = np.arange(nb, dtype=np.uint64) * L
    for lens in (np.full(nb, L, np.uint32),  # back to back, 64-byte multiples: direct copy
                 np.array([L - (i % 7) * 13 for i in range(nb)], np.uint32)):  # ragged: staged
        a = e.chunk_batch(data, offs, lens)
        b = e.chunk_batch(pin.numpy(), offs, lens)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    # caller memory page-locked through the C-ABI (what a JNI shim does with its direct buffers)
    reg = np.array(data)  # a fresh, page-aligned-enough numpy buffer
    _lib.check(_lib.load().sdfs_cdc_host_register(reg.ctypes.data, reg.nbytes))
    try:
        c = e.chunk_batch(reg, offs, np.full(nb, L, np.uint32))
        a = e.chunk_batch(data, offs, np.full(nb, L, np.uint32))
        for x, y in zip(a, c):
            assert np.array_equal(x, y)
    finally:
        _lib.check(_lib.load().sdfs_cdc_host_unregister(reg.ctypes.data))
    e.destroy()


@pytest.mark.parametrize("algo", [O.SHA256, O.SHA256_160])
def test_small_batch_latency_form_equals_throughput_form(algo):
    """Batches too small to fill the GPU fingerprint with the two-wave latency kernel
    (chunk_hash_split_kernel: message schedule and rounds in separate waves); larger ones with
    the one-lane-per-chunk kernel.  The same buffers through both sizes give identical records,
    and the small batch equals the oracle, including maxLen chunks (long zero-free runs with no
    candidate) and dense-candidate buffers."""
    prm = P(hash_algo=algo)
    e = engine_for(prm)
    buf_len = 262144
    host = _dense_candidate_buffers(32, buf_len)
    host[7] = 0xFF  # no candidate anywhere: maxLen chunks
    host[9, 100000:200000] = 0x55  # a candidate-free stretch inside random data
    small = DeviceBatch(e, nbuf=32, buf_len=buf_len)  # 32 x cap tasks: latency form
    small.data.copy_(torch.from_numpy(host.reshape(-1)))
    small.run()
    big = DeviceBatch(e, nbuf=1024, buf_len=buf_len)  # 1024 x cap tasks: throughput form
    big.fill_streams(first_stream=5, bufs_per_stream=256)
    big.data[: 32 * buf_len].copy_(small.data)
    big.run()
    cs, ss, ls, ds, _ = small.host_results()
    cb, sb, lb, db, _ = big.host_results()
    assert (cs == cb[:32]).all()
    assert (ss == sb[:32]).all() and (ls == lb[:32]).all() and (ds == db[:32]).all()
    dl = O.Params(**prm).digest_len
    for b in list(range(0, 32, 3)) + [7]:
        es, el, ed = O.chunk(host[b].tobytes(), O.Params(**prm))
        c = cs[b]
        assert ss[b, :c].tolist() == es.tolist() and ls[b, :c].tolist() == el.tolist(), b
        assert (ds[b, :c, :dl] == ed).all(), b
    assert int(ls.max()) == prm["max_len"]  # a full maxLen chain went through the latency form


def test_config2_8gib_half_duplicate_full_size():
    """BASELINE configs[2] at its full size on one GPU: 8 GiB = 32768 write buffers of 256 KiB,
    the second half byte copies of the first (50 % duplicate).  Copies give identical chunk lists
    and digests; through the dedup-hit index every record of the second half is a duplicate whose
    hashloc is its original's, every first-half record is new; a sample of buffers equals the
    oracle (SparseDedupFile.java:435-446 drives the index this way)."""
    from sdfs_amd.index import HipHashesMap

    prm = P()
    e = engine_for(prm)
    half = 16384
    batch = DeviceBatch(e, nbuf=2 * half, buf_len=262144)
    batch.fill_streams(first_stream=0, bufs_per_stream=256)
    v = batch.data.view(2 * half, 262144)
    v[half:].copy_(v[:half])
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    _check_cover(counts, st, ln, 262144, prm)
    assert (counts[half:] == counts[:half]).all()
    assert (st[half:] == st[:half]).all() and (ln[half:] == ln[:half]).all() and (dg[half:] == dg[:half]).all()
    _check_batch_against_oracle(batch, counts, st, ln, dg, prm, 256, 0, [0, 5000, 16383])
    n1 = int(counts[:half].sum())
    ix = HipHashesMap(1 << 22)
    dup, loc, _, new_count = ix.put_records(batch.record_table(), batch.total, pos_base=1)
    torch.cuda.synchronize()
    dup, loc = dup.cpu().numpy(), loc.cpu().numpy()
    assert int(new_count.item()) == n1
    assert (dup[:n1] == 0).all() and (dup[n1:total] == 1).all()
    assert (loc[n1:total] == loc[:n1]).all()
    ix.destroy()


def test_config4_backup_per_gpu_share_16gib():
    """BASELINE configs[4] (BACKUP_VOLUME, 128 GiB over 8 GPUs) at one GPU's share: 409 write
    buffers of 40 MiB = 16 GiB, maxLen 128 KiB (VolumeConfigWriter.java:298-307), LDS-staged cut
    walk.  Exact cover / min / max on every buffer; a sample equals the oracle."""
    prm = P(max_len=131072)
    e = engine_for(prm)
    nbuf, L = 409, 40960 * 1024
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=L, records=False)
    batch.fill_streams(first_stream=900, bufs_per_stream=1)
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    _check_cover(counts, st, ln, L, prm)
    _check_batch_against_oracle(batch, counts, st, ln, dg, prm, 1, 900, [0, 204, 408])
    mean = nbuf * L / total
    assert 7000 < mean < 9000, mean


def test_config4_tar_stream_per_gpu_share_16gib():
    """BASELINE configs[4] (BACKUP_VOLUME, 128 GiB tar-like stream over 8 GPUs) at one GPU's share
    with its real content: 409 write buffers of 40 MiB = 16 GiB of 512-byte headers, log-uniform
    1 KiB-64 MiB bodies zero-padded to 512 and 20 % repeated bodies (sdfs_amd.device.tar_layout,
    SURVEY.md 8(d) B4), maxLen 128 KiB (VolumeConfigWriter.java:298-307).  Exact cover / min / max on
    every buffer; the first and last buffers and the buffers holding repeated bodies and their
    originals equal the oracle; and a repeated body dedups: after the first cut inside it, its
    chunks are the original's chunks (same offsets in the body, same digests)."""
    from sdfs_amd.device import tar_layout

    prm = P(max_len=131072)
    e = engine_for(prm)
    nbuf, L = 409, 40960 * 1024
    lay = tar_layout(nbuf * L)
    assert len(lay.repeats) > 50 and len(lay.bodies) > 500
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=L, records=False)
    batch.fill_tar(lay)
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    _check_cover(counts, st, ln, L, prm)
    mean = nbuf * L / total
    assert 6000 < mean < 9000, mean
    # repeated bodies of >= 4 MiB: chunk lists realign
    valid = np.arange(st.shape[1])[None, :] < counts[:, None]
    gs = (st.astype(np.int64) + (np.arange(nbuf, dtype=np.int64) * L)[:, None])[valid]
    gl = ln.astype(np.int64)[valid]
    gd = dg[valid]
    order = np.argsort(gs)
    gs, gl, gd = gs[order], gl[order], gd[order]

    def inside(a, n):
        i0, i1 = np.searchsorted(gs, a), np.searchsorted(gs, a + n)
        keep = [i for i in range(i0, i1) if gs[i] + gl[i] <= a + n]
        return {(int(gs[i] - a), int(gl[i])): bytes(gd[i]) for i in keep}

    checked = 0
    sample = {0, nbuf - 1}
    for c, o, n in lay.repeats:
        if n < (4 << 20):
            continue
        cp, og = inside(c, n), inside(o, n)
        common = set(cp) & set(og)
        assert all(cp[k] == og[k] for k in common)
        covered = sum(k[1] for k in common) / max(sum(k[1] for k in cp), 1)
        assert covered > 0.9, (c, o, n, covered)
        if checked < 3:
            sample |= {c // L, o // L}
        checked += 1
    assert checked >= 10
    # sampled buffers against the oracle
    sample = sorted(sample)
    host = np.stack([G.tar_bytes(lay, b * L, L) for b in sample])
    dev = batch.data.view(nbuf, L)
    for j, b in enumerate(sample):
        assert torch.equal(dev[b].cpu(), torch.from_numpy(host[j])), b
    offs = (np.arange(len(sample), dtype=np.uint64) * L).astype(np.uint64)
    ec, es, el, ed = O.chunk_batch(host.reshape(-1), offs, np.full(len(sample), L, np.uint32), O.Params(**prm),
                                   nthreads=16)
    for j, b in enumerate(sample):
        c = int(ec[j])
        assert counts[b] == c and (st[b, :c] == es[j, :c]).all() and (ln[b, :c] == el[j, :c]).all(), b
        assert (dg[b, :c] == ed[j, :c]).all(), b


_SCAN_VARIANT_CHECK = r"""
import os, sys
import numpy as np
sys.path.insert(0, os.environ["ROOT"])
from oracle import cdc_oracle as O
from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig
from tests.test_gpu_parity import _dense_candidate_buffers
nbuf, L = 32, 262144
dense = _dense_candidate_buffers(nbuf, L)
rnd = np.stack([O.synth(O.SYNTH_SEED, 7, b * L, L) for b in range(nbuf)])
# ragged lengths too: the guarded tail blocks and the separate cut walk
rl = [1, 47, 48, 300, 4095, 4097, 65537, 262143, 262144, 200003]
rb = np.concatenate([O.synth(5, 3, 0, n) for n in rl])
ro = np.concatenate([[0], np.cumsum(rl[:-1])]).astype(np.uint64)
PRMS = ((0xFFF, 4095), (0x7FF, 2047), (0x1FFF, 4095), (0x5A5, 4095))
exp = {}
for mask, min_len in PRMS:
    p = O.Params(min_len=min_len, pred_mask=mask)
    exp[mask] = ([[O.chunk(h[b].tobytes(), p) for b in range(nbuf)] for h in (dense, rnd)],
                 [O.chunk(rb[int(ro[b]): int(ro[b]) + n].tobytes(), p) for b, n in enumerate(rl)])
VARIANTS = [int(v) for v in os.environ.get("SCAN_VARIANTS", "0,29,30,31,32").split(",")]
if os.environ.get("LOWK_ONLY") == "1":  # round-3 sweep forms: the one-compare predicate only
    PRMS = tuple(p for p in PRMS if (p[0] & (p[0] + 1)) == 0)
for variant in VARIANTS:
    os.environ["SDFS_SCAN_VARIANT"] = str(variant)  # read at create (tuning library only)
    for mask, min_len in PRMS:
        cfg = SdfsConfig(min_len=min_len, pred_mask=mask)
        e = HipVariableSha256HashEngine(config=cfg)
        # 32 buffers: the short-segment scan + separate cut walk of small batches; 1024 buffers
        # (the 64 tiled 16 times): the fused one-wave-per-buffer scan and queue walk
        for reps, host, ex in ((1, dense, exp[mask][0][0]), (1, rnd, exp[mask][0][1]),
                               (16, np.concatenate([dense, rnd]), exp[mask][0][0] + exp[mask][0][1])):
            big = np.tile(host, (reps, 1))
            n = big.shape[0]
            offs = np.arange(n, dtype=np.uint64) * L
            c, st, ln, dg = e.chunk_batch(big.reshape(-1), offs, np.full(n, L, np.uint32))
            for b in range(n):
                es, el, ed = ex[b % len(ex)]
                k = int(c[b])
                assert st[b, :k].tolist() == es.tolist() and ln[b, :k].tolist() == el.tolist(), (variant, mask, n, b)
                assert (dg[b, :k] == ed).all(), (variant, mask, n, b)
        c, st, ln, dg = e.chunk_batch(rb, ro, np.array(rl, np.uint32))
        for b, n in enumerate(rl):
            es, el, ed = exp[mask][1][b]
            k = int(c[b])
            assert st[b, :k].tolist() == es.tolist() and ln[b, :k].tolist() == el.tolist(), (variant, mask, "ragged", b)
            assert (dg[b, :k] == ed).all(), (variant, mask, "ragged", b)
        e.destroy()
print("scan variants ok")
"""


def _run_scan_variant_check(variants, lowk_only=False):
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ROOT=root, SDFS_CDC_LIB=_lib.TUNING_LIB, SCAN_VARIANTS=",".join(map(str, variants)),
               LOWK_ONLY="1" if lowk_only else "0")
    r = subprocess.run([sys.executable, "-c", _SCAN_VARIANT_CHECK], capture_output=True, text=True, env=env,
                       timeout=110, cwd=root)
    assert r.returncode == 0 and "scan variants ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


def test_scan_variants_round3_agree():
    """Round-3 scan forms (cdc_sweep_r3.hip): SDWA push address (43), SDWA push +
    pop addresses (44), 16 table copies at 6 / 5 waves per SIMD (46 / 47), group-minimum candidate
    bits in groups of 4 / 8 (48 / 49), pop entries high word first (50), 49 + 50 (51), + the
    bit-select pop address (52), 50 + that (53) — the same oracle checks at the low-k-bit zero
    predicates (12, 11, 13 bits), the only ones those forms are built for."""
    _run_scan_variant_check([43, 44, 46, 47, 48, 49], lowk_only=True)
    _run_scan_variant_check([50, 51, 52, 53], lowk_only=True)


def test_scan_variants_agree():
    """The scan forms the A/B measurements of DESIGN.md §4/§8 compare (production; 29 plain rolling
    state; 30 mirrored state without the SGPR-mask candidate bits; 31 the round-2 cut walk; 32 =
    the production form as a sweep variant) all give the oracle's chunks and digests: dense
    candidate runs (summary overflow), random data, ragged lengths, 12-/11-/13-bit and pattern
    predicates.  Non-production forms exist only in the tuning library, so this runs in a child
    process bound to it."""
    import os
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, ROOT=root, SDFS_CDC_LIB=_lib.TUNING_LIB)
    r = subprocess.run([sys.executable, "-c", _SCAN_VARIANT_CHECK], capture_output=True, text=True, env=env,
                       timeout=110, cwd=root)
    assert r.returncode == 0 and "scan variants ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]


# ---------------------------------------------------------------- chunks longer than 32 KiB
@pytest.mark.parametrize("algo", [O.SHA256, O.SHA256_160, O.MD5])
@pytest.mark.parametrize("mask", [0xFFFFFF, 0xFFFF], ids=["forced", "mixed"])
def test_device_long_chunks_latency_form(algo, mask):
    """maxLen 128 KiB (the backup profile) makes chunks of more than 512 SHA-256 blocks; those head
    the longest-first task list and take the two-wave latency form inside chunk_hash_long_kernel
    (SHA-256 / SHA-256/160; MD5 keeps one lane per chunk).  A 24-bit predicate makes nearly every
    chunk a forced 128 KiB cut (2 048 long chunks, 32 latency-form groups), a 16-bit one a mix of
    4 KiB .. 128 KiB chunks; every chunk of every buffer against the oracle."""
    prm = P(max_len=131072, pred_mask=mask, hash_algo=algo)
    e = engine_for(prm)
    nbuf, L = 64, 4 * 2**20
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=L, records=False)
    batch.fill_streams(first_stream=910, bufs_per_stream=1)
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    nlong = int(sum((ln[b, :counts[b]] > 32768).sum() for b in range(nbuf)))
    assert nlong > (1500 if mask == 0xFFFFFF else 64), nlong
    _check_batch_against_oracle(batch, counts, st, ln, dg, prm, 1, 910, None)


def test_device_long_chunks_beyond_split_cap():
    """More long chunks than kLongSplitMax (16 384) in one batch: every chunk takes the lane form
    (the latency form would cost throughput there).  520 x 4 MiB with forced 128 KiB cuts =
    16 640 long chunks; exact cover, every length a forced cut or a tail, a sample vs the oracle,
    and identical digests for identical chunks across buffers."""
    prm = P(max_len=131072, pred_mask=0xFFFFFF)
    e = engine_for(prm)
    nbuf, L = 520, 4 * 2**20
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=L, records=False)
    batch.fill_streams(first_stream=1200, bufs_per_stream=1)
    v = batch.data.view(nbuf, L)
    v[1::2].copy_(v[0::2])  # odd buffers copy even ones: their chunk lists must be identical
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    nlong = int(sum((ln[b, :counts[b]] > 32768).sum() for b in range(nbuf)))
    assert nlong > 16384, nlong
    _check_cover(counts, st, ln, L, prm)
    for b in range(0, nbuf, 2):
        c = counts[b]
        assert counts[b + 1] == c and (st[b + 1, :c] == st[b, :c]).all() and (dg[b + 1, :c] == dg[b, :c]).all()
    host = batch.data.view(nbuf, L)
    for b in (0, 1, 257, 518):
        buf = host[b].cpu().numpy()
        es, el, ed = O.chunk(buf, O.Params(**prm))
        c = counts[b]
        assert st[b, :c].tolist() == es.tolist() and ln[b, :c].tolist() == el.tolist(), b
        assert (dg[b, :c] == ed).all(), b


def test_sectioned_mixed_joined_and_stitched_buffers():
    """One batch of 5 MiB buffers (sectioned cut walk) where some buffers' sections all join in
    parallel and others need the sequential stitch (all-zero data whose cuts never line up with
    the sections; a 16-bit predicate's forced cuts out of phase): each buffer exactly as the oracle,
    and the record table consistent with the slots (the histogram both passes feed)."""
    prm = P(min_len=2999, max_len=131072)
    L, nbuf = 5 * 2**20, 6
    e = engine_for(prm)
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=L)
    batch.fill_streams(first_stream=1300, bufs_per_stream=1)
    v = batch.data.view(nbuf, L)
    v[1].zero_()                      # never joins: falls back
    v[4, 1_000_000:3_500_000].zero_()  # a zero run across two sections
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    host = v.cpu().numpy()
    for b in range(nbuf):
        es, el, ed = O.chunk(host[b], O.Params(**prm))
        c = counts[b]
        assert st[b, :c].tolist() == es.tolist() and ln[b, :c].tolist() == el.tolist(), b
        assert (dg[b, :c] == ed).all(), b
    recs = batch.record_table().cpu().numpy()
    assert len(recs) == total
    want = sorted(bytes(dg[b, i]) for b in range(nbuf) for i in range(counts[b]))
    assert sorted(bytes(r[:32]) for r in recs) == want  # every chunk fingerprinted exactly once


def _list_walk_buffers(nbuf: int, buf_len: int, seed: int) -> np.ndarray:
    """Random buffers with constant-byte stretches (a constant window is not a candidate, so the
    walk meets max_len chunks ending at non-candidates there) of varying length and place: none,
    one short, one longer than max_len mid-buffer, one running to the buffer end, several."""
    rng = np.random.default_rng(seed)
    host = rng.integers(0, 256, nbuf * buf_len, dtype=np.uint8).reshape(nbuf, buf_len)
    for b in range(nbuf):
        kind = b % 5
        if kind == 1:
            o = int(rng.integers(0, buf_len - 8192))
            host[b, o:o + int(rng.integers(100, 8000))] = 0x5A
        elif kind == 2:
            o = int(rng.integers(0, buf_len // 2))
            host[b, o:o + int(rng.integers(70000, 120000))] = 0xA5
        elif kind == 3:
            host[b, buf_len - int(rng.integers(1000, 90000)):] = 0x33
        elif kind == 4:
            for _ in range(6):
                o = int(rng.integers(0, buf_len - 40000))
                host[b, o:o + int(rng.integers(2000, 40000))] = 0x77
    return host


@pytest.mark.parametrize("prm", [
    P(),                                                  # the reference default mix
    P(min_len=2047, pred_mask=0x7FF),                     # the metric's 4 KiB-mean mix
    P(min_len=10239, pred_mask=0x7FF, max_len=65536),     # minLen spans several scan segments
    P(min_len=511, pred_mask=0x3FF, max_len=6000),        # ~256 candidates per buffer: list full or over
    P(min_len=2047, pred_mask=0x1FFF, max_len=8192),      # max_len chunks at non-candidates everywhere
], ids=["default", "mix4k", "long_min", "list_cap", "forced"])
def test_fused_list_walk_edges(prm):
    """The fused walk's list form (scan epilogue, uniform 256 KiB buffers) and its fall-back to the
    queue walk (summary overflow, > 256 candidates per buffer, forced cuts), buffer by buffer
    against the oracle.  1024 buffers: smaller batches scan in short segments, without the fused
    walk."""
    e = engine_for(prm)
    nbuf, buf_len = 1024, 262144
    host = _list_walk_buffers(nbuf, buf_len, seed=len(str(prm)))
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=buf_len)
    batch.data.copy_(torch.from_numpy(host.reshape(-1)))
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == counts.sum()
    dl = O.Params(**prm).digest_len
    for b in range(nbuf):
        es, el, ed = O.chunk(host[b].tobytes(), O.Params(**prm))
        c = counts[b]
        assert c == len(es), b
        assert st[b, :c].tolist() == es.tolist() and ln[b, :c].tolist() == el.tolist(), b
        assert (dg[b, :c, :dl] == ed).all(), b


def test_sectioned_batch_with_empty_buffers_after_a_full_batch():
    """A ragged host batch holding a >= 4 MiB buffer (sectioned walk with the parallel join/place)
    and EMPTY buffers, run right after batches that left non-zero counts in the reused result
    slots: an empty buffer has no section, so the place kernel settles it (count 0) — before, its
    join flag was stale workspace memory and a stale count could come back."""
    prm = P()
    e = engine_for(prm)
    for _ in range(2):
        full = O.synth(SYNTH_SEED, 1400, 0, 4 * 262144)
        c0, *_ = e.chunk_batch(full, np.arange(4, dtype=np.uint64) * 262144, np.full(4, 262144, np.uint32))
        assert (c0 > 0).all()
        lens = np.array([0, 5 * 2**20 + 3, 0, 300000, 0], dtype=np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64))]).astype(np.uint64)
        base = O.synth(SYNTH_SEED, 1401, 0, int(lens.sum()))
        counts, st, ln, dg = e.chunk_batch(base, offs, lens)
        for b in range(len(lens)):
            if lens[b] == 0:
                assert counts[b] == 0, b
                continue
            buf = base[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
            c = counts[b]
            assert_same((st[b, :c], ln[b, :c], dg[b, :c]), O.chunk(buf, O.Params(**prm)), b)


def test_piece_mode_sections_joined_and_stitched():
    """Piece mode: a uniform batch of long buffers large enough for full 4 KiB scan segments
    (>= num_cus * 4 * 64 of them) whose 256 Ki-position sections are exactly one wave's 64
    segments, so the scan's epilogue walks every section from the lanes' summaries and the bitmap is
    stored only sparsely.  Buffers whose sections never join (all zero; a zero run across sections;
    cuts out of phase with the sections) take the stitch fallback, which then searches the segment
    summaries (find_first_sum).  Every buffer against the oracle."""
    prm = P(min_len=2999, max_len=131072)
    L, nbuf = 5 * 2**20, 64
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    # the engine's piece-mode conditions (cdc_engine.hip run_pipeline): full-length segments for a
    # batch of >= ncu*4*64 of them, section = 2^18 positions = 64 segments of 4 KiB, uniform_len % section == 0
    assert nbuf * L // 4096 >= ncu * 4 * 64 and L % (1 << 18) == 0 and 2 * prm["max_len"] <= (1 << 18)
    e = engine_for(prm)
    batch = DeviceBatch(e, nbuf=nbuf, buf_len=L)
    batch.fill_streams(first_stream=1500, bufs_per_stream=1)
    v = batch.data.view(nbuf, L)
    v[1].zero_()
    v[4, 1_000_000:3_500_000].zero_()
    v[9, 262_100:262_200].zero_()
    v[17, :].fill_(0x5A)               # constant: no candidates, forced cuts only
    v[33, 2**20:].zero_()
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    host = v.cpu().numpy()
    offs = (np.arange(nbuf, dtype=np.uint64) * L).astype(np.uint64)
    ec, es, el, ed = O.chunk_batch(host.reshape(-1), offs, np.full(nbuf, L, np.uint32), O.Params(**prm), nthreads=16)
    for b in range(nbuf):
        c = int(ec[b])
        assert counts[b] == c and (st[b, :c] == es[b, :c]).all() and (ln[b, :c] == el[b, :c]).all(), b
        assert (dg[b, :c] == ed[b, :c]).all(), b


def test_jar_fixtures_bit_exact():
    """tests/golden/jar_cdc.json, when present, holds the rabinwindow jar's OWN chunk lists for the
    inputs of cdc.json (tools/java/JarParity.java --emit on a host with a JDK and the jar; absent in
    this image).  Every fixture whose knob setting reproduces the jar's list is then run on the GPU
    with that setting and must equal the jar — boundary parity pinned to the reference itself."""
    import os

    path = os.path.join(G.GOLDEN, "jar_cdc.json")
    if not os.path.exists(path):
        pytest.skip("no jar_cdc.json: the rabinwindow jar has not been run (INTEGRATION.md §4)")
    jar = {f["name"]: f for f in G.load("jar_cdc.json")["fixtures"]}
    matched = 0
    for fx in G.fixtures():
        j = jar.get(fx["name"])
        if j is None or (j["starts"], j["lens"], j["digests"]) != (fx["starts"], fx["lens"], fx["digests"]):
            continue
        matched += 1
        data = G.fixture_input(fx)
        got = engine_for(fx["params"]).chunk_arrays(data)
        assert_same(got, (j["starts"], j["lens"], [bytes.fromhex(h) for h in j["digests"]]), fx["name"])
    assert matched > 0, "no knob setting of cdc.json reproduces the jar: add its detector to make_golden.py"
