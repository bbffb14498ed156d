"""GPU parity of the DIVISOR form of the boundary detector, fp % D == R (the jar's
BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR, VariableSha256HashEngine.java:42, is either a bitmask
or a divisor detector, and which one is unpinned here).  Powers of two run as the equivalent mask;
every other divisor runs the scan's f64 remainder (cdc_device.h cand_shift<3>).  Bar: bit-exact
against the oracle (oracle/cdc_ref.c with the same detector), through the C-ABI.

The golden fixtures with a divisor (div*_256k ...) run in test_gpu_parity.py::test_golden_fixture_bit_exact."""
import numpy as np
import pytest

from oracle import cdc_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from sdfs_amd import HipVariableSha256HashEngine, SdfsConfig  # noqa: E402
from sdfs_amd import _lib  # noqa: E402
from sdfs_amd.device import SYNTH_SEED, DeviceBatch  # noqa: E402
from tests.test_gpu_parity import _check_cover, _dense_candidate_buffers  # noqa: E402

DIVS = [(4096, 0), (4096, 4095), (8192, 0), (8192, 8191), (4099, 0), (4099, 4098), (6007, 17), (12289, 12288)]


def _engine(div, rem, **kw):
    cfg = SdfsConfig(pred_kind=_lib.PRED_DIV, pred_div=div, pred_rem=rem, **kw)
    return HipVariableSha256HashEngine(config=cfg), O.Params(pred_kind=O.PRED_DIV, pred_div=div, pred_rem=rem,
                                                             min_len=cfg.min_len, max_len=cfg.max_len)


def _compare_all(host: np.ndarray, counts, st, ln, dg, p: O.Params):
    nbuf, buf_len = host.shape
    offs = (np.arange(nbuf, dtype=np.uint64) * buf_len).astype(np.uint64)
    lens = np.full(nbuf, buf_len, np.uint32)
    ec, es, el, ed = O.chunk_batch(host.reshape(-1), offs, lens, p, nthreads=16)
    for b in range(nbuf):
        c = int(ec[b])
        assert counts[b] == c, b
        assert (st[b, :c] == es[b, :c]).all() and (ln[b, :c] == el[b, :c]).all(), b
        assert (dg[b, :c] == ed[b, :c]).all(), b


@pytest.mark.parametrize("div,rem", DIVS)
def test_device_batch_random(div, rem):
    """256 write buffers of 256 KiB (fused walk), every buffer against the oracle."""
    e, p = _engine(div, rem)
    batch = DeviceBatch(e, nbuf=256, buf_len=262144)
    batch.fill_streams(first_stream=600 + div % 7, bufs_per_stream=64)
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    assert total == int(counts.sum())
    host = batch.data.cpu().numpy().reshape(256, 262144)
    _compare_all(host, counts, st, ln, dg, p)
    e.destroy()


@pytest.mark.parametrize("div", [4096, 4099, 8192, 3])
def test_device_batch_dense(div):
    """Zero runs: an all-zero window fingerprints to 0, so with R = 0 every position in a run is a
    candidate (register-summary overflow, bitmap path) under the divisor form too."""
    kw = dict(min_len=1023, max_len=8192) if div == 3 else {}
    e, p = _engine(div, 0, **kw)
    host = _dense_candidate_buffers(32, 262144)
    batch = DeviceBatch(e, nbuf=32, buf_len=262144)
    batch.data.copy_(torch.from_numpy(host.reshape(-1)))
    batch.run()
    counts, st, ln, dg, _ = batch.host_results()
    _compare_all(host, counts, st, ln, dg, p)
    e.destroy()


def test_host_paths_ragged_and_single():
    """Ragged host batch (small-segment scan + separate resolve) and single getChunks calls (the
    coalescing queue) with a non-power-of-two divisor and the 4 KiB-mean minLen."""
    e, p = _engine(2039, 5, min_len=2047)
    rng = np.random.default_rng(77)
    lens = rng.integers(1, 300000, 24).astype(np.uint32)
    lens[2] = 0
    offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 7)]).astype(np.uint64)
    base = O.synth(SYNTH_SEED, 640, 0, int(offs[-1] + lens[-1]))
    counts, st, ln, dg = e.chunk_batch(base, offs, lens)
    for b in range(len(lens)):
        buf = base[int(offs[b]): int(offs[b]) + int(lens[b])].tobytes()
        es, el, ed = O.chunk(buf, p) if lens[b] else ([], [], np.zeros((0, 32), np.uint8))
        c = counts[b]
        assert st[b, :c].tolist() == list(es) and ln[b, :c].tolist() == list(el), b
        assert (dg[b, :c] == ed).all(), b
    for n in (100, 4096, 262144):
        d = O.synth(SYNTH_SEED, 650 + n % 13, 0, n)
        s2, l2, d2 = e.chunk_arrays(d)
        es, el, ed = O.chunk(d, p)
        assert s2.tolist() == es.tolist() and l2.tolist() == el.tolist() and (d2 == ed).all(), n
    e.destroy()


def test_backup_buffer_sectioned_walk():
    """A 40 MiB BACKUP_VOLUME buffer (sectioned cut walk) with a divisor detector."""
    cfg = SdfsConfig.backup_volume(pred_kind=_lib.PRED_DIV, pred_div=8191, pred_rem=0)
    e = HipVariableSha256HashEngine(config=cfg)
    p = O.Params(pred_kind=O.PRED_DIV, pred_div=8191, pred_rem=0, max_len=131072)
    buf = O.synth(SYNTH_SEED, 660, 0, 40960 * 1024)
    s2, l2, d2 = e.chunk_arrays(buf)
    es, el, ed = O.chunk(buf, p)
    assert s2.tolist() == es.tolist() and l2.tolist() == el.tolist() and (d2 == ed).all()
    e.destroy()


def test_full_size_properties_non_power_of_two():
    """configs[1]'s full 4 GiB with D = 4099: exact cover, min/max, a sample vs the oracle, and the
    mean chunk length the divisor predicts (one candidate per D positions after minLen)."""
    e, p = _engine(4099, 0)
    batch = DeviceBatch(e, nbuf=16384, buf_len=262144, records=False)
    batch.fill_streams(first_stream=0, bufs_per_stream=256)
    batch.run()
    counts, st, ln, dg, total = batch.host_results()
    prm = dict(min_len=4095, max_len=32768)
    _check_cover(counts, st, ln, 262144, prm)
    sample = [0, 1, 4097, 9000, 16383]
    for b in sample:
        buf = O.synth(SYNTH_SEED, b // 256, (b % 256) * 262144, 262144)
        es, el, ed = O.chunk(buf, p)
        c = counts[b]
        assert st[b, :c].tolist() == es.tolist() and ln[b, :c].tolist() == el.tolist() and (dg[b, :c] == ed).all(), b
    mean = 262144 * 16384 / total
    assert 7000 < mean < 9500, mean
    e.destroy()


def test_invalid_divisor_parameters_fail():
    for kw in (dict(pred_div=0), dict(pred_div=1 << 32)):
        with pytest.raises(_lib.SdfsCdcError):
            HipVariableSha256HashEngine(config=SdfsConfig(pred_kind=_lib.PRED_DIV, **kw))
    with pytest.raises(_lib.SdfsCdcError):  # f64 form needs deg(P) <= 53
        HipVariableSha256HashEngine(config=SdfsConfig(pred_kind=_lib.PRED_DIV, pred_div=4099,
                                                      poly=(1 << 55) | 0x1B))
