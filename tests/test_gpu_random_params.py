"""Seeded random parameter sets through the GPU path against the oracle (bit-exact): polynomials
of every supported degree (48..55), windows 16/32/48/64, min/max lengths from 0 to 128 KiB, both
min comparisons, arbitrary boundary masks and values (one-word, two-word and low-k-zero forms),
the divisor detector, SHA-256 / SHA-256/160 / MD5; each set on a ragged host batch (random data,
zero runs, a repeated buffer, empty and sub-window buffers) and on single queued calls.  The
reference's parameters come from HashFunctionPool (HashFunctionPool.java:45-69); the jar accepts
any polynomial (Polynomial.createFromLong) and window, so the engine must too."""
import numpy as np
import pytest

from oracle import cdc_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from sdfs_amd import HipVariableMD5HashEngine, HipVariableSha256HashEngine, SdfsConfig  # noqa: E402

N_SETS = 24


def _random_params(rng):
    deg = int(rng.integers(48, 56))
    poly = (1 << deg) | int(rng.integers(1, 1 << 40)) | 1
    window = int(rng.choice([16, 32, 48, 64]))
    min_len = int(rng.choice([0, 1, 63, 511, 1023, 2047, 4095, 8191, int(rng.integers(0, 6000))]))
    max_len = int(min(131072, max(min_len + 1, min_len + int(rng.integers(1, 40000)))))
    if rng.random() < 0.15:
        max_len = int(rng.integers(1, min_len + 2))  # max below min: every cut forced
    min_cmp = int(rng.integers(0, 2))
    algo = int(rng.choice([O.SHA256, O.SHA256_160, O.MD5]))
    kind = rng.random()
    prm = dict(poly=poly, window=window, min_len=min_len, max_len=max_len, min_cmp=min_cmp, hash_algo=algo)
    if kind < 0.35:  # low k bits zero (the mirrored scan's one-compare form)
        k = int(rng.integers(6, 14))
        prm.update(pred_mask=(1 << k) - 1, pred_value=0)
    elif kind < 0.6:  # a scattered one-word mask with a value inside it
        m = int(rng.integers(1, 1 << 32)) & int(rng.integers(1, 1 << 32))
        while bin(m).count("1") > 14:
            m &= m - 1
        prm.update(pred_mask=m, pred_value=int(rng.integers(0, 1 << 32)) & m)
    elif kind < 0.8:  # a mask reaching into the high word
        hi_bit = int(rng.integers(32, deg))
        m = (1 << hi_bit) | ((1 << int(rng.integers(4, 11))) - 1)
        prm.update(pred_mask=m, pred_value=int(rng.integers(0, 1 << 62)) & m)
    else:  # the divisor detector (f64 form needs degree <= 53)
        d = int(rng.choice([3, 1000, 4099, 6007, 4096, 8192]))
        if d & (d - 1) and deg > 53:
            prm["poly"] = (1 << 53) | int(rng.integers(1, 1 << 40)) | 1
        prm.update(pred_kind=O.PRED_DIV, pred_div=d, pred_rem=int(rng.integers(0, d)))
    return prm


def _engine(prm):
    cfg = SdfsConfig(min_len=prm["min_len"], max_len=prm["max_len"], window=prm["window"], poly=prm["poly"],
                     pred_mask=prm.get("pred_mask", 0), pred_value=prm.get("pred_value", 0),
                     min_cmp=prm["min_cmp"], pred_kind=prm.get("pred_kind", 0), pred_div=prm.get("pred_div", 0),
                     pred_rem=prm.get("pred_rem", 0))
    if prm["hash_algo"] == O.MD5:
        return HipVariableMD5HashEngine(cfg)
    return HipVariableSha256HashEngine(
        HipVariableSha256HashEngine.HASH160 if prm["hash_algo"] == O.SHA256_160 else HipVariableSha256HashEngine.HASH256, cfg)


@pytest.mark.parametrize("seed", range(N_SETS))
def test_random_parameter_set_bit_exact(seed):
    rng = np.random.default_rng(0x5DF5 + seed)
    prm = _random_params(rng)
    p = O.Params(**prm)
    e = _engine(prm)
    try:
        bufs = []
        for i in range(6):
            n = int(rng.integers(1, 300000)) if i else int(rng.choice([0, 5, prm["window"] - 1, 262144]))
            b = rng.integers(0, 256, n, dtype=np.uint8)
            if n > 20000 and rng.random() < 0.5:
                z = int(rng.integers(0, n - 10000))
                b[z:z + int(rng.integers(100, 10000))] = 0
            bufs.append(b)
        bufs.append(bufs[1].copy())  # a repeated buffer: identical lists
        lens = np.array([len(b) for b in bufs], dtype=np.uint32)
        offs = np.concatenate([[0], np.cumsum(lens[:-1].astype(np.uint64) + 7)]).astype(np.uint64)  # unaligned
        base = np.zeros(int(offs[-1]) + int(lens[-1]) + 64, np.uint8)
        for o, b in zip(offs, bufs):
            base[int(o):int(o) + len(b)] = b
        counts, st, ln, dg = e.chunk_batch(base, offs, lens)
        dl = p.digest_len
        for i, b in enumerate(bufs):
            es, el, ed = O.chunk(b.tobytes(), p) if len(b) else ([], [], [])
            c = counts[i]
            assert st[i, :c].tolist() == list(es) and ln[i, :c].tolist() == list(el), (seed, i, prm)
            assert [bytes(x[:dl]) for x in dg[i, :c]] == [bytes(x) for x in ed], (seed, i, prm)
        for i in (1, 2):  # single queued calls (the coalescing queue's small-pass route)
            gs, gl, gd = e.chunk_arrays(bufs[i].tobytes())
            es, el, ed = O.chunk(bufs[i].tobytes(), p)
            assert gs.tolist() == list(es) and gl.tolist() == list(el) and (gd == ed).all(), (seed, i, prm)
    finally:
        e.destroy()
