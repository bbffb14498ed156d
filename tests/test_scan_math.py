"""CPU tests of the scan kernel's word-level arithmetic (sdfs_amd/csrc/cdc_device.h roll_step):
the 32-bit operations the kernel issues per byte, restated in Python, reproduce the oracle's
window fingerprint at every position.

Covers the mirrored (bit-reversed) rolling state used by the production scan: R = bitrev64(fp)
held as hi:lo, data dwords bit-reversed, tables indexed by the reversed byte, and the one-compare
predicate `hi < 2^(32-k)` for (fp & (2^k - 1)) == 0.  The GPU kernels themselves are checked
against the oracle in tests/test_gpu_parity.py.
"""
import numpy as np
import pytest

from oracle import cdc_oracle as O

M32 = 0xFFFFFFFF


def bitrev(v: int, n: int) -> int:
    return int(format(v, f"0{n}b")[::-1], 2)


def perm(s0: int, s1: int, sel: int) -> int:
    """v_perm_b32: selector byte 0-3 -> s1 byte, 4-7 -> s0 byte, 0x0C -> 0x00."""
    src = s1.to_bytes(4, "little") + s0.to_bytes(4, "little")
    out = 0
    for i in range(4):
        k = (sel >> (8 * i)) & 0xFF
        b = src[k] if k < 8 else 0
        out |= b << (8 * i)
    return out


def alignbit(a: int, b: int, s: int) -> int:
    return (((a << 32) | b) >> s) & M32


def mirrored_tables(poly: int, window: int):
    d = poly.bit_length() - 1
    push = [(i << d) ^ O.gf2_mod(i << d, poly) for i in range(256)]
    pop = [O.gf2_mod(i << (8 * window), poly) for i in range(256)]
    mp = [bitrev(push[bitrev(x, 8)], 64) for x in range(256)]
    mq = [bitrev(pop[bitrev(x, 8)], 64) for x in range(256)]
    return mp, mq


def mirrored_scan(data: bytes, poly: int, window: int):
    """Per-position (lo, hi) of the mirrored state, as the kernel computes it (first segment of a
    buffer: zero window history)."""
    d = poly.bit_length() - 1
    jshift = 64 - d
    mp, mq = mirrored_tables(poly, window)
    n = len(data)
    padded = data + bytes((-n) % 4)
    dws = [bitrev(int.from_bytes(padded[i:i + 4], "little"), 32) for i in range(0, len(padded), 4)]
    lo = hi = 0
    out = []
    for i in range(n):
        dw = dws[i >> 2]
        p = i & 3
        x = ((lo >> (jshift - 8)) & 0xFF00) >> 8           # bitop3_and_or(lo >> (jshift-8), 0xFF00, base)
        nlo = alignbit(hi, lo, 8)
        nhi = perm(hi, dw, 0x00070605 | ((3 - p) << 24))
        pv = mp[x]
        lo, hi = nlo ^ (pv & M32), nhi ^ (pv >> 32)
        if i >= window:                                    # the byte leaving the window
            o = i - window
            odw = dws[o >> 2]
            q = o & 3
            qa = (odw & 0xFF00) if q == 2 else perm(odw, 0, 0x0C0C0000 | ((4 + 3 - q) << 8))
            qv = mq[qa >> 8]
            lo, hi = lo ^ (qv & M32), hi ^ (qv >> 32)
        out.append((lo, hi))
    return out


@pytest.mark.parametrize("window", [16, 32, 48, 64])
def test_mirrored_state_is_bitrev_of_window_fp(window):
    rng = np.random.default_rng(100 + window)
    data = rng.integers(0, 256, 1500, dtype=np.uint8).tobytes()
    fps = O.window_fps(data, O.POLY, window)
    st = mirrored_scan(data, O.POLY, window)
    for i, (lo, hi) in enumerate(st):
        assert (hi << 32 | lo) == bitrev(int(fps[i]), 64), i


@pytest.mark.parametrize("deg", [48, 50, 53, 55])
def test_mirrored_state_other_degrees(deg):
    rng = np.random.default_rng(deg)
    poly = (1 << deg) | int(rng.integers(1, 1 << 40)) | 1
    data = rng.integers(0, 256, 700, dtype=np.uint8).tobytes()
    fps = O.window_fps(data, poly, 48)
    for i, (lo, hi) in enumerate(mirrored_scan(data, poly, 48)):
        assert (hi << 32 | lo) == bitrev(int(fps[i]), 64), i


@pytest.mark.parametrize("k", [1, 8, 11, 12, 13, 16, 32])
def test_one_compare_predicate(k):
    """(fp & (2^k-1)) == 0  <=>  hi < 2^(32-k) for hi = bitrev64(fp) >> 32 (engine: sa.thr)."""
    rng = np.random.default_rng(k)
    thr = 1 if k == 32 else 1 << (32 - k)
    mask = (1 << k) - 1
    vals = [int(v) for v in rng.integers(0, 1 << 53, 4000, dtype=np.uint64)]
    vals += [v & ~mask for v in vals[:200]] + [(v & ~mask) | (1 << (k - 1)) for v in vals[200:400]]
    for fp in vals:
        hi = bitrev(fp, 64) >> 32
        assert ((fp & mask) == 0) == (hi < thr), (fp, k)
