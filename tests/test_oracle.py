"""CPU tests: pin the oracle (oracle/cdc_ref.c + oracle/cdc_oracle.py) against the golden vectors
and against independent restatements, before it is trusted as the GPU checker.

Pinned: SHA-256 (FIPS 180-2 vectors), MD5 (RFC 1321 suite), the reference's blank-chunk digests
(WritableCacheBuffer.java:93-94, HashStore.java:63-71), the rolling tables and every window
fingerprint (GF(2) definition).  Boundary rules: parity unpinned —
checked here only for self-consistency of three restatements (C loop, Python loop, two-phase
candidate+resolve formulation that the GPU implements).
"""
import hashlib

import numpy as np
import pytest

from oracle import cdc_oracle as O
from tests import golden_util as G


def test_sha256_md5_known_answers():
    kat = G.load("kat.json")
    for msg, h in kat["sha256"]:
        assert O.hash_bytes(msg.encode(), O.SHA256).hex() == h
    assert O.hash_bytes(b"a" * 1000000, O.SHA256).hex() == kat["sha256_million_a"]
    for msg, h in kat["md5"]:
        assert O.hash_bytes(msg.encode(), O.MD5).hex() == h


def test_reference_blank_chunk_constants():
    kat = G.load("kat.json")["blank"]
    assert O.hash_bytes(bytes(4096)).hex() == kat["sha256_zero_4096"]
    assert O.hash_bytes(bytes(262144)).hex() == kat["sha256_zero_262144"]
    # HASH160 variant is the 20-byte prefix (VariableSha256HashEngine.java:60-65)
    assert O.hash_bytes(bytes(4096), O.SHA256_160).hex() == kat["sha256_zero_4096"][:40]


@pytest.mark.parametrize("n", [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128, 4095, 4096, 4097, 32768])
def test_hash_lengths_vs_hashlib(n):
    data = O.synth(1, 99, 0, n).tobytes()
    assert O.hash_bytes(data, O.SHA256) == hashlib.sha256(data).digest()
    assert O.hash_bytes(data, O.MD5) == hashlib.md5(data).digest()


def test_tables_match_gf2_definition_and_golden():
    t = G.load("tables.json")
    push, pop = O.tables(O.POLY, 48)
    assert [hex(int(v)) for v in push] == t["push"]
    assert [hex(int(v)) for v in pop] == t["pop"]
    assert int(push[1]) == O.POLY  # holds by construction
    # only push[0..255] are reachable since fp < 2^53
    pp, _ = O.py_tables(O.POLY, 48)
    assert all(pp[i] >> 53 == i for i in range(512))


@pytest.mark.parametrize("window", [16, 32, 48, 64])
def test_window_fp_is_the_gf2_residue(window):
    rng = np.random.default_rng(window)
    data = rng.integers(0, 256, 3000, dtype=np.uint8).tobytes()
    fps = O.window_fps(data, O.POLY, window)
    for k in list(range(0, 70)) + rng.integers(70, 3000, 200).tolist():
        assert int(fps[k]) == O.gf2_window_fp(data, k, O.POLY, window), k


def test_synth_numpy_matches_c():
    for stream, off, n in [(0, 0, 4096), (5, 13, 1000), (63, 64 << 20, 777), (2**40, 7, 65)]:
        assert (O.synth(O.SYNTH_SEED, stream, off, n) == O.synth_c(O.SYNTH_SEED, stream, off, n)).all()


@pytest.mark.parametrize("fx", G.fixtures(), ids=lambda f: f["name"])
def test_oracle_reproduces_golden_fixture(fx):
    data = G.fixture_input(fx)
    st, ln, dg = O.chunk(data, G.oracle_params(fx))
    assert st.tolist() == fx["starts"]
    assert ln.tolist() == fx["lens"]
    assert [d.tobytes().hex() for d in dg] == fx["digests"]


@pytest.mark.parametrize("fx", G.fixtures(), ids=lambda f: f["name"])
def test_chunk_list_contract(fx):
    """Ascending, contiguous, exact cover, len > 0; interior chunks respect min/max
    (SparseDedupFile.java:535-564, HashLocPair.java:66-68)."""
    p = G.oracle_params(fx)
    st, ln = np.array(fx["starts"], np.int64), np.array(fx["lens"], np.int64)
    total = fx["input"]["len"]
    if total == 0:
        assert len(st) == 0
        return
    assert st[0] == 0 and (ln > 0).all()
    assert (st[1:] == st[:-1] + ln[:-1]).all() and st[-1] + ln[-1] == total
    shortest = p.min_len + 1 if p.min_cmp == O.MIN_GT else p.min_len
    assert (ln[:-1] >= min(shortest, p.max_len)).all() and (ln <= p.max_len).all()


@pytest.mark.parametrize("name", ["rand_256k", "rand_256k_ge", "rand_256k_small", "rand_256k_dense", "hole_256k",
                                  "zeros_256k", "rand_256k_mask64", "rand_256k_min0", "rand_256k_w64",
                                  "div4099_r0_256k", "div3_dense_256k", "div4099_never_256k", "div4099_zeros_256k",
                                  "div8192_rmax_256k"])
def test_two_phase_formulation_equals_rolling_loop(name):
    """The GPU computes a candidate bitmap over ALL positions, then resolves cuts greedily; that
    must equal the reference's byte-serial loop for every knob combination."""
    fx = next(f for f in G.fixtures() if f["name"] == name)
    data = G.fixture_input(fx)
    p = G.oracle_params(fx)
    fps = O.window_fps(data, p.poly, p.window)
    cand = p.is_boundary(fps)
    got = O.resolve_from_candidates(cand, len(data), p)
    assert got == list(zip(fx["starts"], fx["lens"]))


def test_zero_buffer_chunks_into_blank_blocks():
    """fp == 0 on zero data, so a zero CHUNK_LENGTH buffer cuts every minLen+1 = 4096 bytes and
    every chunk hashes to WritableCacheBuffer.bk (the hint behind the A.3 defaults)."""
    st, ln, dg = O.chunk(bytes(262144))
    assert ln.tolist() == [4096] * 64
    assert {d.tobytes().hex() for d in dg} == {G.load("kat.json")["blank"]["sha256_zero_4096"]}


def test_batch_equals_single_calls_and_threads():
    bufs = [O.synth(O.SYNTH_SEED, s, 0, n).tobytes() for s, n in [(0, 262144), (1, 1000), (2, 70000), (3, 0)]]
    offs = np.cumsum([0] + [len(b) for b in bufs[:-1]]).astype(np.uint64)
    lens = np.array([len(b) for b in bufs], np.uint32)
    base = np.frombuffer(b"".join(bufs), np.uint8)
    for nt in (1, 3):
        counts, st, ln, dg = O.chunk_batch(base, offs, lens, nthreads=nt)
        for i, b in enumerate(bufs):
            s1, l1, d1 = O.chunk(b) if len(b) else (np.zeros(0), np.zeros(0), np.zeros((0, 32)))
            assert counts[i] == len(s1)
            assert st[i, : counts[i]].tolist() == list(s1) and ln[i, : counts[i]].tolist() == list(l1)
            assert (dg[i, : counts[i]] == d1).all()


@pytest.mark.parametrize("fx", G.fixtures(), ids=lambda f: f["name"])
def test_fast_cpu_form_equals_reference_loop(fx):
    """oracle/cdc_fast.c (bench.py's CPU baseline: table loop + OpenSSL digests) gives the same
    chunks and digests as the restatement on every golden fixture."""
    data = G.fixture_input(fx)
    p = O.Params(**fx["params"])
    got, exp = O.chunk_fast(data, p), O.chunk(data, p)
    for x, y in zip(got, exp):
        assert np.array_equal(x, y), fx["name"]


def test_fast_cpu_form_edge_lengths_and_params():
    for n in (0, 1, 47, 48, 49, 4095, 4096, 4097, 32767, 32768, 32769, 262144):
        data = O.synth(O.SYNTH_SEED, 5, 3, n)
        for p in (O.Params(), O.Params(min_len=0, max_len=100, pred_mask=0xF), O.Params(min_len=2047, pred_mask=0x7FF),
                  O.Params(min_cmp=O.MIN_GE, hash_algo=O.MD5), O.Params(hash_algo=O.SHA256_160, window=32)):
            got, exp = O.chunk_fast(data, p), O.chunk(data, p)
            for x, y in zip(got, exp):
                assert np.array_equal(x, y), (n, p)
    z = np.zeros(262144, np.uint8)
    assert np.array_equal(O.chunk_fast(z)[1], O.chunk(z)[1])


def test_divisor_detector_power_of_two_is_the_mask_and_others_differ():
    """fp >= 0, so fp % 2^k == R is (fp & (2^k-1)) == R (the engine runs it as the mask); a divisor
    that is not a power of two picks other boundaries; C loop == Python loop for the divisor form."""
    data = O.synth(O.SYNTH_SEED, 4321, 0, 200000).tobytes()
    for k, r in ((12, 0), (12, 4095), (13, 77)):
        a = O.chunk(data, O.Params(pred_kind=O.PRED_DIV, pred_div=1 << k, pred_rem=r))
        b = O.chunk(data, O.Params(pred_mask=(1 << k) - 1, pred_value=r))
        assert a[0].tolist() == b[0].tolist() and a[1].tolist() == b[1].tolist()
    p = O.Params(pred_kind=O.PRED_DIV, pred_div=4099, pred_rem=7)
    st, ln, dg = O.chunk(data, p)
    assert st.tolist() != O.chunk(data)[0].tolist()
    ref = O.py_chunk(data[:60000], p)
    st2, ln2, dg2 = O.chunk(data[:60000], p)
    assert [(int(a), int(b), d.tobytes()) for a, b, d in zip(st2, ln2, dg2)] == ref
    # Java long remainder of the (non-negative) window fp: the candidates are exactly the positions
    # whose definitional GF(2) fingerprint leaves remainder R
    fps = O.window_fps(data[:5000])
    for k in range(0, 5000, 97):
        fp = O.gf2_window_fp(data, k)
        assert int(fps[k]) == fp and p.is_boundary(fp) == (fp % 4099 == 7)


def test_java_parity_harness_generates_the_fixture_inputs():
    """tools/java/JarParity.java (run where a JDK and the jar exist) must rebuild cdc.json's inputs
    with the same generator: its SplitMix64 constants, stream key and default seed are the oracle's,
    and it knows every input kind make_golden.py uses."""
    import os
    src = open(os.path.join(os.path.dirname(G.GOLDEN), "..", "tools", "java", "JarParity.java")).read()
    for const in ("0x9E3779B97F4A7C15L", "0xBF58476D1CE4E5B9L", "0x94D049BB133111EBL", "0xD1B54A32D192ED03L",
                  "0x5DF50001L", ">>> 30", ">>> 27", ">>> 31"):
        assert const in src, const
    kinds = {fx["input"]["kind"] for fx in G.fixtures()}
    for k in kinds:
        assert f'case "{k}"' in src, k
    assert O.SYNTH_SEED == 0x5DF50001 and G.load("cdc.json")["seed"] == O.SYNTH_SEED
