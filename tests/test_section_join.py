"""The parallel stitch of long buffers' sectioned cut walk (cdc_kernels.hip: cdc_resolve_spec_kernel,
cdc_resolve_join_kernel, cdc_resolve_place_kernel, with cdc_resolve_stitch_kernel as the fallback),
restated step for step in Python and checked against the greedy walk
(oracle.cdc_oracle.resolve_from_candidates) on CPU: the join's induction (section
j's true entry is the first start section j-1's chain reaches past its end), the "passes through"
case, and which inputs must fall back to the sequential stitch.  The GPU kernels themselves are
checked against the oracle by tests/test_gpu_parity.py (sectioned and long-chunk tests)."""
import numpy as np
import pytest

from oracle import cdc_oracle as O

K_JOIN_EXTRA = 8  # kJoinExtra


def first_cand(pos, lo, hi):
    i = np.searchsorted(pos, lo)
    return int(pos[i]) if i < len(pos) and pos[i] <= hi else -1


def step(pos, p, n, p_):
    lo, forced = p + p_.min_len, p + p_.max_len - 1  # first_off = min_len for n > minLen
    hi = min(forced, n - 1)
    k = first_cand(pos, lo, hi) if lo <= hi else -1
    return (k if k >= 0 else hi) + 1


def spec(pos, n, sec, p_):
    """cdc_resolve_spec_kernel: per section, chunk starts from an assumed start at its first byte."""
    out = []
    for r0 in range(0, (n + sec - 1) // sec * sec, sec):
        if r0 >= n:
            out.append(([], n))
            continue
        r1, st, x = min(r0 + sec, n), [], r0
        while x < r1:
            st.append(x)
            x = step(pos, x, n, p_)
        out.append((st, x))
    return out


def join_place(pos, n, sec, p_):
    """cdc_resolve_join_kernel + cdc_resolve_place_kernel; None = the buffer needs the sequential
    stitch (some section's chains did not meet)."""
    sp = spec(pos, n, sec, p_)
    joins = []
    for j, (st, nxt) in enumerate(sp):
        r0 = j * sec
        if j == 0 or r0 >= n:
            joins.append((0, []))
            continue
        r1, p, extra = min(r0 + sec, n), sp[j - 1][1], []
        if p >= n:
            joins.append((len(st), []))
            continue
        while True:
            if p >= r1:
                m = len(st) if p == nxt else None
                break
            if p in st:
                m = st.index(p)
                break
            if len(extra) == K_JOIN_EXTRA:
                m = None
                break
            extra.append(p)
            p = step(pos, p, n, p_)
        if m is None:
            return None
        joins.append((m, extra))
    starts = []
    for (st, nxt), (m, extra) in zip(sp, joins):
        starts += extra + st[m:]
    return starts


def reference(pos, n, p_):
    cand = np.zeros(n, bool)
    cand[pos] = True
    return [s for s, _ in O.resolve_from_candidates(cand, n, p_)]


def candidates(data, p_):
    fp = O.window_fps(data, p_.poly, p_.window)
    return np.flatnonzero(p_.is_boundary(fp)).astype(np.int64)


@pytest.mark.parametrize("min_len,max_len,mask,sec", [
    (4095, 131072, 0xFFF, 1 << 20),   # backup profile, default sections
    (4095, 131072, 0xFFF, 1 << 18),   # shorter sections
    (2047, 32768, 0x7FF, 1 << 17),    # the 4 KiB-mean mix
    (4095, 131072, 0xFFFFFF, 1 << 18),  # forced 128 KiB cuts (a rare candidate shifts the phase)
    (4095, 131072, 0xFFFF, 1 << 18),  # 4 KiB .. 128 KiB chunks, frequent forced cuts
])
def test_join_place_equals_greedy_walk_on_random_data(min_len, max_len, mask, sec):
    p_ = O.Params(min_len=min_len, max_len=max_len, pred_mask=mask)
    for s in range(3):
        n = 5 * (1 << 20) + 17 * s
        data = O.synth(O.SYNTH_SEED, 4000 + s, 0, n)
        pos = candidates(data, p_)
        got = join_place(pos, n, sec, p_)
        if mask <= 0xFFF:
            assert got is not None, "random data at the reference's predicate: every section's chains meet"
        if got is not None:  # otherwise the sequential stitch walks this buffer
            assert got == reference(pos, n, p_)


def test_chains_that_never_meet_fall_back():
    """All-zero data: every position is a candidate, cuts every min_len + 1 bytes; when that does
    not divide the section length the speculative chains never meet the true one, so the join
    must refuse (the sequential stitch then walks the buffer) — never place a wrong list."""
    p_ = O.Params(min_len=2999, max_len=131072)
    n = 6 * (1 << 20) + 5
    pos = np.arange(n, dtype=np.int64)
    assert join_place(pos, n, 1 << 20, p_) is None
    # with min_len + 1 dividing the section length the chains coincide and the join places them
    p2 = O.Params(min_len=4095, max_len=131072)
    assert join_place(pos, n, 1 << 20, p2) == reference(pos, n, p2)


def test_pass_through_and_candidate_free_stretches():
    """Long candidate-free stretches (forced cuts that cross section ends) and a buffer tail shorter
    than a section: whatever the join returns equals the greedy walk."""
    p_ = O.Params(min_len=4095, max_len=131072)
    n = 4 * (1 << 20) + 3000
    data = O.synth(O.SYNTH_SEED, 4100, 0, n)
    pos = candidates(data, p_)
    keep = np.ones(len(pos), bool)
    for a, b in [(200_000, 330_000), (1_000_000, 1_100_000), (2_090_000, 2_250_000)]:
        keep &= ~((pos >= a) & (pos < b))
    pos = pos[keep]
    got = join_place(pos, n, 1 << 18, p_)
    if got is not None:
        assert got == reference(pos, n, p_)


def test_forced_cut_phase_shift_falls_back():
    """A forced cut whose phase differs from a section's speculative chain through a whole
    section (the 16-bit predicate's candidate-free stretches): the true chain passes the section
    end elsewhere than the speculative one, so the join refuses rather than guess."""
    p_ = O.Params(min_len=4095, max_len=131072, pred_mask=0xFFFF)
    n = 5 * (1 << 20) + 17
    data = O.synth(O.SYNTH_SEED, 4001, 0, n)
    pos = candidates(data, p_)
    assert join_place(pos, n, 1 << 18, p_) is None
