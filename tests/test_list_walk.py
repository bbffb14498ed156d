"""The scan epilogue's list cut walk (cdc_device.h: resolve_from_list, production for uniform
256 KiB buffers since round 4), restated phase for phase in Python and checked against the greedy
walk (oracle.cdc_oracle.resolve_from_candidates) on CPU:

  1. the lanes' candidates (<= kSumCands = 8 per 4 KiB segment) in one ascending list at the
     prefix of the lanes' counts;
  2. every entry's next-cut pointer from the segment T holding pos + 1 + first_off: T's list base
     plus its entries below that bound (the entry after T's last is the next segment's first);
  3. the pointer chase from the first cut;
  4. chunk = previous cut + 1 .. cut, then the tail;

and its refusals (summary overflow, > kListCap = 256 candidates, a forced cut before the tail), on
which the queue walk resolves the buffer instead.  The GPU code itself is checked against the
oracle by tests/test_gpu_parity.py::test_fused_list_walk_edges."""
import numpy as np
import pytest

from oracle import cdc_oracle as O

SUM_CANDS = 8   # kSumCands
LIST_CAP = 256  # kListCap
SEG = 4096      # the production scan segment; 64 segments per 256 KiB buffer


def first_off(p_):
    return p_.min_len if p_.min_cmp == O.MIN_GT else max(p_.min_len - 1, 0)


def list_walk(pos, n, p_, seg=SEG):
    """resolve_from_list: list of (start, len), or None where the GPU declines."""
    fo = first_off(p_)
    lanes = (n + seg - 1) // seg
    per_lane = [pos[(pos >= l * seg) & (pos < (l + 1) * seg)] for l in range(lanes)]
    counts = np.array([len(c) for c in per_lane])
    if (counts > SUM_CANDS).any() or seg & (seg - 1):
        return None
    base = np.concatenate([[0], np.cumsum(counts)[:-1]])
    total = int(counts.sum())
    if total > LIST_CAP:
        return None
    lst = np.concatenate(per_lane) if total else np.zeros(0, np.int64)  # phase 1
    nxt = [None] * total
    for e in range(total):  # phase 2
        p = int(lst[e])
        lo, hi = p + 1 + fo, min(p + p_.max_len, n - 1)
        if lo > hi:
            continue
        t = lo // seg
        tb, tn = int(base[t]), int(counts[t])
        window = lst[tb:tb + tn + 1]  # the segment's entries and the one after them
        less = int((window < lo).sum())
        f = tb + less
        if f < total and lst[f] <= hi:
            nxt[e] = f
    first = int((lst < fo).sum())  # phase 3
    idx = first if first < total and lst[first] <= min(p_.max_len - 1, n - 1) else None
    cuts = []
    while idx is not None:
        cuts.append(int(lst[idx]))
        idx = nxt[idx]
    start = cuts[-1] + 1 if cuts else 0
    if start < n and start + p_.max_len - 1 < n - 1:
        return None  # a forced cut: the queue walk's case
    out, prev = [], 0  # phase 4
    for c in cuts:
        out.append((prev, c + 1 - prev))
        prev = c + 1
    if start < n:
        out.append((start, n - start))
    return out


def greedy(pos, n, p_):
    cand = np.zeros(n, bool)
    cand[pos] = True
    return [tuple(x) for x in O.resolve_from_candidates(cand, n, p_)]


def candidates(data, p_):
    fp = O.window_fps(data, p_.poly, p_.window)
    return np.flatnonzero(p_.is_boundary(fp)).astype(np.int64)


@pytest.mark.parametrize("min_len,max_len,mask", [
    (4095, 32768, 0xFFF),    # the reference default
    (2047, 32768, 0x7FF),    # the metric's 4 KiB-mean mix
    (10239, 65536, 0x7FF),   # minLen reaches several segments ahead
    (511, 6000, 0x3FF),      # ~256 candidates per buffer: at or over the list's capacity
    (2047, 8192, 0x1FFF),    # max_len cuts at non-candidates in most buffers
])
def test_list_walk_equals_greedy_or_declines(min_len, max_len, mask):
    p_ = O.Params(min_len=min_len, max_len=max_len, pred_mask=mask)
    n = 1 << 18
    taken = 0
    for s in range(12):
        data = O.synth(O.SYNTH_SEED, 5000 + s, 0, n)
        pos = candidates(data, p_)
        got = list_walk(pos, n, p_)
        ref = greedy(pos, n, p_)
        if got is None:
            counts = np.bincount(pos // SEG, minlength=n // SEG)
            forced = any(ln == max_len and (st + ln - 1) not in set(pos.tolist()) for st, ln in ref[:-1])
            assert (counts > SUM_CANDS).any() or len(pos) > LIST_CAP or forced
        else:
            taken += 1
            assert got == ref
    if mask in (0xFFF, 0x7FF) and min_len < 10000:
        assert taken >= 10, "random data at the reference's predicates: the list walk is the common case"


def test_edges_last_byte_cut_empty_and_tail_only():
    p_ = O.Params(min_len=2047, max_len=32768, pred_mask=0x7FF)
    n = 1 << 18
    # a cut at the last byte: no tail chunk
    pos = np.array([3000, 9000, n - 1], np.int64)
    with_last = list_walk(pos, n, p_)
    assert with_last is None or with_last == greedy(pos, n, p_)
    # no candidates at all: max_len forced cuts -> declined (the queue walk's case)
    assert list_walk(np.zeros(0, np.int64), n, p_) is None
    # a short buffer without candidates is one tail chunk
    assert list_walk(np.zeros(0, np.int64), 20000, p_) == [(0, 20000)]
    # candidates closer than minLen are skipped by the pointers
    pos = np.arange(0, n, 1500, dtype=np.int64)
    got = list_walk(pos, n, p_)
    assert got is not None and got == greedy(pos, n, p_)


def test_overflow_and_capacity_decline():
    p_ = O.Params(min_len=2047, max_len=32768, pred_mask=0x7FF)
    n = 1 << 18
    dense = np.arange(100, 100 + 9, dtype=np.int64)  # nine candidates in one segment
    assert list_walk(dense, n, p_) is None
    spread = np.arange(0, n, n // 257, dtype=np.int64)[:257]  # 257 candidates, <= 8 per segment
    assert list_walk(spread, n, p_) is None
    ok = spread[:256]
    got = list_walk(ok, n, p_)
    assert got is None or got == greedy(ok, n, p_)


def test_constants_match_the_kernel_header():
    """The restatement's capacities are the kernel's (cdc_device.h)."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(__file__), "..", "sdfs_amd", "csrc", "cdc_device.h")).read()
    assert int(re.search(r"constexpr uint32_t kListCap = (\d+);", src).group(1)) == LIST_CAP
    assert int(re.search(r"constexpr uint32_t kSumCands = (\d+);", src).group(1)) == SUM_CANDS
