"""CPU tests of the configs[4] tar-like stream layout (sdfs_amd.device.tar_layout):
pieces tile the stream, members are 512-byte headers + bodies padded to 512, bodies are log-uniform
1 KiB-64 MiB, ~20 % repeat an earlier body byte for byte; and the oracle's restatement of the bytes
(tests/golden_util.tar_bytes) agrees with the layout."""
import numpy as np

from sdfs_amd.device import TAR_HEADER_STREAM, tar_layout
from tests import golden_util as G


def test_layout_tiles_the_stream_like_ustar():
    total = 409 * 40960 * 1024
    lay = tar_layout(total)
    assert lay == tar_layout(total)  # seeded: reproducible
    p = 0
    for dst, n, src in lay.pieces:
        assert dst == p and n > 0
        p += n
    assert p == total
    hdr = [pc for pc in lay.pieces if TAR_HEADER_STREAM <= pc[2] < 2 * TAR_HEADER_STREAM]
    assert all(n == 512 for _, n, _ in hdr[:-1]) and all(dst % 512 == 0 for dst, _, _ in hdr)
    lens = np.array([n for _, n, _ in lay.bodies[:-1]])
    assert lens.min() >= 1024 and lens.max() < (64 << 20)
    assert abs(np.median(np.log2(lens)) - 18) < 1.0  # log-uniform over [10, 26)
    frac = len(lay.repeats) / len(lay.bodies)
    assert 0.17 < frac < 0.23, frac
    src_of = {dst: src for dst, _, src in lay.bodies}
    for c, o, n in lay.repeats:
        assert src_of[c] == src_of[o] and o < c


def test_oracle_bytes_of_a_repeat_equal_its_original():
    lay = tar_layout(64 << 20, seed=11)
    assert lay.repeats
    for c, o, n in lay.repeats[:3]:
        k = min(n, 200000)
        assert (G.tar_bytes(lay, c, k) == G.tar_bytes(lay, o, k)).all()
    # header, body, padding of the first member
    first = G.tar_bytes(lay, 0, 4096)
    dst, n, src = lay.pieces[1]
    assert (first[512:512 + min(n, 3584)] == G.O.synth(lay.seed, src, 0, min(n, 3584))).all()
