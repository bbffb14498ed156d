"""Shared loaders for the committed golden fixtures (tests/golden/, made by make_golden.py)."""
import bisect
import hashlib
import json
import os

import numpy as np

from oracle import cdc_oracle as O  # tests may use the oracle as the checker
from tests.golden.make_golden import make_input  # noqa: F401  (input generators)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def fixtures():
    return load("cdc.json")["fixtures"]


def fixture_input(fx) -> bytes:
    data = make_input(fx["input"])
    assert hashlib.sha256(data).hexdigest() == fx["input_sha256"], fx["name"]
    return data


def oracle_params(fx) -> "O.Params":
    return O.Params(**fx["params"])


def tar_bytes(layout, off: int, n: int) -> np.ndarray:
    """Stream bytes [off, off+n) of a tar-like layout (sdfs_amd.device.TarLayout), restated on the
    CPU with the oracle's synthetic generator."""
    out = np.zeros(n, np.uint8)
    starts = [pc[0] for pc in layout.pieces]
    i = max(bisect.bisect_right(starts, off) - 1, 0)
    while i < len(layout.pieces) and layout.pieces[i][0] < off + n:
        dst, ln, src = layout.pieces[i]
        lo, hi = max(dst, off), min(dst + ln, off + n)
        if src >= 0 and hi > lo:
            out[lo - off:hi - off] = O.synth(layout.seed, src, lo - dst, hi - lo)
        i += 1
    return out
