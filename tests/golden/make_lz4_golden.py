"""Regenerate tests/golden/lz4.json — committed fixtures for the LZ4 parity tests.

    python tests/golden/make_lz4_golden.py

Every fixture is an input spec (counter-based generator, no stored bytes) with the SHA-256 of the
input and, per mode, the length and SHA-256 of the oracle's LZ4 block (oracle/lz4_ref.c).  The
V19 blocks are asserted here to equal the image's liblz4 1.9.x LZ4_compress_default output byte
for byte; the R123 blocks (lz4-java 1.3.0's bundled r123, the reference) are asserted to decode
back to the input with both the oracle's decoder and liblz4's LZ4_decompress_safe.
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import lz4_oracle as Z  # noqa: E402
from tests.golden.make_golden import make_input as cdc_input  # noqa: E402

SEED = 0x5DF50001
LENGTHS = [0, 1, 4, 12, 13, 14, 16, 100, 4095, 4096, 8191, 32768, 65535, 65546, 65547, 100003, 131072]
KINDS = ["synth", "zeros", "fill", "ramp", "text", "mixed"]


def make_input(spec: dict) -> bytes:
    kind, n = spec["kind"], spec["len"]
    if kind == "text":
        return Z.text_like(SEED, spec["stream"], n).tobytes()
    if kind == "mixed":
        return Z.mixed(SEED, spec["stream"], n).tobytes()
    return cdc_input(spec)


def specs():
    out = []
    for ki, kind in enumerate(KINDS):
        for li, n in enumerate(LENGTHS):
            s = dict(kind=kind, len=n, stream=100 + 31 * ki + li)
            if kind == "fill":
                s["byte"] = 0xA5
            out.append(s)
    return out


def main() -> None:
    assert Z.system_lz4() is not None, "the image's liblz4 is needed to pin the V19 mode"
    fixtures = []
    for spec in specs():
        data = make_input(spec)
        n = len(data)
        rec = dict(input=spec, input_sha256=hashlib.sha256(data).hexdigest())
        for name, mode in Z.MODES.items():
            blk = Z.compress(data, mode)
            assert Z.decompress(blk, n) == data and Z.system_decompress(blk, n) == data
            if mode == Z.V19:
                assert blk == Z.system_compress(data), spec
            rec[name] = dict(len=len(blk), sha256=hashlib.sha256(blk).hexdigest())
            if len(blk) <= 64:
                rec[name]["hex"] = blk.hex()
        fixtures.append(rec)
        print(f"{spec['kind']:6s} {n:7d} -> r123 {rec['r123']['len']:7d}  v19 {rec['v19']['len']:7d}")
    with open(os.path.join(HERE, "lz4.json"), "w") as f:
        json.dump(dict(note="oracle/lz4_ref.c blocks; v19 == liblz4 1.9.x LZ4_compress_default (asserted when "
                            "generated); r123 = lz4-java 1.3.0's bundled LZ4 r123 rules (two rules unpinned)",
                       liblz4_version=Z.system_lz4().LZ4_versionNumber(), fixtures=fixtures), f, indent=0)


if __name__ == "__main__":
    main()
