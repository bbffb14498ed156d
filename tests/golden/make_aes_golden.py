"""Regenerate tests/golden/aes.json — committed fixtures for the AES-CBC parity tests.

    python tests/golden/make_aes_golden.py

Every fixture is an input spec (counter-based generator, no stored bytes), a key, an IV and an
optional 4-byte big-endian prefix (the putChunk record's nz), with the length and SHA-256 of the
ciphertext (the full hex when short).  Each expected ciphertext is produced by the image's
``openssl enc -aes-N-cbc`` (an independent AES implementation, PKCS#7 padding) on
[prefix][input] and asserted equal to the oracle (oracle/aes_ref.c) here.
"""
from __future__ import annotations

import hashlib
import json
import os
import struct
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import aes_oracle as A  # noqa: E402
from oracle import cdc_oracle as C  # noqa: E402

SEED = 0x5DF50001
LENGTHS = [0, 1, 11, 12, 15, 16, 17, 31, 32, 100, 4095, 4096, 8191, 32768, 131072]


def make_input(spec: dict) -> bytes:
    return C.synth(SEED, spec["stream"], 0, spec["len"]).tobytes()


def specs():
    out = []
    k = 0
    for key_len in (32, 16, 24):
        for n in LENGTHS if key_len == 32 else LENGTHS[:8]:
            for prefix in (None, -1, 4096):
                if key_len != 32 and prefix == 4096:
                    continue
                key = C.synth(SEED ^ 0xAE5, 1000 + k, 0, key_len).tobytes()
                iv = C.synth(SEED ^ 0x1F, 2000 + k, 0, 16).tobytes()
                out.append({"stream": 10 + k, "len": n, "key": key.hex(), "iv": iv.hex(),
                            "prefix": prefix})
                k += 1
    # SDFS's own key derivation: SHA-256 of the passphrase (EncryptUtils.java:47-52)
    out.append({"stream": 999, "len": 5000, "key": A.key_from_passphrase("Password").hex(),
                "iv": "00" * 16, "prefix": -1, "passphrase": "Password"})
    return out


def main():
    fixtures = []
    for spec in specs():
        data = make_input(spec)
        key, iv = bytes.fromhex(spec["key"]), bytes.fromhex(spec["iv"])
        pre = b"" if spec["prefix"] is None else struct.pack(">i", spec["prefix"])
        ref = A.openssl_encrypt(key, iv, pre + data)
        assert ref is not None, "openssl is required to regenerate the fixtures"
        assert A.cbc_encrypt(key, iv, data, prefix=pre) == ref, spec
        assert A.cbc_decrypt(key, iv, ref) == pre + data
        f = dict(spec, input_sha256=hashlib.sha256(data).hexdigest(), out_len=len(ref),
                 out_sha256=hashlib.sha256(ref).hexdigest())
        if len(ref) <= 64:
            f["out_hex"] = ref.hex()
        fixtures.append(f)
    with open(os.path.join(HERE, "aes.json"), "w") as fh:
        json.dump({"seed": SEED, "generator": "openssl enc -aes-N-cbc (image), checked against oracle/aes_ref.c",
                   "fixtures": fixtures}, fh, indent=0)
    print(len(fixtures), "fixtures")


if __name__ == "__main__":
    main()
