"""Shared loaders for the committed golden fixtures (tests/golden/, made by make_golden.py)."""
import hashlib
import json
import os

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
