#!/bin/bash
# Round 6, GPU session 26: the default bench line with the longer caller sweep (48 calls per thread).
set -o pipefail
O=gpurun_out/r6s26
mkdir -p $O
timeout -k 10 600 python -u bench.py > $O/bench_default.jsonl 2> $O/bench_default.err && echo "bench ok"
