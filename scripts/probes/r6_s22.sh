#!/bin/bash
# Round 6, GPU session 22: 100 s queue soak on the final tree (every-lane latency form,
# per-request wakeups), every result checked.
set -o pipefail
O=gpurun_out/r6s22
mkdir -p $O
SOAK_SECS=100 timeout -k 10 300 python -u scripts/queue_soak.py > $O/soak_final.jsonl 2> $O/soak.err || exit 1
tail -3 $O/soak_final.jsonl
