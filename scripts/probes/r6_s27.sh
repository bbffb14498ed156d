#!/bin/bash
# Round 6, GPU session 27: 256 callers, 48 calls each, both mixes: rate, tail, CPU per call and the
# cgroup's throttling (the bench line's 256-caller point).
set -o pipefail
O=gpurun_out/r6s27
mkdir -p $O
for rep in 1 2; do
  for mb in 11 12; do
    MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=128,256 CALLS_PER_THREAD=48 \
      timeout -k 10 240 python -u scripts/queue_probe.py >> $O/t256.jsonl 2>> $O/err.log || exit 1
  done
done
echo done
