#!/bin/bash
# A/B on one box: the round-1 library (sdfs_amd/libsdfs_cdc_r01.so, built from d751c46) against
# the current one, interleaved, one-stream device path, same bench flags.
set -o pipefail
F="--steps 20 --warmup 5 --streams-in-flight 1 --threads= --other-mix 0 --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
for i in 1 2 3; do
  SDFS_CDC_LIB=sdfs_amd/libsdfs_cdc_r01.so timeout -k 10 120 python bench.py $F | python -c "import json,sys; d=json.load(sys.stdin); print('r01', d['value'], d['kernels_ms']['cdc_scan'], d['kernels_ms']['chunk_hash'],)" || exit 1
  timeout -k 10 120 python bench.py $F | python -c "import json,sys; d=json.load(sys.stdin); print('r02', d['value'], d['kernels_ms']['cdc_scan'], d['kernels_ms']['chunk_hash'],)" || exit 1
done
