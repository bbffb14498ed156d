#!/bin/bash
# Issue priority for waves of long chunks (production) against none (hash sweep variant 31), with
# two batches in flight (tuning library), interleaved twice; default and 4 KiB-mean mixes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
Q="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
bash scripts/gpu_session.sh \
  "prio1:120:python bench.py $Q" \
  "noprio1:120:SDFS_HASH_VARIANT=31 python bench.py $Q" \
  "prio2:120:python bench.py $Q" \
  "noprio2:120:SDFS_HASH_VARIANT=31 python bench.py $Q"
