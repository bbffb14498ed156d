#!/bin/bash
# Caller threads (JNI fill entry, 4 KiB mix) with and without the tiny-batch scan, interleaved,
# tuning library: gpurun_out/tiny_callers_{0,1}.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
L=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for r in 1 2; do
  for t in 0 1; do
    SDFS_CDC_LIB=$L SDFS_TINY_SCAN=$t MODE=fill MASK_BITS=11 MIN_SEG_KIB=2 THREADS=1,8,48,96 \
      timeout -k 10 200 python3 scripts/queue_probe.py >> gpurun_out/tiny_callers_$t.jsonl || exit 1
  done
done
