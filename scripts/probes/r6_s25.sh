#!/bin/bash
# Round 6, GPU session 25: per-buffer latency-form groups (SDFS_SPLIT_BYBUF) A/B on the final
# queue (notifications outside the lock), 48/128 callers, both mixes, 150 calls per thread.
set -o pipefail
O=gpurun_out/r6s25
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for rep in 1 2 3; do
  for mb in 12 11; do
    for bb in 0 1; do
      SDFS_SPLIT_BYBUF=$bb MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1,48,128 CALLS_PER_THREAD=150 SDFS_CDC_LIB=$TL \
        timeout -k 10 240 python -u scripts/queue_probe.py | sed "s/^{/{\"bybuf\": $bb, /" >> $O/bybuf.jsonl 2>> $O/err.log || exit 1
    done
    echo "rep $rep mix $mb ok"
  done
done
