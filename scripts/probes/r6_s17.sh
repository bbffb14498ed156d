#!/bin/bash
# Round 6, GPU session 17: per-buffer latency-form groups (SDFS_SPLIT_BYBUF=1) on top of the
# full-exec latency form, 1/8/48/128 callers, both mixes (tuning library).
set -o pipefail
O=gpurun_out/r6s17
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for rep in 1 2 3; do
  for mb in 12 11; do
    for bb in 0 1; do
      MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1,8,48,128 SDFS_CDC_LIB=$TL SDFS_SPLIT_BYBUF=$bb \
        timeout -k 10 240 python -u scripts/queue_probe.py | sed "s/^{/{\"bybuf\": $bb, /" >> $O/queue_bybuf.jsonl 2>> $O/queue.err || exit 1
    done
    echo "rep $rep mix $mb ok"
  done
done
