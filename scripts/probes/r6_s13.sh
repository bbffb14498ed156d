#!/bin/bash
# Round 6, GPU session 13: per-buffer latency-form groups with one group per CU (SDFS_SPLIT_BYBUF=1
# SDFS_SPLIT_SPREAD=1) against production, 1/8/48/128 callers, both mixes (tuning library).
set -o pipefail
O=gpurun_out/r6s13
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for rep in 1 2; do
  for mb in 12 11; do
    for bb in 0 1; do
      MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1,8,48,128 SDFS_CDC_LIB=$TL SDFS_SPLIT_BYBUF=$bb SDFS_SPLIT_SPREAD=$bb \
        timeout -k 10 240 python -u scripts/queue_probe.py | sed "s/^{/{\"bybuf_spread\": $bb, /" >> $O/queue_bybuf_spread.jsonl 2>> $O/queue.err || exit 1
    done
    echo "rep $rep mix $mb ok"
  done
done
