#!/bin/bash
# Round 6, GPU session 15: latency-form stamps (scripts/split_stamps.py), both mixes.
set -o pipefail
O=gpurun_out/r6s15c
mkdir -p $O
for mb in 11 12; do
  STAMPS_OUT=$PWD/$O/rows.jsonl MASK_BITS=$mb SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so timeout -k 10 300 python -u scripts/split_stamps.py >> $O/split_stamps.jsonl 2>> $O/err.log || exit 1
done
cat $O/split_stamps.jsonl
