#!/bin/bash
# Round 6, GPU session 10: the work-queue scan against the static stride on the backup profile's
# 40 MiB buffers (sectioned cut walk) and on configs[2], interleaved twice (tuning library).
set -o pipefail
O=gpurun_out/r6s10
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for rep in 1 2; do
  for dyn in 0 1; do
    for cfg in backup dedup; do
      SDFS_CDC_LIB=$TL SDFS_SCAN_DYN=$dyn CONFIG=$cfg STEPS=5 timeout -k 10 300 python -u scripts/config_bench.py | sed "s/^{/{\"scan_dyn\": $dyn, /" >> $O/configs_dyn_ab.jsonl 2>> $O/configs.err || exit 1
    done
  done
  echo "rep $rep ok"
done
