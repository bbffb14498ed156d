#!/bin/bash
# Round 6, GPU session 6: the queue's dispatch threshold (a slot goes once it holds active callers /
# (lanes x SDFS_Q_SHARE_DIV)) and linger, with early completion and six lanes, JNI fill entry.
set -o pipefail
O=gpurun_out/r6s6
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for rep in 1 2; do
  for mb in 11 12; do
    for cfg in "1 250" "2 250" "4 250" "2 100"; do
      set -- $cfg
      MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=8,48,128 SDFS_CDC_LIB=$TL SDFS_Q_SHARE_DIV=$1 SDFS_Q_LINGER_US=$2 \
        timeout -k 10 240 python -u scripts/queue_probe.py | sed "s/^{/{\"share_div\": $1, \"linger\": $2, /" >> $O/queue_share.jsonl 2>> $O/queue.err || exit 1
    done
    echo "rep $rep mix $mb ok"
  done
done
