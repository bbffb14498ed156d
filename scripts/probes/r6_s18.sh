#!/bin/bash
# Round 6, GPU session 18: queue policy scan on the full-exec latency form at 48 / 128 callers,
# both mixes (tuning library): per-buffer groups, share divisor, lanes, linger; 150 calls per
# thread per point (the probe's default 8 is a few milliseconds: too noisy for an A/B).
set -o pipefail
O=gpurun_out/r6s18b
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
run() {  # label, env...
  local lab=$1; shift
  env "$@" MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=48,128 CALLS_PER_THREAD=150 SDFS_CDC_LIB=$TL \
    timeout -k 10 240 python -u scripts/queue_probe.py | sed "s/^{/{\"cfg\": \"$lab\", /" >> $O/policy.jsonl 2>> $O/queue.err
}
for rep in 1 2 3; do
  for mb in 12 11; do
    run base SDFS_SPLIT_BYBUF=0 || exit 1
    run masked SDFS_SPLIT_MASKED=1 || exit 1
    run bybuf SDFS_SPLIT_BYBUF=1 || exit 1
    run bybuf_sd2 SDFS_SPLIT_BYBUF=1 SDFS_Q_SHARE_DIV=2 || exit 1
    run bybuf_l8 SDFS_SPLIT_BYBUF=1 SDFS_Q_INFLIGHT=8 || exit 1
    run bybuf_lin100 SDFS_SPLIT_BYBUF=1 SDFS_Q_LINGER_US=100 || exit 1
    echo "rep $rep mix $mb ok"
  done
done
