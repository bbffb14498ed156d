#!/bin/bash
# Round 6, GPU session 2: the one-GPU projection of the 8-rank exchange (paced proxy copy) with
# the static and the dynamic scan, the queue's early completion A/B (tuning library,
# SDFS_Q_EARLY=0/1, both mixes, JNI fill entry) and the fingerprint's clock / tail / load split.
set -o pipefail
O=gpurun_out/r6s2
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
Q="--steps 20 --warmup 3 --cpu-secs 0 --e2e-mib 0 --threads= --other-mix 0"
for px in 0 8; do
  timeout -k 10 180 python -u bench.py $Q --exchange-proxy $px >> $O/proxy_static.jsonl 2>> $O/proxy.err || exit 1
  SDFS_CDC_LIB=$TL SDFS_SCAN_DYN=1 timeout -k 10 180 python -u bench.py $Q --exchange-proxy $px >> $O/proxy_dyn.jsonl 2>> $O/proxy.err || exit 1
  echo "proxy $px ok"
done &&
for mb in 12 11; do
  for ea in 0 1; do
    MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1,8,48,128 SDFS_CDC_LIB=$TL SDFS_Q_EARLY=$ea \
      timeout -k 10 240 python -u scripts/queue_probe.py >> $O/queue_early.jsonl 2>> $O/queue.err || exit 1
    echo "queue $mb $ea ok"
  done
done &&
SDFS_CDC_LIB=$TL timeout -k 10 240 python -u scripts/hash_stamps.py > $O/hash_stamps.json 2> $O/hash_stamps.err &&
echo "stamps ok"
