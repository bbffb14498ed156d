#!/bin/bash
# Round 6, GPU session 3: (a) the dynamic scan work queue against the static stride, interleaved,
# both mixes, no interference; (b) the exchange proxy's cost surface with the dynamic scan
# (record size, RCCL-like workgroup count, stream priority); (c) queue lanes with early
# completion; (d) the fingerprint's raw per-wave stamps.
set -o pipefail
O=gpurun_out/r6s3
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
Q="--steps 30 --warmup 3 --cpu-secs 0 --e2e-mib 0 --threads= --other-mix 0"
for rep in 1 2; do
  for mix in "--min-seg-kib 2 --mask-bits 11" "--min-seg-kib 4 --mask-bits 12"; do
    for dyn in 0 1; do
      SDFS_CDC_LIB=$TL SDFS_SCAN_DYN=$dyn timeout -k 10 180 python -u bench.py $Q $mix >> $O/dyn_ab.jsonl 2>> $O/dyn.err || exit 1
    done
  done
  echo "dyn A/B $rep ok"
done &&
for px in "--proxy-wgs 16" "--proxy-wgs 64" "--proxy-record-bytes 36" "--proxy-prio 1" "--proxy-wgs 32"; do
  SDFS_CDC_LIB=$TL SDFS_SCAN_DYN=1 timeout -k 10 180 python -u bench.py $Q --exchange-proxy 8 $px >> $O/proxy_dyn_surface.jsonl 2>> $O/proxy.err || exit 1
done &&
SDFS_CDC_LIB=$TL SDFS_SCAN_DYN=0 timeout -k 10 180 python -u bench.py $Q --exchange-proxy 8 --proxy-prio 1 >> $O/proxy_static_prio.jsonl 2>> $O/proxy.err &&
echo "proxy surface ok" &&
for mb in 12 11; do
  for qi in "1 6" "1 8" "0 8"; do
    set -- $qi
    MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=48,128 SDFS_CDC_LIB=$TL SDFS_Q_EARLY=$1 SDFS_Q_INFLIGHT=$2 \
      timeout -k 10 240 python -u scripts/queue_probe.py >> $O/queue_lanes.jsonl 2>> $O/queue.err || exit 1
  done
  echo "queue $mb ok"
done &&
STAMPS_OUT=$O/stamps_raw.npy SDFS_CDC_LIB=$TL timeout -k 10 240 python -u scripts/hash_stamps.py > $O/hash_stamps.json 2> $O/hash_stamps.err &&
echo "stamps ok"
