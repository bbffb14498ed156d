#!/bin/bash
# Round 6, GPU session 16: latency form with every lane running every block (production) vs the
# masked form (SDFS_SPLIT_MASKED=1): stamps, parity of the small-batch paths, callers A/B.
set -o pipefail
O=gpurun_out/r6s16
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for mk in 1 0; do
  for mb in 11 12; do
    STAMPS_OUT=$PWD/$O/rows_masked$mk.jsonl MASK_BITS=$mb SDFS_CDC_LIB=$TL SDFS_SPLIT_MASKED=$mk timeout -k 10 300 python -u scripts/split_stamps.py \
      | sed "s/^{/{\"masked\": $mk, /" >> $O/split_stamps.jsonl 2>> $O/err.log || exit 1
  done
done
echo "stamps ok"
timeout -k 10 900 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_parity.py tests/test_jni.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo "tests ok"
for rep in 1 2; do
  for mb in 12 11; do
    for mk in 1 0; do
      MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1,8,48,128 SDFS_CDC_LIB=$TL SDFS_SPLIT_MASKED=$mk \
        timeout -k 10 240 python -u scripts/queue_probe.py | sed "s/^{/{\"masked\": $mk, /" >> $O/queue_masked.jsonl 2>> $O/queue.err || exit 1
    done
    echo "rep $rep mix $mb ok"
  done
done
