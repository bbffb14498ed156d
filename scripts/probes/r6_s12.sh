#!/bin/bash
# Round 6, GPU session 12: latency-form groups per buffer (split_bybuf) — parity of the small-batch
# paths on the production library, then A/B through the JNI fill entry at 1/8/48/128 callers, both
# mixes (tuning library, SDFS_SPLIT_BYBUF).
set -o pipefail
O=gpurun_out/r6s12
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_parity.py tests/test_jni.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo "tests ok"
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for rep in 1 2; do
  for mb in 12 11; do
    for bb in 0 1; do
      MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1,8,48,128 SDFS_CDC_LIB=$TL SDFS_SPLIT_BYBUF=$bb \
        timeout -k 10 240 python -u scripts/queue_probe.py | sed "s/^{/{\"bybuf\": $bb, /" >> $O/queue_bybuf.jsonl 2>> $O/queue.err || exit 1
    done
    echo "rep $rep mix $mb ok"
  done
done
