#!/bin/bash
# Round 6, GPU session 24 (admissions and launches notified outside the queue lock, then a soak): host CPU per getChunks call (callers / queue threads / runtime) at
# 1/8/48/128 callers, both mixes, production library, 150 calls per thread.
set -o pipefail
O=gpurun_out/r6s24
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue.py tests/test_gpu_share.py tests/test_jni.py -m gpu -x -v \
  --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo "tests ok"
for mb in 12 11; do
  MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1,8,48,128 CALLS_PER_THREAD=150 \
    timeout -k 10 300 python -u scripts/queue_probe.py >> $O/cpu.jsonl 2>> $O/err.log || exit 1
done
SOAK_SECS=100 timeout -k 10 300 python -u scripts/queue_soak.py > $O/soak.jsonl 2> $O/soak.err || exit 1
tail -1 $O/soak.jsonl
