#!/bin/bash
# Round 5: scan segment length of small batches (queue passes), 512 (production) vs 256 bytes
# (tuning, SDFS_SMALL_SEG_LEN): GPU parity tests at 256, then the single-call breakdown of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
T=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
bash scripts/gpu_session.sh \
  "tests256:600:SDFS_CDC_LIB=$T SDFS_SMALL_SEG_LEN=256 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_divisor.py -x -q --timeout 150 --timeout-method thread" \
  "single512:200:SDFS_CDC_LIB=$T python3 scripts/single_call_probe.py > gpurun_out/single512.jsonl" \
  "single256:200:SDFS_CDC_LIB=$T SDFS_SMALL_SEG_LEN=256 python3 scripts/single_call_probe.py > gpurun_out/single256.jsonl" \
  "q512:200:SDFS_CDC_LIB=$T MODE=fill MASK_BITS=11 MIN_SEG_KIB=2 THREADS=1,8,48 python3 scripts/queue_probe.py > gpurun_out/q512.jsonl" \
  "q256:200:SDFS_CDC_LIB=$T SDFS_SMALL_SEG_LEN=256 MODE=fill MASK_BITS=11 MIN_SEG_KIB=2 THREADS=1,8,48 python3 scripts/queue_probe.py > gpurun_out/q256.jsonl"
