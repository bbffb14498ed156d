#!/bin/bash
# Round 5: LDS-staged small-batch cut walk (cdc_resolve_small_kernel): GPU tests, the single-call
# breakdown (scripts/single_call_probe.py) and the caller-thread probe at the 4 KiB mix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
  "single:200:python3 scripts/single_call_probe.py > gpurun_out/single_call.jsonl" \
  "qprobe:200:MASK_BITS=11 MIN_SEG_KIB=2 THREADS=1,8,48 python3 scripts/queue_probe.py > gpurun_out/qprobe.jsonl"
