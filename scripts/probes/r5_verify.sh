#!/bin/bash
# GPU tests, smoke, single-call breakdown and caller threads on the production library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
  "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "single:200:python3 scripts/single_call_probe.py > gpurun_out/single_call.jsonl" \
  "qprobe:200:MODE=fill MASK_BITS=11 MIN_SEG_KIB=2 THREADS=1,8,48,128 python3 scripts/queue_probe.py > gpurun_out/qprobe.jsonl"
