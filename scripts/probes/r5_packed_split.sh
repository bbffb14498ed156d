#!/bin/bash
# Round 5: the packed latency form (two lanes per chunk): GPU tests, single-call breakdown, caller
# threads, and an interleaved-process A/B against the one-lane form (tuning, SDFS_SPLIT_PACKED=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
T=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
  "single:200:python3 scripts/single_call_probe.py > gpurun_out/single_call.jsonl" \
  "single_onelane:200:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=0 python3 scripts/single_call_probe.py > gpurun_out/single_call_onelane.jsonl" \
  "qprobe:200:MODE=fill MASK_BITS=11 MIN_SEG_KIB=2 THREADS=1,8,48,128 python3 scripts/queue_probe.py > gpurun_out/qprobe.jsonl" \
  "qprobe_onelane:200:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=0 MODE=fill MASK_BITS=11 MIN_SEG_KIB=2 THREADS=1,8,48,128 python3 scripts/queue_probe.py > gpurun_out/qprobe_onelane.jsonl"
