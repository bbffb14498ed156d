#!/bin/bash
# Round 5: the DPP-bank pairing of the packed latency form (SDFS_SPLIT_PACKED=2, tuning) against
# the adjacent-lane pairing (1, production): parity tests at 2, single-call breakdowns, callers.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
T=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
bash scripts/gpu_session.sh \
  "tests2:600:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=2 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue.py tests/test_gpu_divisor.py -x -q --timeout 150 --timeout-method thread" \
  "single1:200:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=1 python3 scripts/single_call_probe.py > gpurun_out/single1.jsonl" \
  "single2:200:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=2 python3 scripts/single_call_probe.py > gpurun_out/single2.jsonl" \
  "single1b:200:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=1 python3 scripts/single_call_probe.py > gpurun_out/single1b.jsonl" \
  "single2b:200:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=2 python3 scripts/single_call_probe.py > gpurun_out/single2b.jsonl" \
  "backup2:300:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=2 CONFIG=backup python3 scripts/config_bench.py > gpurun_out/backup2.json" \
  "backup1:300:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=1 CONFIG=backup python3 scripts/config_bench.py > gpurun_out/backup1.json"
