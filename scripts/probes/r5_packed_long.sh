#!/bin/bash
# Round 5: the packed latency form for long chunks (backup profile, chunk_hash_long_kernel): GPU
# tests, then the configs[4] slice (tar-like stream, maxLen 128 KiB) with the packed form
# (production) and the one-lane form (tuning, SDFS_SPLIT_PACKED=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
T=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
  "backup:300:CONFIG=backup python3 scripts/config_bench.py > gpurun_out/backup_packed.json" \
  "backup_onelane:300:SDFS_CDC_LIB=$T SDFS_SPLIT_PACKED=0 CONFIG=backup python3 scripts/config_bench.py > gpurun_out/backup_onelane.json"
