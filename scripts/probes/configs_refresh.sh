#!/bin/bash
# BASELINE configs[2] (dedup) and configs[4] (backup slice) on the current kernels.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
  "cfg_dedup:240:CONFIG=dedup python scripts/config_bench.py" \
  "cfg_backup:240:CONFIG=backup python scripts/config_bench.py"
