#!/bin/bash
# Small-batch cut walk A/B (cdc_resolve_small_kernel): candidate list + successor pointers vs
# 64-word ballots, one 256 KiB buffer per pass, kernel durations from the kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_session.sh \
  "list:200:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so SDFS_SMALL_BALLOT=0 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_list -o t -- python3 scripts/single_call_probe.py" \
  "ballot:200:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so SDFS_SMALL_BALLOT=1 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_ballot -o t -- python3 scripts/single_call_probe.py"
