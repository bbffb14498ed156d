#!/bin/bash
# Segment length of a lone queue pass's scan (tuning SDFS_TINY_SEG_LEN; production 256): parity
# of the small-batch tests at 128 on the tuning library, then one 256 KiB buffer per pass under a
# kernel trace at 256 / 192 / 128.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
bash scripts/gpu_session.sh \
  "par128:300:SDFS_CDC_LIB=$L SDFS_TINY_SEG_LEN=128 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k 'small_batch or queue or dense or concurrent'" \
  "t256:200:SDFS_CDC_LIB=$L SDFS_TINY_SEG_LEN=256 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_t256 -o t -- python3 scripts/single_call_probe.py" \
  "t192:200:SDFS_CDC_LIB=$L SDFS_TINY_SEG_LEN=192 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_t192 -o t -- python3 scripts/single_call_probe.py" \
  "t128:200:SDFS_CDC_LIB=$L SDFS_TINY_SEG_LEN=128 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_t128 -o t -- python3 scripts/single_call_probe.py"
