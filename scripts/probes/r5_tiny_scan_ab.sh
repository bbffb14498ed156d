#!/bin/bash
# Tiny-batch scan (ScanTiny: 64-byte blocks, tuning SDFS_TINY_SCAN=1) at 64 / 128-byte segments
# against production (ScanProd, 256-byte segments): parity of the small-batch tests on the tuning
# library, then one 256 KiB buffer per pass under a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
K="small_batch or queue or dense or concurrent or divisor or ragged"
bash scripts/gpu_session.sh \
  "par64:300:SDFS_CDC_LIB=$L SDFS_TINY_SCAN=1 SDFS_TINY_SEG_LEN=64 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_divisor.py -m gpu -x -q --timeout 150 --timeout-method thread -k '$K'" \
  "par128:300:SDFS_CDC_LIB=$L SDFS_TINY_SCAN=1 SDFS_TINY_SEG_LEN=128 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread -k '$K'" \
  "p256:200:SDFS_CDC_LIB=$L REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_p256 -o t -- python3 scripts/single_call_probe.py" \
  "s64:200:SDFS_CDC_LIB=$L SDFS_TINY_SCAN=1 SDFS_TINY_SEG_LEN=64 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_s64 -o t -- python3 scripts/single_call_probe.py" \
  "s128:200:SDFS_CDC_LIB=$L SDFS_TINY_SCAN=1 SDFS_TINY_SEG_LEN=128 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_s128 -o t -- python3 scripts/single_call_probe.py"
