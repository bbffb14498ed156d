#!/bin/bash
# Small-batch cut walk: the chain of candidate cuts marked in parallel (pointer jumping,
# production) vs the serial list walk (tuning SDFS_SMALL_BALLOT=2): parity of the small-batch
# tests on the production library, then one 256 KiB buffer per pass under a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
L=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
K="small_batch or queue or dense or concurrent or divisor or ragged or empty"
bash scripts/gpu_session.sh \
  "par:300:python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_divisor.py -m gpu -x -q --timeout 150 --timeout-method thread -k '$K'" \
  "jump:200:SDFS_CDC_LIB=$L SDFS_SMALL_BALLOT=0 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_jump -o t -- python3 scripts/single_call_probe.py" \
  "serial:200:SDFS_CDC_LIB=$L SDFS_SMALL_BALLOT=2 REPS=32 rocprofv3 --kernel-trace -d gpurun_out/ab_serial -o t -- python3 scripts/single_call_probe.py"
