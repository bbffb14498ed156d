#!/bin/bash
# Round 5: which hardware queues the bench's two in-flight streams land on (kernel trace Queue_Id)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
mkdir -p gpurun_out/ts
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/ts/trace -- \
  python3 $R/bench.py --steps 10 --warmup 2 --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 1 --e2e-mib 0 --threads= > $R/gpurun_out/ts/bench.log 2>&1
