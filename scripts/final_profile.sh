#!/bin/bash
# Round-end evidence for the production kernels: smoke, rocprofv3 kernel-trace stats of the
# default-workload bench (the bench's own HIP-event times in the same run for comparison), and the
# PMC passes of scripts/pmc_scan.sh.  Everything lands in gpurun_out/final/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out/final
export TMPDIR=/tmp
BENCH_ABS="python3 $R/bench.py --steps 20 --warmup 3 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
bash scripts/gpu_session.sh \
  "smoke:180:python3 -c 'import __graft_entry__ as g; g.smoke()'" \
  "prof:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final/prof -- $BENCH_ABS > $R/gpurun_out/final/bench_under_rocprof.log 2>&1" \
  "pmc:600:bash scripts/pmc_scan.sh gpurun_out/final/pmc"
