#!/bin/bash
# rocprofv3 kernel-trace stats of a bench run whose launches are almost all timed two-stream
# steps (200 timed, 3 warmup, 10 breakdown, no clock ramp), so the summary's chunk_hash average is
# the figure bench.py's roofline divides by.  Output under gpurun_out/final_timed/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out/final_timed
export TMPDIR=/tmp
B="python3 $R/bench.py --steps 200 --warmup 3 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
bash scripts/gpu_session.sh \
  "proft:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/final_timed/prof -- $B > $R/gpurun_out/final_timed/bench_under_rocprof.log 2>&1"
