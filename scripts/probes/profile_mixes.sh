#!/bin/bash
# Round-3 evidence for both chunk mixes: rocprofv3 kernel-trace stats of runs made of timed
# two-stream steps (the headline 4 KiB-mean mix, then the reference default), and the PMC passes
# (instruction mix, stalls, HBM traffic) of the one-stream bench for each mix.
# Output: gpurun_out/mix4k/, gpurun_out/mixdef/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/mix4k gpurun_out/mixdef
T="--steps 200 --warmup 3 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
DEF="--min-seg-kib 4 --mask-bits 12"
bash scripts/gpu_session.sh \
  "prof4k:240:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/mix4k/prof -- python3 $R/bench.py $T > $R/gpurun_out/mix4k/bench_under_rocprof.log 2>&1" \
  "profdef:240:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/mixdef/prof -- python3 $R/bench.py $T $DEF > $R/gpurun_out/mixdef/bench_under_rocprof.log 2>&1" \
  "pmc4k:400:bash scripts/pmc_scan.sh gpurun_out/mix4k/pmc" \
  "pmcdef:400:MIX_ARGS='$DEF' bash scripts/pmc_scan.sh gpurun_out/mixdef/pmc"
