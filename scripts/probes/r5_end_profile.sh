#!/bin/bash
# Round-5 end profiles of the production tree: rocprofv3 kernel stats of the one-stream bench (the
# roofline's chunk_hash launch time) and of the two-stream timed region, then the PMC passes
# (instruction mix / waits, FETCH_SIZE, WRITE_SIZE) at both chunk mixes.  Output: gpurun_out/end/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
mkdir -p gpurun_out/end
export TMPDIR=/tmp
B1="python3 $R/bench.py --steps 20 --warmup 3 --streams-in-flight 1 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
B2="python3 $R/bench.py --steps 200 --warmup 3 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
bash scripts/gpu_session.sh \
  "prof1:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/end/prof_one_stream -- $B1 > $R/gpurun_out/end/bench_one_stream.log 2>&1" \
  "prof2:300:cd /tmp && rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/end/prof_two_stream -- $B2 > $R/gpurun_out/end/bench_two_stream.log 2>&1" \
  "pmc4k:600:bash scripts/pmc_scan.sh gpurun_out/end/pmc_mix4k" \
  "pmcdef:600:MIX_ARGS='--min-seg-kib 4 --mask-bits 12' bash scripts/pmc_scan.sh gpurun_out/end/pmc_mixdef"
