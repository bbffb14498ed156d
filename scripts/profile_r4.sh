#!/bin/bash
# Round-4 evidence for both chunk mixes, on the committed tree:
#  * roofline runs: rocprofv3 kernel-trace stats of bench.py with ONE batch in flight, so every
#    4 GiB chunk_hash launch is stream-ordered like the launches bench.py's roofline divides by
#    (its one-stream timed region); the summary's chunk_hash average must agree with the line's
#    roofline.kernel_ms;
#  * timed-region runs: the production two-stream steps (what the stages cost inside the step);
#  * PMC passes (instruction mix, stalls, HBM traffic) of the one-stream bench.
# Output: gpurun_out/r4_<mix>/.  Usage: scripts/profile_r4.sh [pmc]
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4_mix4k gpurun_out/r4_mixdef
Q="--warmup 3 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
DEF="--min-seg-kib 4 --mask-bits 12"
RP="rocprofv3 --kernel-trace --stats --output-format csv"
steps=(
  "roof4k:240:cd /tmp && $RP -d $R/gpurun_out/r4_mix4k/roof -- python3 $R/bench.py --steps 100 --streams-in-flight 1 $Q > $R/gpurun_out/r4_mix4k/bench_roof.log 2>&1"
  "roofdef:240:cd /tmp && $RP -d $R/gpurun_out/r4_mixdef/roof -- python3 $R/bench.py --steps 100 --streams-in-flight 1 $Q $DEF > $R/gpurun_out/r4_mixdef/bench_roof.log 2>&1"
  "timed4k:240:cd /tmp && $RP -d $R/gpurun_out/r4_mix4k/timed -- python3 $R/bench.py --steps 200 $Q > $R/gpurun_out/r4_mix4k/bench_timed.log 2>&1"
  "timeddef:240:cd /tmp && $RP -d $R/gpurun_out/r4_mixdef/timed -- python3 $R/bench.py --steps 200 $Q $DEF > $R/gpurun_out/r4_mixdef/bench_timed.log 2>&1"
)
if [ "$1" = "pmc" ]; then
  steps+=("pmc4k:400:bash scripts/pmc_scan.sh gpurun_out/r4_mix4k/pmc"
          "pmcdef:400:MIX_ARGS='$DEF' bash scripts/pmc_scan.sh gpurun_out/r4_mixdef/pmc")
fi
bash scripts/gpu_session.sh "${steps[@]}"
