#!/bin/bash
# Round-4 end evidence on the committed tree (both chunk mixes): one-stream roofline runs and
# two-stream timed-region runs under rocprofv3 kernel-trace stats, the PMC passes of
# scripts/pmc_scan.sh, and a clock pass (kernel trace + GRBM_GUI_ACTIVE / SQ_INSTS_VALU in one
# run: per-kernel cycles beside per-kernel durations, so VALU utilisation and the clock come from
# the same launches).  Output: gpurun_out/r4end_<mix>/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
cd "$R" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/r4end_mix4k gpurun_out/r4end_mixdef
Q="--warmup 3 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
DEF="--min-seg-kib 4 --mask-bits 12"
RP="rocprofv3 --kernel-trace --stats --output-format csv"
CLK="rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv"
O=$R/gpurun_out
bash scripts/gpu_session.sh \
  "roof4k:240:cd /tmp && $RP -d $O/r4end_mix4k/roof -- python3 $R/bench.py --steps 100 --streams-in-flight 1 $Q > $O/r4end_mix4k/bench_roof.log 2>&1" \
  "roofdef:240:cd /tmp && $RP -d $O/r4end_mixdef/roof -- python3 $R/bench.py --steps 100 --streams-in-flight 1 $Q $DEF > $O/r4end_mixdef/bench_roof.log 2>&1" \
  "timed4k:240:cd /tmp && $RP -d $O/r4end_mix4k/timed -- python3 $R/bench.py --steps 200 $Q > $O/r4end_mix4k/bench_timed.log 2>&1" \
  "timeddef:240:cd /tmp && $RP -d $O/r4end_mixdef/timed -- python3 $R/bench.py --steps 200 $Q $DEF > $O/r4end_mixdef/bench_timed.log 2>&1" \
  "clock4k:180:cd /tmp && timeout -s KILL 150 $CLK -d $O/r4end_mix4k/clock -- python3 $R/bench.py --steps 6 --warmup 2 --streams-in-flight 1 $Q > $O/r4end_mix4k/bench_clock.log 2>&1" \
  "clockdef:180:cd /tmp && timeout -s KILL 150 $CLK -d $O/r4end_mixdef/clock -- python3 $R/bench.py --steps 6 --warmup 2 --streams-in-flight 1 $Q $DEF > $O/r4end_mixdef/bench_clock.log 2>&1" \
  "pmc4k:400:bash scripts/pmc_scan.sh gpurun_out/r4end_mix4k/pmc" \
  "pmcdef:400:MIX_ARGS='$DEF' bash scripts/pmc_scan.sh gpurun_out/r4end_mixdef/pmc"
