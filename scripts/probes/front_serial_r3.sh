#!/bin/bash
# Round 3: with two batches in flight, a batch's scan waits for the previous batch's
# prefix/scatter (SDFS_FRONT_SERIAL=1, tuning library) vs production order; bench.py two-stream
# steps at both mixes, alternated twice, then a kernel trace of the serialized order.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
export TMPDIR=/tmp
export SDFS_CDC_LIB=$R/sdfs_amd/libsdfs_cdc_tuning.so
mkdir -p gpurun_out/front
T="--steps 60 --warmup 5 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
DEF="--min-seg-kib 4 --mask-bits 12"
bash scripts/gpu_session.sh \
  "off4k_a:120:python3 bench.py $T" \
  "on4k_a:120:SDFS_FRONT_SERIAL=1 python3 bench.py $T" \
  "offdef_a:120:python3 bench.py $T $DEF" \
  "ondef_a:120:SDFS_FRONT_SERIAL=1 python3 bench.py $T $DEF" \
  "off4k_b:120:python3 bench.py $T" \
  "on4k_b:120:SDFS_FRONT_SERIAL=1 python3 bench.py $T" \
  "offdef_b:120:python3 bench.py $T $DEF" \
  "ondef_b:120:SDFS_FRONT_SERIAL=1 python3 bench.py $T $DEF" \
  "profon:240:cd /tmp && SDFS_FRONT_SERIAL=1 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/front/prof -- python3 $R/bench.py $T --steps 200 > $R/gpurun_out/front/bench_under_rocprof.log 2>&1"
