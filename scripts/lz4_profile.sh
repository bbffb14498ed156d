#!/bin/bash
# LZ4 of unique chunks, profiled: the kernel split (rocprofv3 --kernel-trace
# --stats) of scripts/lz4_bench.py on random (incompressible) and text-like chunks, then PMC passes
# (instruction mix / waits, FETCH_SIZE, WRITE_SIZE: one pass each) per data set, R123 mode.
# usage: scripts/lz4_profile.sh OUTDIR
set -o pipefail
OUT=${1:-gpurun_out/lz4prof}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export CPU_SECS=0 MODES=r123 NBUF=${NBUF:-4096}
for set in random text; do
  SETS=$set timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_$set" -- \
    python3 scripts/lz4_bench.py > "$OUT/trace_$set.jsonl" 2> "$OUT/trace_$set.err" || exit 2
  B="python3 scripts/lz4_bench.py"
  run() {  # name counters...
    local name=$1; shift
    SETS=$set timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/${name}_$set" -- $B > "$OUT/${name}_$set.log" 2>&1
  }
  run insts SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit 3
  run stalls SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM || exit 4
  run fetch FETCH_SIZE || exit 5
  run write WRITE_SIZE || exit 6
done
echo lz4 profile done
