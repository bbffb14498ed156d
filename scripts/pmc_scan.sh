#!/bin/bash
# PMC passes over the one-stream 4 GiB bench (BASELINE configs[1]): instruction mix and stall
# counters of cdc_scan / chunk_hash, HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes:
# gfx950 cannot collect both in one TCC pass).  Each pass is its own run under a time limit.
# usage: scripts/pmc_scan.sh OUTDIR   (PMC_CMD overrides the profiled command, e.g. the LZ4 bench)
set -o pipefail
OUT=${1:-gpurun_out/pmc}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
# MIX_ARGS picks the chunk mix (default: the bench's headline, the 4 KiB-mean mix; the reference
# default is "--min-seg-kib 4 --mask-bits 12")
B=${PMC_CMD:-"python3 bench.py --steps 6 --warmup 2 --threads= --other-mix 0 --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0 --streams-in-flight 1 --ramp-secs 0 ${MIX_ARGS:-}"}
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -- $B > "$OUT/$name.log" 2>&1
}
run insts SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE || exit 2
run stalls SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM || exit 3
run fetch FETCH_SIZE || exit 4
run write WRITE_SIZE || exit 5
echo pmc passes done
