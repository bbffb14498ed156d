#!/bin/bash
# Round 3: PMC of the production scan against its no-LDS ablation (sweep variant 35), plus the
# instruction-cache counters, one-stream bench runs of the tuning library (4 KiB-mean mix).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/scanpmc
mkdir -p $OUT
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/list_avail.txt 2>&1
grep -o -E "SQC?_[A-Z0-9_]*(ICACHE|IFETCH|INST_LEVEL|WAIT|LEVEL_WAVES|INSTS_SALU|ACTIVE)[A-Z0-9_]*" $OUT/list_avail.txt | sort -u > $OUT/counters_of_interest.txt
B="python3 bench.py --steps 4 --warmup 1 --threads= --other-mix 0 --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0 --streams-in-flight 1 --ramp-secs 0"
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
run() {  # name variant counters...
  local name=$1 v=$2; shift 2
  SDFS_SCAN_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -- $B > "$OUT/$name.log" 2>&1
}
run prod_wait 0 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA || exit 2
run nolds_wait 35 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_ACTIVE_INST_SCA || exit 3
run prod_ic 0 SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQ_IFETCH || echo "icache pass failed"
run prod_lvl 0 SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVES || echo "level pass failed"
echo done
