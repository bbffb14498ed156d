#!/bin/bash
# Round 3: memory-pipeline counters of the production scan and fingerprint kernels (one-stream
# bench, 4 KiB-mean mix): L1 (TCP) accesses / L2 requests / stalls, address translation, TA.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/scanmem
mkdir -p $OUT
B="python3 bench.py --steps 4 --warmup 1 --threads= --other-mix 0 --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0 --streams-in-flight 1 --ramp-secs 0"
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -- $B > "$OUT/$name.log" 2>&1
}
run t1 TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum || exit 2
run t2 TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum || exit 3
run t3 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 4
run t4 TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum || exit 5
echo done
