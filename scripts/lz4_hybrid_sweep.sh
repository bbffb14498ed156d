#!/bin/bash
# LZ4 hybrid (lane pass, bailed chunks to the wave kernel) sweep: bail threshold x lane
# workgroups per CU, on random / text / mixed chunk sets (tuning library).
# usage: scripts/lz4_hybrid_sweep.sh OUTDIR "BAILS" "WPCS"
set -o pipefail
OUT=${1:-gpurun_out/lz4hyb}
BAILS=${2:-"96 128 192"}
WPCS=${3:-"1 2 4"}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export SDFS_CDC_LIB=sdfs_amd/libsdfs_cdc_tuning.so SETS=${SETS:-random,text,mixed} CPU_SECS=0 MODES=r123
for b in $BAILS; do
  for w in $WPCS; do
    SDFS_LZ4_LANE=2 SDFS_LZ4_BAIL=$b SDFS_LZ4_LANE_WG_PER_CU=$w timeout -k 10 120 \
      python scripts/lz4_bench.py > "$OUT/b${b}_w$w.log" 2>&1 || exit 3
    grep -h '^{' "$OUT/b${b}_w$w.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(json.dumps({'bail': $b, 'lane_wg_per_cu': $w, 'data': d['data'], 'kernel_ms': d['kernel_ms'], 'gibps': d['gibps']}))" | tee -a "$OUT/sweep.jsonl"
  done
done
