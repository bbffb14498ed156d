#!/bin/bash
# Scan workgroup width vs co-residency with the fingerprint kernel (tuning library): a 512-thread
# scan workgroup leaves half of every SIMD's registers to the other batch's chunk_hash waves when
# two batches are in flight.  bench.py at each width, REPS interleaved rounds.
# usage: scripts/probes/scan_width_ab.sh OUTDIR [REPS] [WIDTHS]
# WIDTHS entries are W or W:HASH_VARIANT:HASH_WG_PER_CU (persistent fingerprint grids sized to
# leave the other half of each SIMD to the scan).
set -o pipefail
OUT=${1:-gpurun_out/scanwidth}
REPS=${2:-2}
WIDTHS=${3:-"1024 512"}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
X="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --other-mix 0 --steps 30 --warmup 5"
for r in $(seq "$REPS"); do
  for spec in $WIDTHS; do
    IFS=: read -r w hv wpc <<< "$spec"
    tag=$(echo "$spec" | tr ':' '_')
    SDFS_CDC_LIB=sdfs_amd/libsdfs_cdc_tuning.so SDFS_SCAN_MAX_BLOCK=$w SDFS_HASH_VARIANT=${hv:-0} \
      SDFS_HASH_WG_PER_CU=${wpc:-2} timeout -k 10 120 python bench.py $X > "$OUT/w$tag.$r.log" 2>&1 || exit 3
    grep '^{' "$OUT/w$tag.$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'spec':'$spec','rep':$r,'value':d['value'],'one_stream':d['one_stream']['value'],'scan_ms':d['kernels_ms']['cdc_scan'],'hash_ms_2s':d['kernels_ms']['chunk_hash'],'identical':d['config']['records_identical_across_streams']}))" | tee -a "$OUT/ab.jsonl"
  done
done
