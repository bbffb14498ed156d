#!/bin/bash
# LZ4 wave kernel vs hybrid (lane pass + wave pass for bailed chunks) by batch size: where the
# hybrid starts to pay (tuning library; NBUF 256 KiB buffers of engine chunks per batch).
# usage: scripts/probes/lz4_batch_sweep.sh OUTDIR "NBUFS"
set -o pipefail
OUT=${1:-gpurun_out/lz4batch}
NBUFS=${2:-"16 64 256 1024 4096"}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=sdfs_amd/libsdfs_cdc_tuning.so SETS=${SETS:-random,text} CPU_SECS=0 MODES=r123
for nb in $NBUFS; do
  for lm in 0 2; do
    NBUF=$nb SDFS_LZ4_LANE=$lm timeout -k 10 120 python scripts/lz4_bench.py > "$OUT/n${nb}_l$lm.log" 2>&1 || exit 3
    grep -h '^{' "$OUT/n${nb}_l$lm.log" | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l)
    print(json.dumps({'nbuf': $nb, 'lane_mode': $lm, 'chunks': d['chunks'], 'data': d['data'], 'kernel_ms': d['kernel_ms'], 'gibps': d['gibps']}))" | tee -a "$OUT/sweep.jsonl"
  done
done
