#!/bin/bash
# Exchange cost at N = 1 through the driver's launch path (torch.distributed.run, RCCL), VERDICT
# round 1 item 4: bench.py without the exchange vs with it (snapshot-copy and direct-slot modes),
# interleaved REPS times; then one kernel trace of the direct mode (what RCCL adds per step).
# usage: scripts/exchange_ab.sh OUTDIR [REPS]
set -o pipefail
OUT=${1:-gpurun_out/exchange}
REPS=${2:-2}
mkdir -p "$OUT"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
X="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --other-mix 0 --compare 0 --steps 30 --warmup 5"
P=29611
for r in $(seq "$REPS"); do
  for mode in none copy direct; do
    P=$((P + 1))
    if [ "$mode" = none ]; then ex="--exchange 0"; else ex="--exchange 1 --exchange-mode $mode"; fi
    timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
      --master-port $P bench.py --gpus 1 $X $ex > "$OUT/$mode.$r.log" 2>&1 || exit 3
    grep '^{' "$OUT/$mode.$r.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps({'mode':'$mode','rep':$r,'value':d['value'],'ms_per_step':d['ms_per_step'],'chunk_hash_ms':d['kernels_ms']['chunk_hash'],'exchange':d['config']['exchange']}))" | tee -a "$OUT/ab.jsonl"
  done
done
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
MASTER_ADDR=127.0.0.1 MASTER_PORT=29690 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 120 \
  rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_direct" -- \
  python3 bench.py --gpus 1 $X --exchange 1 --exchange-mode direct > "$OUT/trace_direct.log" 2>&1 || exit 4
echo exchange a/b done
