#!/bin/bash
# Round 6, GPU session 7: the coalescing queue's soak with early completion (every result checked
# against the batch path and hashlib), and three batches in flight against two with the
# work-queue scan (interleaved, 4 KiB mix).
set -o pipefail
O=gpurun_out/r6s7
mkdir -p $O
SOAK_SECS=100 timeout -k 10 300 python -u scripts/queue_soak.py > $O/soak.jsonl 2> $O/soak.err &&
echo "soak ok" &&
for rep in 1 2 3; do
  for sif in 2 3; do
    timeout -k 10 180 python -u bench.py --steps 30 --warmup 3 --cpu-secs 0 --e2e-mib 0 --threads= --other-mix 0 --compare 0 \
      --streams-in-flight $sif >> $O/sif_ab.jsonl 2>> $O/sif.err || exit 1
  done
done &&
echo "sif ok"
