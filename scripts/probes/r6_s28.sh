#!/bin/bash
# Round 6, GPU session 28: the final tree's synchronous-caller table: JNI fill
# entry at 1/8/48/128 callers, 150 calls each, both mixes, two runs; the 1-thread CPU restatement
# at both mixes on the same host.
set -o pipefail
O=gpurun_out/r6s28
mkdir -p $O
timeout -k 10 120 python -u -c '
import json, bench
for mb, ml in ((11, 2047), (12, 4095)):
    r = bench.cpu_baseline(4, 1, dict(min_len=ml, pred_mask=(1 << mb) - 1))
    print(json.dumps({"mask_bits": mb, **r}))
' > $O/cpu_1t.jsonl 2> $O/cpu.err || exit 1
for rep in 1 2; do
  for mb in 12 11; do
    MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1,8,48,128 CALLS_PER_THREAD=150 \
      timeout -k 10 240 python -u scripts/queue_probe.py >> $O/callers.jsonl 2>> $O/err.log || exit 1
  done
done
echo done
