#!/bin/bash
# Round-6 end, fourth pass (per-buffer latency-form groups on): GPU suite, smoke, the default bench line.
set -o pipefail
O=gpurun_out/r6end4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 180 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench_default.jsonl 2> $O/bench_default.err &&
echo "bench ok" &&
SOAK_SECS=60 timeout -k 10 200 python -u scripts/queue_soak.py > $O/soak.jsonl 2> $O/soak.err &&
tail -1 $O/soak.jsonl
