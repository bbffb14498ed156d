#!/bin/bash
# Round 5: the bench's getChunks thread sweep is slower than scripts/queue_probe.py at equal thread
# counts; find which difference matters: probe in "fill" mode, then the bench's sweep alone under a
# kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
mkdir -p gpurun_out/qb2
MODE=fill MASK_BITS=11 MIN_SEG_KIB=2 THREADS=8,48 timeout -k 10 200 python3 scripts/queue_probe.py > gpurun_out/qb2/probe_fill.jsonl 2>gpurun_out/qb2/probe_fill.err || exit 2
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/qb2/trace -- \
  python3 $R/bench.py --steps 2 --warmup 1 --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0 --e2e-mib 0 --threads 8,48 > $R/gpurun_out/qb2/bench.log 2>&1
