#!/bin/bash
# Round 5: why T synchronous getChunks callers get less than T x 256 KiB per single-call latency:
# the coalescing-queue probe (scripts/queue_probe.py) at 1 / 8 / 48 caller threads under a
# rocprofv3 kernel trace (per-kernel start/end, queue id, LDS size, grid), to see whether the
# passes of the four device lanes overlap on the GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
mkdir -p gpurun_out/qtrace
cd /tmp && export TMPDIR=/tmp
THREADS=${THREADS:-1,8,48} timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/qtrace/trace -- \
  python3 $R/scripts/queue_probe.py > $R/gpurun_out/qtrace/probe.jsonl 2> $R/gpurun_out/qtrace/probe.err
