#!/bin/bash
# Round 6: where a coalescing-queue pass's time goes at 48 callers (4 KiB mix, JNI fill entry,
# early completion, 6 lanes) against a lone caller: rocprofv3 kernel + memory-copy trace of
# scripts/queue_probe.py; scripts/queue_pass_timeline.py summarises it per pass.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
mkdir -p gpurun_out/r6qt
cd /tmp && export TMPDIR=/tmp
MASK_BITS=11 MIN_SEG_KIB=2 MODE=fill THREADS=1,48 timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
  -d $R/gpurun_out/r6qt/trace -- python3 $R/scripts/queue_probe.py > $R/gpurun_out/r6qt/probe.jsonl 2> $R/gpurun_out/r6qt/probe.err
