#!/bin/bash
# Round 5: coalescing-queue lanes 4 vs 8 (tuning library, SDFS_Q_INFLIGHT), T synchronous getChunks
# callers at the bench's 4 KiB-mean mix, then a kernel trace of the 8-lane run (do passes on
# streams that share a hardware queue overlap?).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
mkdir -p gpurun_out/qlanes
export SDFS_CDC_LIB=$R/sdfs_amd/libsdfs_cdc_tuning.so MASK_BITS=11 MIN_SEG_KIB=2
for qi in 4 8; do
  THREADS=1,8,48,128 SDFS_Q_INFLIGHT=$qi timeout -k 10 200 python3 scripts/queue_probe.py > gpurun_out/qlanes/qi$qi.jsonl 2> gpurun_out/qlanes/qi$qi.err || exit 2
done
cd /tmp && export TMPDIR=/tmp
THREADS=48 SDFS_Q_INFLIGHT=8 timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/qlanes/trace8 -- \
  python3 $R/scripts/queue_probe.py > $R/gpurun_out/qlanes/trace8.jsonl 2> $R/gpurun_out/qlanes/trace8.err
