#!/bin/bash
# Round 5 (after the CU-masked lane streams): queue lanes 4 / 6 / 8 (tuning library,
# SDFS_Q_INFLIGHT), T synchronous getChunks callers at the 4 KiB-mean mix, JNI fill entry; then the
# new small-walk parity test.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out/qlanes
export MASK_BITS=11 MIN_SEG_KIB=2 MODE=fill
for qi in 4 6 8; do
  SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so THREADS=1,8,48,128 SDFS_Q_INFLIGHT=$qi timeout -k 10 200 python3 scripts/queue_probe.py > gpurun_out/qlanes/qi$qi.jsonl 2> gpurun_out/qlanes/qi$qi.err || exit 2
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "small_batch_walk or ragged or edge_lengths" -x -q --timeout 150 --timeout-method thread > gpurun_out/qlanes/tests.log 2>&1
