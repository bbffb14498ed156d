#!/bin/bash
# Round 6, GPU session 14: kernel trace of lone-caller passes, latency-form groups longest-first
# (production) vs per buffer (SDFS_SPLIT_BYBUF=1), both mixes (tuning library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
mkdir -p gpurun_out/r6s14
cd /tmp && export TMPDIR=/tmp
for mb in 11 12; do
  for bb in 0 1; do
    MASK_BITS=$mb MIN_SEG_KIB=$((mb == 12 ? 4 : 2)) MODE=fill THREADS=1 SDFS_CDC_LIB=$R/sdfs_amd/libsdfs_cdc_tuning.so SDFS_SPLIT_BYBUF=$bb \
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $R/gpurun_out/r6s14/m${mb}_b${bb} -- python3 $R/scripts/queue_probe.py > $R/gpurun_out/r6s14/m${mb}_b${bb}.jsonl 2> $R/gpurun_out/r6s14/m${mb}_b${bb}.err || exit 1
    echo "mix $mb bybuf $bb ok"
  done
done
