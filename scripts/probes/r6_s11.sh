#!/bin/bash
# Round 6, GPU session 11: LZ4 lane kernel on text with fewer chains in flight (SDFS_LZ4_LANE_GRID
# caps the 256-lane workgroups: 32 -> 8 192 lanes, 256 MiB of tables, Infinity-Cache sized) —
# does a cache-resident table set beat more chains with tables in HBM?  Tuning library.
set -o pipefail
O=gpurun_out/r6s11
mkdir -p $O
TL=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
for g in 32 64 128 256 512 0; do
  SDFS_CDC_LIB=$TL SDFS_LZ4_LANE_GRID=$g SETS=text MODES=r123 CPU_SECS=0.5 REPS=3 timeout -k 10 300 python -u scripts/lz4_bench.py \
    | sed "s/^{/{\"lane_grid\": $g, /" >> $O/lz4_lane_grid.jsonl 2>> $O/lz4.err || exit 1
  echo "grid $g ok"
done
