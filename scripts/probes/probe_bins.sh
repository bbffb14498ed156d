#!/bin/bash
# Exact-count fingerprint binning (kMaxBins 1024: lanes of a wave hash chunks of identical block
# count) against the 512-bin build (two adjacent counts per bin), product builds, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
Q="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
O=$PWD/sdfs_amd/libsdfs_cdc_bins512.so
N=$PWD/sdfs_amd/libsdfs_cdc.so
bash scripts/gpu_session.sh \
  "b512a:120:SDFS_CDC_LIB=$O python bench.py $Q" \
  "b1024a:120:SDFS_CDC_LIB=$N python bench.py $Q" \
  "b512b:120:SDFS_CDC_LIB=$O python bench.py $Q" \
  "b1024b:120:SDFS_CDC_LIB=$N python bench.py $Q" \
  "b512c:120:SDFS_CDC_LIB=$O python bench.py $Q" \
  "b1024c:120:SDFS_CDC_LIB=$N python bench.py $Q"
