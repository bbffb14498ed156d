#!/bin/bash
# Co-residency of the next batch's scan with this batch's fingerprint kernel (two batches in
# flight, tuning library): 512-thread scan workgroups (2 waves/SIMD, SDFS_SCAN_MAX_BLOCK) and/or
# a fingerprint kernel whose 15 KiB of LDS per workgroup caps it at 2 waves/SIMD beside a scan
# workgroup (hash sweep variant 30).  Interleaved, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
Q="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --other-mix 0 --compare 0"
bash scripts/gpu_session.sh \
  "base1:120:python bench.py $Q" \
  "both1:120:SDFS_SCAN_MAX_BLOCK=512 SDFS_HASH_VARIANT=30 python bench.py $Q" \
  "s512:120:SDFS_SCAN_MAX_BLOCK=512 python bench.py $Q" \
  "pad:120:SDFS_HASH_VARIANT=30 python bench.py $Q" \
  "base2:120:python bench.py $Q" \
  "both2:120:SDFS_SCAN_MAX_BLOCK=512 SDFS_HASH_VARIANT=30 python bench.py $Q"
