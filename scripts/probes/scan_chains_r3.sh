#!/bin/bash
# Round 3: two rolling chains per lane in the mirrored / SGPR-mask scan (more independent LDS
# round trips in flight per SIMD): 2 chains x 4 waves (variant 37, 128-B blocks, 128 VGPRs),
# 2 chains x 3 waves (38, 150 VGPRs) against production and its whole-blocks form (36).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;full:SDFS_SCAN_VARIANT=36;ch2w4:SDFS_SCAN_VARIANT=37;ch2w3:SDFS_SCAN_VARIANT=38'
bash scripts/gpu_session.sh \
 "ch4k:200:CONFIGS='$C' ROUNDS=10 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "chdef:200:CONFIGS='$C' ROUNDS=10 python3 scripts/ab.py"
