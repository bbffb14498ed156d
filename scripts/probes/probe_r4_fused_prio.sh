#!/bin/bash
# Round 4: the fused scan + fingerprint kernel with the scan items at issue priority 2 (forms 5-7:
# 1 / 2 / 3 scan-first waves per SIMD) against form 2 and production, both mixes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;f2:SDFS_FUSED_PROBE=2;f5:SDFS_FUSED_PROBE=5;f6:SDFS_FUSED_PROBE=6;f7:SDFS_FUSED_PROBE=7'
bash scripts/gpu_session.sh \
 "fprio_4k:200:CONFIGS='$C' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "fprio_def:200:CONFIGS='$C' ROUNDS=8 python3 scripts/ab.py"
