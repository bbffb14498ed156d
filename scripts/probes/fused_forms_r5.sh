#!/bin/bash
# Round 5: the fused scan + fingerprint kernel's forms 5-7 (scan items at issue priority 2) beside
# production and the best round-4 form (2), 4 KiB-mean mix, one process (scripts/ab.py): the
# fused kernel's duration is `chunk_hash` of the SDFS_FUSED_PROBE configs (it re-runs the batch's
# scan and then fingerprints), to compare with production's cdc_scan + chunk_hash.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;f2:SDFS_FUSED_PROBE=2;f5:SDFS_FUSED_PROBE=5;f6:SDFS_FUSED_PROBE=6;f7:SDFS_FUSED_PROBE=7'
CONFIGS="$C" ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py
