#!/bin/bash
# Round 3: what else the production scan's time is made of: without the candidate test (39),
# without the global loads (40), without both (41), without loads, test and LDS reads (42: the
# bare rolling chain); interleaved in one process (scripts/ab.py), both mixes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;nocand:SDFS_SCAN_VARIANT=39;noload:SDFS_SCAN_VARIANT=40;noload_nocand:SDFS_SCAN_VARIANT=41;bare:SDFS_SCAN_VARIANT=42'
bash scripts/gpu_session.sh \
 "abl2_4k:200:CONFIGS='$C' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "abl2_def:200:CONFIGS='$C' ROUNDS=8 python3 scripts/ab.py"
