#!/bin/bash
# Round 3: the push address as one SDWA shift (43), push + pop addresses as SDWA (44), 43 on
# whole-block batches (45), against production; then the remaining ablations of the production
# kernel (39-42); interleaved in one process (scripts/ab.py), both mixes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;sdwa:SDFS_SCAN_VARIANT=43;sdwa_pop:SDFS_SCAN_VARIANT=44;sdwa_full:SDFS_SCAN_VARIANT=45;c16w6:SDFS_SCAN_VARIANT=46;c16w5:SDFS_SCAN_VARIANT=47'
A='prod:;nocand:SDFS_SCAN_VARIANT=39;noload:SDFS_SCAN_VARIANT=40;noload_nocand:SDFS_SCAN_VARIANT=41;bare:SDFS_SCAN_VARIANT=42'
bash scripts/gpu_session.sh \
 "sdwa_4k:200:CONFIGS='$C' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "sdwa_def:200:CONFIGS='$C' ROUNDS=8 python3 scripts/ab.py" \
 "abl2_4k:200:CONFIGS='$A' ROUNDS=6 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py"
