#!/bin/bash
# Round 3: what the production scan's time is made of — the same kernel without its pop-table
# read, without its push-table read (no LDS round trip in the per-byte chain), without both;
# interleaved in one process (scripts/ab.py), at the 4 KiB-mean and the reference-default mix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;nopop:SDFS_SCAN_VARIANT=33;nopush:SDFS_SCAN_VARIANT=34;nolds:SDFS_SCAN_VARIANT=35'
bash scripts/gpu_session.sh \
 "abl4k:200:CONFIGS='$C' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "abldef:200:CONFIGS='$C' ROUNDS=8 python3 scripts/ab.py"
