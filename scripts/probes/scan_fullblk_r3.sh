#!/bin/bash
# Round 3: the production scan vs its whole-blocks form (sweep variant 36, kAblFullBlocks: no
# guarded load path in the block loop, so hipcc waits for the block's loads per 64 bytes instead of
# for all 16 at a control-flow merge); interleaved in one process (scripts/ab.py), both mixes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;full:SDFS_SCAN_VARIANT=36'
bash scripts/gpu_session.sh \
 "full4k:200:CONFIGS='$C' ROUNDS=10 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "fulldef:200:CONFIGS='$C' ROUNDS=10 python3 scripts/ab.py"
