#!/bin/bash
# Round 4: where chunk_hash's time above the register-only SHA-256 ceiling goes, at the 4 KiB-mean
# mix: production against sweep variant 1 (message words synthesized from the state: no loads)
# and variant 2 (loads kept, compression replaced by a fold: the cost of everything but SHA-256).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
bash scripts/gpu_session.sh \
 "hash_ablate_4k:200:CONFIGS='prod:;noload:SDFS_HASH_VARIANT=1;nocomp:SDFS_HASH_VARIANT=2' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py"
