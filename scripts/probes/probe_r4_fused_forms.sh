#!/bin/bash
# Round 4: the fused scan + fingerprint kernel with 1 / 2 / 3 scan-first waves per SIMD (forms
# 2 / 3 / 4; form 1 = two, interleaved) against production (scan + fingerprint kernels), and the
# fingerprint kernel's line re-fetch bound at the 4 KiB-mean mix (hash variant 10 reads every
# chunk from its start rounded down to 128 B: wrong digests, the traffic a fix could save).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;f1:SDFS_FUSED_PROBE=1;f2:SDFS_FUSED_PROBE=2;f3:SDFS_FUSED_PROBE=3;f4:SDFS_FUSED_PROBE=4'
H='prod:;aligned:SDFS_HASH_VARIANT=10'
bash scripts/gpu_session.sh \
 "fforms_4k:200:CONFIGS='$C' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "fforms_def:200:CONFIGS='$C' ROUNDS=8 python3 scripts/ab.py" \
 "hash_aligned_4k:200:CONFIGS='$H' ROUNDS=10 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py"
