#!/bin/bash
# Interleaved A/B: production scan against sweep variant 32 (candidate bits from per-position
# SGPR compare masks, kAblSgprPred), at the default and the 4 KiB-mean mixes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
  "ab:300:CONFIGS='prod:;sgpr:SDFS_SCAN_VARIANT=32' ROUNDS=12 python scripts/ab.py" \
  "ab4k:300:CONFIGS='prod:;sgpr:SDFS_SCAN_VARIANT=32' ROUNDS=12 MIN_SEG_KIB=2 MASK_BITS=11 python scripts/ab.py"
