#!/bin/bash
# Round 4: what the fused cut walk in the scan's epilogue costs at each mix: production against
# the same scan without the walk (SDFS_SKIP_WALK=1: no chunk lists, measurement only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
bash scripts/gpu_session.sh \
 "walk_4k:200:CONFIGS='prod:;nowalk:SDFS_SKIP_WALK=1' ROUNDS=10 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "walk_def:200:CONFIGS='prod:;nowalk:SDFS_SKIP_WALK=1' ROUNDS=10 python3 scripts/ab.py"
