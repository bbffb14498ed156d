#!/bin/bash
# Round 4: what the list walk's parts cost inside the scan (SDFS_SKIP_WALK, measurement only):
# nowalk = 1; compute = 2 (walk, no outputs); stores = 3 (chunk stores + LDS histogram, no
# counts, no global histogram flush); list = production.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C="list:;nowalk:SDFS_SKIP_WALK=1;compute:SDFS_SKIP_WALK=2;stores:SDFS_SKIP_WALK=3;queue:SDFS_LIST_WALK=0"
bash scripts/gpu_session.sh \
 "parts_4k:200:CONFIGS='$C' ROUNDS=${ROUNDS:-60} MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "parts_def:200:CONFIGS='$C' ROUNDS=${ROUNDS:-60} python3 scripts/ab.py"
