#!/bin/bash
# Round 4: the list walk (production) against the queue walk (SDFS_LIST_WALK=0) and the scan
# without any walk (SDFS_SKIP_WALK=1, measurement only).  GPU_TESTS=1 runs the parity suite first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
steps=()
[ "$GPU_TESTS" = 1 ] && steps+=("gpu_tests:300:SDFS_CDC_LIB= python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread")
steps+=("list_4k:200:CONFIGS='list:;queue:SDFS_LIST_WALK=0;nowalk:SDFS_SKIP_WALK=1' ROUNDS=${ROUNDS:-40} MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py"
        "list_def:200:CONFIGS='list:;queue:SDFS_LIST_WALK=0;nowalk:SDFS_SKIP_WALK=1' ROUNDS=${ROUNDS:-40} python3 scripts/ab.py")
bash scripts/gpu_session.sh "${steps[@]}"
