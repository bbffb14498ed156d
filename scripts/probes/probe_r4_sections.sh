#!/bin/bash
# Round 4, backup profile (40 MiB buffers): the long buffers' sectioned cut walk — production
# (256 Ki-position sections walked in the scan's epilogue, parallel join/place) against the same
# sections walked by the spec kernel (SDFS_PIECE_WALK=0), 1 Mi sections (SDFS_SEC_LOG2=20) and the
# round-3 form (1 Mi sections, sequential stitch); one process, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
 "sections_ab:240:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so CONFIGS='prod:;nopiece:SDFS_PIECE_WALK=0;s20:SDFS_SEC_LOG2=20;r3:SDFS_SEC_LOG2=20,SDFS_PAR_STITCH=0' ROUNDS=10 BACKUP=1 python3 scripts/ab.py"
