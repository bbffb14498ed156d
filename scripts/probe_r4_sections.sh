#!/bin/bash
# Round 4, backup profile: section length of the long buffers' speculative cut walk (256 Ki /
# 512 Ki / 1 Mi positions) now that sections are joined in parallel; one process, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/gpu_session.sh \
 "sections_ab:240:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so CONFIGS='s20:;s19:SDFS_SEC_LOG2=19;s18:SDFS_SEC_LOG2=18' ROUNDS=10 BACKUP=1 python3 scripts/ab.py"
