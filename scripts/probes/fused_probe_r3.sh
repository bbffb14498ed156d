#!/bin/bash
# Round 3: the fused scan + fingerprint kernel (cdc_device.h cdc_fused_kernel) measured as a probe:
# with SDFS_FUSED_PROBE=1 the engine replaces a batch's fingerprint kernel by the fused kernel over
# the same batch's scan (again) and its fingerprint tasks, so `chunk_hash` of that config is the
# fused kernel's duration, to compare with `cdc_scan` + `chunk_hash` of production (scripts/ab.py,
# one process, both mixes; records are checked identical).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;fused:SDFS_FUSED_PROBE=1'
bash scripts/gpu_session.sh \
 "fused_4k:200:CONFIGS='$C' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "fused_def:200:CONFIGS='$C' ROUNDS=8 python3 scripts/ab.py"
