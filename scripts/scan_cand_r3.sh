#!/bin/bash
# Round 3: production scan after the SDWA addresses (prod) against the form before (32) and the
# group-minimum candidate bits (48: groups of 4, 49: groups of 8); interleaved in one process
# (scripts/ab.py), both mixes; then the VGPR bank-conflict microbenchmark.  Second run: the
# pop entries high word first (50; with the groups of 8: 51).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;popswap:SDFS_SCAN_VARIANT=50;min8:SDFS_SCAN_VARIANT=49;min8_popswap:SDFS_SCAN_VARIANT=51;pre_sdwa:SDFS_SCAN_VARIANT=32'
bash scripts/gpu_session.sh \
 "cand_4k:200:CONFIGS='$C' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "cand_def:200:CONFIGS='$C' ROUNDS=8 python3 scripts/ab.py" \
 "vbank:120:/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 scripts/vgpr_bank_microbench.hip -o /tmp/vbank && /tmp/vbank"
