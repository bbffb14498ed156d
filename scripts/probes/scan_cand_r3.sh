#!/bin/bash
# Round 3: production scan after the SDWA addresses (prod) against the form before (32) and the
# group-minimum candidate bits (48: groups of 4, 49: groups of 8); interleaved in one process
# (scripts/ab.py), both mixes; then the VGPR bank-conflict microbenchmark.  Second run: the
# pop entries high word first (50; with the groups of 8: 51).  Third run: + the bit-select pop
# address of the byte already in place (52 = 51 + mux, 53 = 50 + mux).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
C='prod:;min8_popswap:SDFS_SCAN_VARIANT=51;min8_popswap_mux:SDFS_SCAN_VARIANT=52;popswap_mux:SDFS_SCAN_VARIANT=53;popswap:SDFS_SCAN_VARIANT=50'
bash scripts/gpu_session.sh \
 "cand_4k:200:CONFIGS='$C' ROUNDS=10 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py" \
 "cand_def:200:CONFIGS='$C' ROUNDS=10 python3 scripts/ab.py"
