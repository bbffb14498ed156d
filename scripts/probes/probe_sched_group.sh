#!/bin/bash
# Scan scheduling-region size (SDFS_SCAN_SCHED_GROUP: 2 / 4 production / 8 bytes) after the
# SGPR-mask candidate bits: product library builds differing only in cdc_kernels.o, one ab.py
# process each, interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
  "g4a:120:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc.so CONFIGS=g4: ROUNDS=12 python scripts/ab.py" \
  "g2a:120:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_sg2.so CONFIGS=g2: ROUNDS=12 python scripts/ab.py" \
  "g8a:120:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_sg8.so CONFIGS=g8: ROUNDS=12 python scripts/ab.py" \
  "g4b:120:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc.so CONFIGS=g4: ROUNDS=12 python scripts/ab.py" \
  "g2b:120:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_sg2.so CONFIGS=g2: ROUNDS=12 python scripts/ab.py" \
  "g8b:120:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_sg8.so CONFIGS=g8: ROUNDS=12 python scripts/ab.py"
