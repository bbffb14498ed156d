#!/bin/bash
# Does the fingerprint kernel's HBM traffic cost it clock?  The production kernel and the same
# kernel without its data loads (hash sweep variant 45, wrong digests) under one counter pass each
# (kernel trace + GRBM_GUI_ACTIVE / SQ_INSTS_VALU), ab.py at the 4 KiB-mean mix.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
export TMPDIR=/tmp SDFS_CDC_LIB=$R/sdfs_amd/libsdfs_cdc_tuning.so ROUNDS=6 MIN_SEG_KIB=2 MASK_BITS=11
mkdir -p gpurun_out/hash_noload
cd /tmp || exit 1
for c in "prod:" "noload:SDFS_HASH_VARIANT=45"; do
  n=${c%%:*}
  CONFIGS="$c" timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES \
    --output-format csv -d $R/gpurun_out/hash_noload/$n -- python3 $R/scripts/ab.py > $R/gpurun_out/hash_noload/$n.log 2>&1 || exit 2
done
