#!/bin/bash
# Round 4: instruction counts of the scan kernel with the list walk, the queue walk and no walk
# (one PMC pass each, ab.py at the 4 KiB-mean mix, one config per run).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
export TMPDIR=/tmp SDFS_CDC_LIB=$R/sdfs_amd/libsdfs_cdc_tuning.so ROUNDS=2 MIN_SEG_KIB=2 MASK_BITS=11
OUT=$R/gpurun_out/walk_pmc
mkdir -p "$OUT"
cd /tmp || exit 1
for c in "list:" "queue:SDFS_LIST_WALK=0" "nowalk:SDFS_SKIP_WALK=1"; do
  n=${c%%:*}
  CONFIGS="$c" timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH \
    --output-format csv -d "$OUT/$n" -- python3 $R/scripts/ab.py > "$OUT/$n.log" 2>&1 || exit 2
  CONFIGS="$c" timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_LDS_BANK_CONFLICT \
    --output-format csv -d "$OUT/${n}_st" -- python3 $R/scripts/ab.py > "$OUT/${n}_st.log" 2>&1 || exit 3
done
echo done
