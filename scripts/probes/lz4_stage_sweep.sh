# LZ4: chunk bytes staged in LDS (SDFS_LZ4_STAGE) vs read from global memory; workgroups per CU
for st in ${STAGES:-0 16384 32768}; do
  for k in ${WGS:-default}; do
    if [ "$k" = default ]; then unset SDFS_LZ4_WG_PER_CU; else export SDFS_LZ4_WG_PER_CU=$k; fi
    SDFS_LZ4_STAGE=$st SETS=text,random MODES=r123 REPS=3 NBUF=1024 CPU_SECS=0 THREADS=2 python scripts/lz4_bench.py | sed "s/^{/{\"stage\": $st, \"wg_per_cu\": \"$k\", /"
  done
done
