# LZ4 decoder: LDS stage size x workgroups per CU (SDFS_LZ4_DEC_STAGE, SDFS_LZ4_DEC_WG_PER_CU)
for cfg in ${CFGS:-8192:16 8192:20 4096:24 4096:32}; do
  st=${cfg%%:*}; k=${cfg##*:}
  SDFS_LZ4_DEC_STAGE=$st SDFS_LZ4_DEC_WG_PER_CU=$k SETS=text,random MODES=r123 REPS=3 CPU_SECS=0 THREADS=2 python scripts/lz4_bench.py | sed "s/^{/{\"dec_stage\": $st, \"dec_wg_per_cu\": $k, /"
done
