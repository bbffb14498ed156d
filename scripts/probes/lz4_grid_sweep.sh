# LZ4 workgroups-per-CU sweep (LDS table) and the global-table variant (SDFS_LZ4_GTAB=1)
for k in ${WGS:-2 4 6 8 9 12}; do SDFS_LZ4_WG_PER_CU=$k SETS=text,random MODES=r123 REPS=3 NBUF=1024 CPU_SECS=0 THREADS=2 python scripts/lz4_bench.py | sed "s/^{/{\"wg_per_cu\": $k, \"gtab\": 0, /"; done
for k in ${GWGS:-}; do SDFS_LZ4_GTAB=1 SDFS_LZ4_WG_PER_CU=$k SETS=text,random MODES=r123 REPS=3 NBUF=1024 CPU_SECS=0 THREADS=2 python scripts/lz4_bench.py | sed "s/^{/{\"wg_per_cu\": $k, \"gtab\": 1, /"; done
