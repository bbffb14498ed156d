#!/bin/bash
# Round 6, GPU session 9: the other BASELINE configurations on the final tree (configs[2]: 8 GiB at
# 50 % duplicates with the index and map images; configs[4] slice: the tar-like backup stream with
# LZ4), and the LZ4 bench (text and random) for the §11 table.
set -o pipefail
O=gpurun_out/r6s9
mkdir -p $O
CONFIG=dedup timeout -k 10 300 python -u scripts/config_bench.py > $O/config_dedup.json 2> $O/config_dedup.err &&
CONFIG=backup timeout -k 10 300 python -u scripts/config_bench.py > $O/config_backup.json 2> $O/config_backup.err &&
echo "configs ok" &&
MODES=r123 CPU_SECS=4 timeout -k 10 400 python -u scripts/lz4_bench.py > $O/lz4_bench.jsonl 2> $O/lz4_bench.err &&
echo "lz4 ok"
