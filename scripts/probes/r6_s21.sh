#!/bin/bash
# Round 6, GPU session 21: the other configs on the final tree (the backup profile's long chunks
# run in the latency form, changed since profiles/r06/configs/).
set -o pipefail
O=gpurun_out/r6s21
mkdir -p $O
CONFIG=backup timeout -k 10 400 python -u scripts/config_bench.py > $O/config_backup.json 2> $O/backup.err || exit 1
echo "backup ok"
CONFIG=dedup timeout -k 10 400 python -u scripts/config_bench.py > $O/config_dedup.json 2> $O/dedup.err || exit 1
echo "dedup ok"
