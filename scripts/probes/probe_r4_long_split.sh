#!/bin/bash
# Round 4, backup profile (40 MiB buffers, maxLen 128 KiB): the chunks > 32 KiB in the latency
# form (chunk_hash_long_kernel; off: SDFS_LONG_SPLIT=0) and the parallel join/place stitch of the
# sections (off: SDFS_PAR_STITCH=0), each against production, one process, interleaved; then the
# configs[4] bench on the product library and a rocprof of it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
 "long_split_ab:240:SDFS_CDC_LIB=$PWD/sdfs_amd/libsdfs_cdc_tuning.so CONFIGS='prod:;nolong:SDFS_LONG_SPLIT=0;seqstitch:SDFS_PAR_STITCH=0;neither:SDFS_LONG_SPLIT=0,SDFS_PAR_STITCH=0' ROUNDS=10 BACKUP=1 python3 scripts/ab.py" \
 "cfg_backup:300:CONFIG=backup python3 scripts/config_bench.py"
# the resolve kernels of the 40 MiB buffers, separately (speculative section walk, stitch)
mkdir -p gpurun_out/backup_prof
cd /tmp && CONFIG=backup STEPS=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/backup_prof" -- python3 "$GRAFT_REPO_ROOT/scripts/config_bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/backup_prof/log.txt" 2>&1
