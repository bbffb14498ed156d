#!/bin/bash
# The backup profile's slice (configs[4]): kernel trace + VALU/cycle counters of config_bench in
# one run (per-kernel clock and VALU utilisation, scripts/valu_clock.py), after a plain run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/backup_clock
bash scripts/gpu_session.sh \
  "cfg_backup:240:CONFIG=backup STEPS=5 python3 scripts/config_bench.py > gpurun_out/backup_clock/cfg.log 2>&1" \
  "clock:240:cd /tmp && CONFIG=backup STEPS=3 timeout -s KILL 200 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --output-format csv -d $R/gpurun_out/backup_clock/clock -- python3 $R/scripts/config_bench.py > $R/gpurun_out/backup_clock/clock.log 2>&1"
