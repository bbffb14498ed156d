#!/bin/bash
# The register-only SHA-256 microbenchmark (scripts/sha_codesize_mb.hip, built as scripts/bin/sha_cs)
# under a kernel trace with GRBM_GUI_ACTIVE / SQ_INSTS_VALU: cycles per wave64 VALU instruction of
# the compression at its own clock (the rate chunk_hash is compared against in DESIGN.md §7).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
R=$PWD
export TMPDIR=/tmp
mkdir -p gpurun_out/sha_clock
cd /tmp && timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES \
  --output-format csv -d $R/gpurun_out/sha_clock/run -- $R/scripts/bin/sha_cs > $R/gpurun_out/sha_clock/run.log 2>&1
