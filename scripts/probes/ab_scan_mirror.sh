#!/bin/bash
# Round 2: GPU tests with the mirrored-state scan in production, then an interleaved A/B of the
# production scan (mirrored) against sweep variant 29 (the same configuration, plain state), then
# the default bench.  Results under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab:300:CONFIGS='mirror:;plain:SDFS_SCAN_VARIANT=29' ROUNDS=12 python scripts/ab.py" \
  "bench:240:python bench.py"
