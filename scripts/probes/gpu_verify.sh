#!/bin/bash
# GPU tests, an interleaved A/B of the production engine against AB_CONFIGS (ab.py syntax) at the
# default and 4 KiB-mean mixes, then the default bench.  Logs under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
AB=${AB_CONFIGS:-"prod:;mirror:SDFS_SCAN_VARIANT=30;plain:SDFS_SCAN_VARIANT=29"}
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab:300:CONFIGS='$AB' ROUNDS=12 python scripts/ab.py" \
  "ab4k:300:CONFIGS='$AB' ROUNDS=12 MIN_SEG_KIB=2 MASK_BITS=11 python scripts/ab.py" \
  "bench:240:python bench.py"
