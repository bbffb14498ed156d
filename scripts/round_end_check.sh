#!/bin/bash
# What the driver runs at round end, on the committed tree: GPU tests, smoke, default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
  "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:240:python bench.py"
