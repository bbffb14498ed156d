#!/bin/bash
# GPU tests, then the queue trace (scripts/probes/queue_trace_r5.sh), then the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
  "qtrace:300:bash scripts/probes/queue_trace_r5.sh" \
  "bench:240:python bench.py"
