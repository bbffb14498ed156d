#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
  "variants:200:python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 150 --timeout-method thread -k scan_variants" \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread"
