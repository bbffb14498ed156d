#!/bin/bash
# New GPU tests first (short limits), then the whole GPU suite, smoke and the default bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
  "newtests:300:python -u -m pytest tests/test_gpu_share.py tests/test_lz4.py -x -v --timeout 150 --timeout-method thread -k 'share or destroy or device_set or backup_buffer or over_128k'" \
  "gputests:700:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
  "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:300:python bench.py"
