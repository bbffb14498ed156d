#!/bin/bash
# Batches in flight (2 vs 3) at the default mix on the current kernels, then the default bench
# (at_4k_mean now three in flight, with the two-stream figure beside it).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
Q="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --other-mix 0"
bash scripts/gpu_session.sh \
  "d3:120:python bench.py $Q --streams-in-flight 3" \
  "d2:120:python bench.py $Q --streams-in-flight 2 --compare 0" \
  "d3b:120:python bench.py $Q --streams-in-flight 3 --compare 0" \
  "bench:240:python bench.py"
