#!/bin/bash
# One vs two vs three batches in flight at the 4 KiB-mean mix (minLen 2047, 11-bit predicate)
# against the default mix, same box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
Q="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --other-mix 0"
bash scripts/gpu_session.sh \
  "d2:120:python bench.py $Q" \
  "k2:120:python bench.py $Q --min-seg-kib 2 --mask-bits 11" \
  "k3:120:python bench.py $Q --min-seg-kib 2 --mask-bits 11 --streams-in-flight 3 --compare 0" \
  "d2b:120:python bench.py $Q" \
  "k2b:120:python bench.py $Q --min-seg-kib 2 --mask-bits 11"
