#!/bin/bash
# The three variable-block hash types on the round-end kernels (bench.py --hash-type).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
Q="--threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --other-mix 0 --compare 0"
bash scripts/gpu_session.sh \
  "sha256:120:python bench.py $Q --hash-type VARIABLE_SHA256" \
  "sha160:120:python bench.py $Q --hash-type VARIABLE_SHA256_160" \
  "md5:120:python bench.py $Q --hash-type VARIABLE_MD5"
