#!/bin/bash
# Round 6, GPU session 8: the randomized-parameter parity tests.
set -o pipefail
O=gpurun_out/r6s8
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_random_params.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_random.log 2>&1 &&
echo "random params ok"
