#!/bin/bash
# Round 5: the bench's exchange path at N = 1 (RecordExchange over RCCL, world 1) and the torchrun
# launch form the driver uses for N > 1, run here with one rank.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
A="--steps 10 --warmup 2 --threads= --e2e-mib 0 --cpu-secs 0 --cpu-1t-secs 0 --other-mix 0 --compare 0"
bash scripts/gpu_session.sh \
  "bench_ex:240:python3 bench.py --exchange 1 $A > gpurun_out/bench_exchange.json" \
  "bench_torchrun:240:python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 1 $A > gpurun_out/bench_torchrun.json" \
  "dist_gpu:300:python -u -m pytest tests/test_dist_gpu.py -x -q --timeout 150 --timeout-method thread"
