#!/bin/bash
# Round 6, GPU session 4 (production defaults: work-queue scan, 6 queue lanes, early completion,
# high-priority exchange streams): GPU suite, smoke, the driver's bench line, the device-set and
# torchrun forms at full length, and the exchange projection with the production scan.
set -o pipefail
O=gpurun_out/r6s4
mkdir -p $O
Q="--steps 20 --warmup 3 --cpu-secs 0 --e2e-mib 0 --threads= --other-mix 0"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 180 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench_default.jsonl 2> $O/bench_default.err &&
echo "bench ok" &&
timeout -k 10 600 python -u bench.py --gpus 1 --inproc 1 > $O/bench_device_set.jsonl 2> $O/bench_device_set.err &&
timeout -k 10 600 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29561 \
  bench.py --gpus 1 --exchange 1 > $O/bench_torchrun_ex.jsonl 2> $O/bench_torchrun_ex.err &&
echo "forms ok" &&
for px in "--exchange-proxy 0" "--exchange-proxy 8 --proxy-prio 1" "--exchange-proxy 8" "--exchange-proxy 8 --proxy-prio 1 --proxy-record-bytes 36"; do
  timeout -k 10 180 python -u bench.py $Q $px >> $O/proxy_prod.jsonl 2>> $O/proxy.err || exit 1
done &&
echo "proxy ok"
