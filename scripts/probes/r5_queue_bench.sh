cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
MASK_BITS=11 MIN_SEG_KIB=2 THREADS=1,8,48 timeout -k 10 200 python3 scripts/queue_probe.py > gpurun_out/probe_prod.jsonl 2>gpurun_out/probe_prod.err && \
timeout -k 10 300 python3 bench.py --cpu-secs 0 --cpu-1t-secs 0 > gpurun_out/bench.log 2>&1
