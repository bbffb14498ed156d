#!/bin/bash
# Round-6 end evidence (second pass, after the latency-form and queue changes) on the final tree: GPU suite, smoke, the driver's default bench line,
# rocprofv3 kernel stats of the one-stream bench (the roofline's chunk_hash launch) and of the
# two-stream timed region, then the PMC passes (instruction mix / waits, FETCH_SIZE, WRITE_SIZE)
# at the metric's 4 KiB mix.  Output: gpurun_out/r6end/.
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/../.." && pwd)}"
cd "$R" || exit 1
O=gpurun_out/r6end2
mkdir -p $O
export TMPDIR=/tmp
B1="python3 $R/bench.py --steps 20 --warmup 3 --streams-in-flight 1 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
B2="python3 $R/bench.py --steps 200 --warmup 3 --ramp-secs 0 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/pytest.log 2>&1 &&
echo "pytest ok" &&
timeout -k 10 180 python -u -c 'import __graft_entry__ as g; g.smoke()' > $O/smoke.log 2>&1 &&
timeout -k 10 600 python -u bench.py > $O/bench_default.jsonl 2> $O/bench_default.err &&
echo "bench ok" &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_one_stream -- $B1 > $R/$O/bench_one_stream.log 2>&1) &&
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/$O/prof_two_stream -- $B2 > $R/$O/bench_two_stream.log 2>&1) &&
echo "rocprof ok"
