#!/bin/bash
# Run-to-run spread of the headline bench line on one box: the default command three times, then
# with a 5x longer timed region, then the default again (value, ms_per_step, one-stream hash ms).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
Q="--e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0"
for spec in "d1:" "d2:" "d3:" "s100:--steps 100" "s100r:--steps 100 --ramp-secs 2" "d4:"; do
  n=${spec%%:*}; a=${spec#*:}
  timeout -k 10 200 python3 bench.py $Q $a > gpurun_out/var_$n.log 2>&1 || exit 3
  echo "$n $(grep '^{' gpurun_out/var_$n.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], d["one_stream"]["value"])')" | tee -a gpurun_out/var_summary.txt
done
