#!/bin/bash
# Round 4: the scan's per-wave work queue (SDFS_SCAN_DYN=1, tuning only) against the static
# workgroup stride (production): GPU parity suite, one-stream stage times (ab.py) at both mixes, then the
# two-stream headline bench with the tuning library, alternating the two forms three times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
T=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
Q="--e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0 --compare 0"
steps=()
[ "$GPU_TESTS" = 1 ] && steps+=("gpu_tests:300:python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread")
steps+=("dyn_4k:200:SDFS_CDC_LIB=$T CONFIGS='static:;dyn:SDFS_SCAN_DYN=1' ROUNDS=40 MIN_SEG_KIB=2 MASK_BITS=11 python3 scripts/ab.py"
        "dyn_def:200:SDFS_CDC_LIB=$T CONFIGS='static:;dyn:SDFS_SCAN_DYN=1' ROUNDS=40 python3 scripts/ab.py")
for r in 1 2 3; do
  steps+=("b_dyn_$r:120:SDFS_CDC_LIB=$T SDFS_SCAN_DYN=1 python3 bench.py $Q" "b_static_$r:120:SDFS_CDC_LIB=$T SDFS_SCAN_DYN=0 python3 bench.py $Q")
done
bash scripts/gpu_session.sh "${steps[@]}"
for f in gpurun_out/b_*.log; do echo "$(basename $f .log) $(grep '^{' $f | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["kernels_ms"]["cdc_scan"])')"; done > gpurun_out/dyn_bench_summary.txt
