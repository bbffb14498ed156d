#!/bin/bash
# Scan wave issue priorities (ScanArgs::wave_prio, tuning SDFS_SCAN_WPRIO) A/B on the headline
# bench, interleaved, tuning library; one JSON line per run in gpurun_out/wprio.jsonl.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
L=$PWD/sdfs_amd/libsdfs_cdc_tuning.so
B="python3 bench.py --steps 20 --warmup 3 --e2e-mib 0 --threads= --other-mix 0 --cpu-secs 0 --cpu-1t-secs 0"
for r in 1 2 3; do
  for p in 0 1; do
    SDFS_CDC_LIB=$L SDFS_SCAN_WPRIO=$p timeout -k 10 120 $B > gpurun_out/wprio_run.json || exit 1
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/wprio_run.json').read().splitlines()[-1]); print(json.dumps({'wprio': $p, 'value': d['value'], 'ms': d['ms_per_step'], 'one_stream_ms': d['one_stream']['ms_per_step'], 'scan_ms': d['kernels_ms']['cdc_scan'], 'hash_ms': d['roofline']['kernel_ms'], 'identical': d['config']['records_identical_across_streams']}))" >> gpurun_out/wprio.jsonl || exit 1
  done
done
