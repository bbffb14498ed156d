#!/bin/bash
# Run named GPU steps, each under its own time limit; stop at the first crash/timeout/abort.
# usage: scripts/gpu_session.sh "name:secs:command" ...
# pytest failures (rc 1) do not stop the session; faults (134/139), timeouts (124/137) do.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
: > gpurun_out/status.txt
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "== $name (limit ${secs}s): $cmd" | tee -a gpurun_out/status.txt
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc $(( $(date +%s) - start ))s" | tee -a gpurun_out/status.txt
  tail -5 "gpurun_out/$name.log"
  case $rc in
    0|1|5) ;;
    *) echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/status.txt; exit $rc ;;
  esac
done
