#!/bin/bash
# gpurun wrapper: re-submits ONLY when the infrastructure failed before the
# command started (status "transient", nothing ran); never re-runs a command
# that ran on a GPU.  Usage: tools/gpu.sh <timeout_s> '<command>'
T=$1; shift
for i in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@"
  rc=$?
  st=$(python3 -c "import json;d=json.load(open('gpurun_out/.last_call.json'));print(d['status'], d.get('run_s') or 0)" 2>/dev/null)
  case "$st" in
    "transient 0"|"transient 0.0") echo "[gpu.sh] infra transient before start; retry in 45s"; sleep 45;;
    *) exit $rc;;
  esac
done
exit $rc
