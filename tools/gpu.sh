#!/bin/bash
# gpurun wrapper for this repo's development loop: runs ONE command on the GPU
# box and, only when the infrastructure reports that nothing ran (status
# "transient", run_s 0 -- box not obtained or lost while being prepared),
# waits and asks again, at most 4 times.  A command that ran is never re-run.
#   tools/gpu.sh TIMEOUT_S 'command'
T=$1; shift
for attempt in 1 2 3 4; do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > /tmp/gpurun_last.out 2>&1
  rc=$?
  tail -3 /tmp/gpurun_last.out
  st=$(python3 -c "import json; d=json.load(open('gpurun_out/.last_call.json')); print(d.get('status'), d.get('run_s'))" 2>/dev/null)
  case "$st" in
    "transient 0"|"transient 0.0"|"transient None") sleep $((30 * attempt)); continue ;;
  esac
  exit $rc
done
exit 3
