#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; each step has its own time
# limit; stop at the first fault / abort / timeout (exit >= 124 or signal).
# usage: tools/gpu_session.sh "<name>|<seconds>|<command>" ...
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then
    echo "stopping after fatal rc=$rc"; exit $rc
  fi
done
exit 0
