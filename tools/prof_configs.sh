#!/bin/bash
# rocprofv3 kernel-trace + stats of the per-config benchmarks (run on the GPU box)
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c$c" -o c$c -- \
    python3 "$R/benchmarks/bench_configs.py" --config "$c" --steps 5 --warmup 2 > "$R/gpurun_out/prof_c$c.log" 2>&1
  rc=$?
  echo "config $c rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
