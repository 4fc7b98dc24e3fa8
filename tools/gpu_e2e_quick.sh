#!/bin/bash
# The sliding e2e configs (2e2e, 4e2e) and the 10k warm restart, one line each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for c in 2e2e 4e2e; do
  timeout -k 10 400 python -u benchmarks/bench_configs.py --config $c --steps 20 --warmup 3 > gpurun_out/e2e_$c.log 2>&1 || exit 1
  grep '^{' gpurun_out/e2e_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['ms_per_step'],3), d['config']['span_ms_median_rank0'])"
done
timeout -k 10 400 python -u benchmarks/bench_configs.py --config 3e2e --steps 5 --warmup 2 --restart > gpurun_out/e2e_restart.log 2>&1 || exit 1
grep "warm restart" gpurun_out/e2e_restart.log | cut -c1-700
