#!/bin/bash
# Round 6: host profiles (cProfile of the timed cycles) of the churn configs.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
prof() {
  name=$1; shift
  FOREMAST_PROFILE_CYCLES=gpurun_out/hp_$name.prof timeout -k 10 420 python -u benchmarks/bench_configs.py "$@" > gpurun_out/hp_$name.log 2>&1 || { echo "$name FAILED"; tail -5 gpurun_out/hp_$name.log; return 1; }
  python -c "
import pstats,sys
s=pstats.Stats('gpurun_out/hp_$name.prof', stream=open('gpurun_out/hp_$name.txt','w'))
s.sort_stats('cumulative').print_stats(60); s.sort_stats('tottime').print_stats(40)"
  grep '^{' gpurun_out/hp_$name.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']
print('$name', round(d['ms_per_step'],2), c.get('span_ms_median_rank0'), c.get('onboarding'))"
}
prof 4e2e_arr --config 4e2e --steps 10 --warmup 3 --arrivals 0.005 &&
prof mixed --config mixed --steps 10 --warmup 3
