#!/bin/bash
# 4e2e departure-only vs 0.5 % arrivals, then a cProfile of the arrivals cycles.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/arr_r6.jsonl
: > $OUT
for a in 0 0.005; do
  timeout -k 10 420 python -u benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3 --arrivals $a > gpurun_out/arr_$a.log 2>&1 || { echo "4e2e $a failed"; tail -5 gpurun_out/arr_$a.log; exit 1; }
  grep '^{' gpurun_out/arr_$a.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']; c['arrivals']=$a
open('$OUT','a').write(json.dumps(d)+'\n')
print('4e2e arrivals=$a', round(d['ms_per_step'],2), c.get('span_ms_median_rank0'), c.get('onboarding'), c.get('lstm_early_launch'))"
done
FOREMAST_PROFILE_CYCLES=gpurun_out/hp_arr.prof timeout -k 10 420 python -u benchmarks/bench_configs.py --config 4e2e --steps 10 --warmup 3 --arrivals 0.005 > gpurun_out/hp_arr.log 2>&1 || { echo prof failed; exit 1; }
python -c "
import pstats
s=pstats.Stats('gpurun_out/hp_arr.prof', stream=open('gpurun_out/hp_arr.txt','w'))
s.sort_stats('cumulative').print_stats(90); s.sort_stats('tottime').print_stats(40)"
echo done
