#!/bin/bash
# Round 6: steady cycles under arrival churn.  Each line is
# one bench_configs JSON; a summary line per run on stdout.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/churn_r6.jsonl
: > $OUT
run() {
  name=$1; shift
  timeout -k 10 420 python -u benchmarks/bench_configs.py "$@" > gpurun_out/churn_$name.log 2>&1 || { echo "$name FAILED rc=$?"; tail -5 gpurun_out/churn_$name.log; return 1; }
  grep '^{' gpurun_out/churn_$name.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); d['config']['run']='$name'; c=d['config']
open('$OUT','a').write(json.dumps(d)+'\n')
print('$name', round(d['ms_per_step'],2), 'p50', round(d.get('p50_decision_latency_ms',0),2), c.get('span_ms_median_rank0'), c.get('onboarding'), c.get('fast_path_churn'), 'gen_ms', c.get('generator_ms_in_timed_cycles'), 'lstm', c.get('lstm_early_launch'))"
}
run 4e2e_dep --config 4e2e --steps 20 --warmup 3 &&
run 4e2e_arr --config 4e2e --steps 20 --warmup 3 --arrivals 0.005 &&
run hpa_resub --config mixed --mixed-class 2 --steps 12 --warmup 3 &&
run mixed --config mixed --steps 12 --warmup 3 &&
run 2e2e_dep --config 2e2e --steps 20 --warmup 3 &&
run 2e2e_arr --config 2e2e --steps 20 --warmup 3 --arrivals 0.005
