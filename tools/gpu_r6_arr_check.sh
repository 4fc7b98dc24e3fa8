#!/bin/bash
# Arrivals in the early LSTM launch: the fast==general parity tests on the
# GPU, then 4e2e departure-only vs 0.5 % arrivals per cycle.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_fastpath_models.py \
  > gpurun_out/arr_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/arr_tests.log; exit 1; }
tail -1 gpurun_out/arr_tests.log
OUT=gpurun_out/arr_r6.jsonl
: > $OUT
for a in 0 0.005; do
  timeout -k 10 420 python -u benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3 --arrivals $a > gpurun_out/arr_$a.log 2>&1 || { echo "4e2e $a failed"; tail -5 gpurun_out/arr_$a.log; exit 1; }
  grep '^{' gpurun_out/arr_$a.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']; c['arrivals']=$a
open('$OUT','a').write(json.dumps(d)+'\n')
print('4e2e arrivals=$a', round(d['ms_per_step'],2), c.get('span_ms_median_rank0'), c.get('onboarding'), c.get('lstm_early_launch'), c.get('fast_path_churn'))"
done
