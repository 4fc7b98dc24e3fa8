#!/bin/bash
# Round 6: XCD split stored as fractions of the rows (survives the row count
# changing with churn).  Canary / fast-path GPU parity tests, then the headline
# bench balancing off vs on, then the canary e2e with 0.5 % arrivals (the row
# count changes every cycle) off vs on.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_canary_ops.py tests/test_fastpath.py tests/test_fastpath_models.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/xf_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/xf_tests.log; exit 1; }
tail -1 gpurun_out/xf_tests.log
OUT=gpurun_out/xcdfrac_ab.jsonl
: > $OUT
for rep in 1 2 3; do
  for b in 0 1; do
    FM_XCD_BALANCE=$b timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/xf_b.log 2>&1 || { echo "bench $b failed"; tail -5 gpurun_out/xf_b.log; exit 1; }
    grep '^{' gpurun_out/xf_b.log | sed "s/^{/{\"run\": \"bench\", \"xcd_balance\": $b, /" >> $OUT
    grep '^{' gpurun_out/xf_b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', $b, round(d['ms_per_step'],4))"
  done
done
for rep in 1 2; do
  for b in 0 1; do
    FM_XCD_BALANCE=$b timeout -k 10 420 python -u benchmarks/bench_configs.py --config 2e2e --steps 20 --warmup 3 --arrivals 0.005 \
      > gpurun_out/xf_e.log 2>&1 || { echo "2e2e $b failed"; tail -5 gpurun_out/xf_e.log; exit 1; }
    grep '^{' gpurun_out/xf_e.log | sed "s/^{/{\"run\": \"2e2e_arrivals\", \"xcd_balance\": $b, /" >> $OUT
    grep '^{' gpurun_out/xf_e.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read()); print('2e2e', $b, round(d['ms_per_step'],3), d['config'].get('span_ms_median_rank0',{}).get('score'))"
  done
done
