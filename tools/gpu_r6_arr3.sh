#!/bin/bash
# Round 6: arrivals after the cache-lookup patch: GPU parity tests of the fast
# path, then 2e2e / 4e2e departure-only vs 0.5 % arrivals.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fastpath_models.py tests/test_model_ops.py -m gpu -x -q --timeout 200 \
  --timeout-method thread > gpurun_out/arr3_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/arr3_tests.log; exit 1; }
tail -1 gpurun_out/arr3_tests.log
OUT=gpurun_out/arr3.jsonl
: > $OUT
for c in 2e2e 4e2e; do
  for a in 0 0.005; do
    timeout -k 10 420 python -u benchmarks/bench_configs.py --config $c --steps 20 --warmup 3 --arrivals $a > gpurun_out/arr3_$c_$a.log 2>&1 || { echo "$c $a failed"; exit 1; }
    grep '^{' gpurun_out/arr3_$c_$a.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']; c['arrivals']=$a; c['run']='${c}_$a'
open('$OUT','a').write(json.dumps(d)+'\n')
print('$c', $a, round(d['ms_per_step'],2), c.get('span_ms_median_rank0'))"
  done
done
