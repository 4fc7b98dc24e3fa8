#!/bin/bash
# Round 6: per-group stable layouts for multi-group fleets (fp_plan._layout_groups):
# GPU parity tests, the mixed-fleet churn bench with and without the layouts
# (FM_GROUP_LAYOUT=0), then a 1,200-cycle soak.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_fastpath_models.py tests/test_fastpath.py tests/test_warm_restart.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > gpurun_out/glay_tests.log 2>&1 || { echo tests failed; tail -30 gpurun_out/glay_tests.log; exit 1; }
tail -1 gpurun_out/glay_tests.log
OUT=gpurun_out/glay_churn.jsonl
: > $OUT
one() { name=$1; shift
  timeout -k 10 420 python -u benchmarks/bench_configs.py "$@" > gpurun_out/glay_$name.log 2>&1 || { echo "$name failed"; tail -5 gpurun_out/glay_$name.log; return 1; }
  grep '^{' gpurun_out/glay_$name.log | python -c "
import json,sys
d=json.loads(sys.stdin.read()); c=d['config']; c['run']='$name'
open('$OUT','a').write(json.dumps(d)+'\n')
print('$name', round(d['ms_per_step'],2), c.get('span_ms_median_rank0'), c.get('fast_path_churn'))"; }
for rep in 1 2; do
  one mixed --config mixed --steps 20 --warmup 3 || exit 1
  FM_GROUP_LAYOUT=0 one mixed_nolay --config mixed --steps 20 --warmup 3 || exit 1
done
one hpa_resub --config mixed --mixed-class 2 --steps 12 --warmup 3 || exit 1
STEPS=${SOAK:-1200} bash tools/gpu_r6_soak.sh; echo "soak rc=$?"
