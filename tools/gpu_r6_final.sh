#!/bin/bash
# Round 6 final validation on one box: every GPU test + smoke + the
# driver-shaped headline bench, the churn configs, then a 2,000-cycle soak.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
bash tools/gpu_check.sh tests smoke bench || exit 1
for i in 2 3; do
  timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_bench_$i.log 2>&1 || exit 1
  grep '^{' gpurun_out/final_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', round(d['ms_per_step'],4))"
done
timeout -k 10 120 python -u bench.py --services 1250 --steps 1000 --warmup 50 > gpurun_out/final_shard.log 2>&1 || exit 1
grep '^{' gpurun_out/final_shard.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('shard', round(d['ms_per_step'],4))"
bash tools/gpu_r6_churn.sh || exit 1
STEPS=${SOAK:-2000} bash tools/gpu_r6_soak.sh; echo "soak rc=$?"
