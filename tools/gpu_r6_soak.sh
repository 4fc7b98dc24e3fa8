#!/bin/bash
# Round 6 soak: 2,000 brain cycles of the mixed fleet over
# HTTP (fake Prometheus in its own processes), arrivals / resubmissions /
# closes every cycle, an async history checkpoint every 30 cycles; resources
# sampled every 100 cycles.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 1000 python -u benchmarks/bench_configs.py --config mixed --source http --steps 2000 --warmup 20 \
  --soak-every 100 --soak-save-every 30 --no-prestage > gpurun_out/soak_r6.log 2>&1
rc=$?
grep '^{' gpurun_out/soak_r6.log > gpurun_out/soak_r6.json
grep '^\[soak\]' gpurun_out/soak_r6.log | tail -3 | cut -c1-400
exit $rc
