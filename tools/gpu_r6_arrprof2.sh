#!/bin/bash
# Round 6: cProfile of 2e2e / 4e2e cycles with 0.5 % arrivals (score-span callees).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
for c in 2e2e 4e2e; do
  FOREMAST_PROFILE_CYCLES=gpurun_out/ap_$c.prof timeout -k 10 400 python -u benchmarks/bench_configs.py --config $c \
    --steps 12 --warmup 3 --arrivals 0.005 > gpurun_out/ap_$c.log 2>&1 || { echo "$c failed"; tail -5 gpurun_out/ap_$c.log; exit 1; }
done
echo done
