#!/bin/bash
# Round 6: where a long mixed-fleet soak's cycle time goes -- cProfile of
# cycles 100-150 and of the last 50 (FOREMAST_SOAK_PROFILE), resources and
# container sizes every 100 cycles.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
FOREMAST_SOAK_PROFILE=gpurun_out/sp timeout -k 10 800 python -u benchmarks/bench_configs.py --config mixed --source http \
  --steps ${STEPS:-1200} --warmup 20 --soak-every 100 --soak-save-every 30 --no-prestage --job-retention-s 21600 \
  --hpalog-retention-s 21600 > gpurun_out/soakprof.log 2>&1 || { echo soak failed; tail -5 gpurun_out/soakprof.log; exit 1; }
for w in early late; do
  python -c "
import pstats,sys
s=pstats.Stats('gpurun_out/sp_$w.prof', stream=open('gpurun_out/sp_$w.txt','w'))
s.sort_stats('tottime').print_stats(60); s.sort_stats('cumulative').print_stats(80)
s.sort_stats('cumulative').print_callees('prepare'); s.print_callees('_layout_groups'); s.print_callees('fetch_all')" || exit 1
done
echo done
