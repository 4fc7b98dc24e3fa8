#!/bin/bash
# Round 6 soak: brain cycles of the mixed fleet over HTTP
# (fake Prometheus in its own processes), arrivals / resubmissions / closes
# every cycle, an async history checkpoint every 30 cycles; resources sampled
# every 100 cycles.  STEPS (default 2000) cycles.  The store applies the
# shipped retention (closed jobs and HPA logs older than 6 simulated hours:
# JOB_RETENTION_SECONDS / HPALOG_RETENTION_SECONDS), so its files reach a
# steady size inside the run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
STEPS=${STEPS:-2000}
timeout -k 10 1000 python -u benchmarks/bench_configs.py --config mixed --source http --steps $STEPS --warmup 20 \
  --soak-every 100 --soak-save-every 30 --no-prestage \
  --job-retention-s ${RET:-21600} --hpalog-retention-s ${RET:-21600} ${EXTRA:-} > gpurun_out/soak_r6.log 2>&1
rc=$?
grep '^{' gpurun_out/soak_r6.log > gpurun_out/soak_r6.json
exit $rc
