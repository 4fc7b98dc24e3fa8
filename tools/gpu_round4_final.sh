#!/bin/bash
# Round-4 measurement session: scan-fit tests + A/B + PMC instruction count,
# the sliding e2e configs (2e2e, 4e2e) and the 10k warm restart.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_ops.py -m gpu -k hw_scan -q --timeout 120 --timeout-method thread \
  > gpurun_out/hwtest.log 2>&1; rc=$?; tail -2 gpurun_out/hwtest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/hw_scan_ab.py --rows 40000 --m 1440 288 720 --reps 5 > gpurun_out/scanab.log 2>&1 || exit 1
grep '^{' gpurun_out/scanab.log
bash tools/pmc_hwscan_phases.sh > /dev/null 2>&1 || exit 1
grep "DEBUG\|VALU\|duration" gpurun_out/pmc_hwscan_phases.txt
for c in 2e2e 4e2e; do
  timeout -k 10 400 python -u benchmarks/bench_configs.py --config $c --steps 20 --warmup 3 > gpurun_out/e2e_$c.log 2>&1 || exit 1
  grep '^{' gpurun_out/e2e_$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', round(d['ms_per_step'],3), d['config']['span_ms_median_rank0'])"
done
timeout -k 10 400 python -u benchmarks/bench_configs.py --config 3e2e --steps 5 --warmup 2 --restart > gpurun_out/e2e_restart.log 2>&1 || exit 1
grep "warm restart" gpurun_out/e2e_restart.log | cut -c1-700
