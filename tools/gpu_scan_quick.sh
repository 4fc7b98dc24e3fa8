mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_ops.py -m gpu -k hw_scan -q --timeout 120 --timeout-method thread > gpurun_out/hwtest.log 2>&1; rc=$?; tail -2 gpurun_out/hwtest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/hw_scan_ab.py --rows 40000 --m 1440 288 720 --reps 5 > gpurun_out/scanab.log 2>&1 || exit 1
grep '^{' gpurun_out/scanab.log
timeout -k 10 120 python -u tools/hw_scan_probe.py > gpurun_out/probe.log 2>&1 || exit 1
cut -c1-700 gpurun_out/probe.log
