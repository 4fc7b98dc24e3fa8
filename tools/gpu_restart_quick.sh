mkdir -p gpurun_out
timeout -k 10 400 python -u benchmarks/bench_configs.py --config 3e2e --steps 5 --warmup 2 --restart > gpurun_out/e2e_restart.log 2>&1 || exit 1
grep "warm restart" gpurun_out/e2e_restart.log | cut -c1-500
