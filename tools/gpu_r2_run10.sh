set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_all.log 2>&1
echo tests=$?
timeout -k 10 120 python bench.py > gpurun_out/bench_final.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_configs.py --config 1 --steps 5 --warmup 2 > gpurun_out/c1_gpu.log 2>&1
timeout -k 10 300 python -u benchmarks/bench_configs.py --config 1 --steps 5 --warmup 2 --device cpu > gpurun_out/c1_cpu.log 2>&1
timeout -k 10 400 python -u benchmarks/bench_configs.py --config 3e2e --steps 30 --warmup 3 > gpurun_out/c3e2e.log 2>&1
timeout -k 10 200 python -u benchmarks/bench_configs.py --config 5 --steps 10 --warmup 3 > gpurun_out/c5.log 2>&1
echo exit=$?
