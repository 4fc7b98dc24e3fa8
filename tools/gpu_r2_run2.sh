set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 120 python bench.py > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 400 python -u benchmarks/bench_configs.py --config 3e2e --steps 20 --warmup 3 > gpurun_out/c3e2e.log 2>&1
echo exit=$?
