set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/resident_ab.py > gpurun_out/resident_ab.log 2>&1 && \
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 120 python bench.py > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 400 python -u benchmarks/bench_configs.py --config 3e2e --steps 30 --warmup 3 > gpurun_out/c3e2e.log 2>&1
echo exit=$?
