set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_ops.py tests/test_brain_e2e.py -m gpu -x -v --timeout 120 --timeout-method thread -k "es_ or brain_every" > gpurun_out/gputests_es.log 2>&1
echo tests=$?
timeout -k 10 200 python -u benchmarks/bench_configs.py --config 2 --steps 5 --warmup 2 > gpurun_out/c2.log 2>&1 && \
timeout -k 10 200 python -u benchmarks/bench_configs.py --config 2 --steps 5 --warmup 2 --detect-period >> gpurun_out/c2.log 2>&1
echo exit=$?
