set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_ops.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests_lstm.log 2>&1
echo tests=$?
for a in "--hidden 128" "--hidden 256 --layers 2 --multivariate" "--hidden 128 --layers 2 --multivariate" "--hidden 256 --layers 2"; do
  timeout -k 10 200 python -u benchmarks/bench_configs.py --config 4 --steps 5 --warmup 2 $a >> gpurun_out/c4_variants.log 2>&1 || exit 1
done
echo exit=$?
