#!/bin/bash
# config 4 variants at the default stacked tilings (H = 256: 4 x 2)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/c4_variants.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_model_ops.py -m gpu -k "lstm" > gpurun_out/lstm_tests.log 2>&1 || exit 1
for a in "--hidden 128" "--hidden 256 --layers 2 --multivariate" "--hidden 128 --layers 2 --multivariate" "--hidden 256 --layers 2" "--hidden 256"; do
  timeout -k 10 200 python benchmarks/bench_configs.py --config 4 $a 2>/dev/null | grep '^{' >> gpurun_out/c4_variants.jsonl || exit 1
done
echo done
