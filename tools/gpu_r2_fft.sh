#!/bin/bash
# FFT rework: numerics tests, stand-alone timing, config 2 with FFT period, kernel trace
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_ops.py tests/test_library.py -m gpu -k "fft or library" > gpurun_out/fft_tests.log 2>&1 &&
timeout -k 10 200 python tools/fft_bench.py > gpurun_out/fft_bench.jsonl 2>&1 &&
timeout -k 10 200 python benchmarks/bench_configs.py --config 2 --detect-period > gpurun_out/c2fft.jsonl 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_fft -o fft -- python3 $GRAFT_REPO_ROOT/tools/fft_bench.py --lengths 10080 --iters 5 > $GRAFT_REPO_ROOT/gpurun_out/prof_fft.log 2>&1 &&
python3 $GRAFT_REPO_ROOT/tools/prof_summary.py $GRAFT_REPO_ROOT/gpurun_out/prof_fft > $GRAFT_REPO_ROOT/gpurun_out/kernels_fft.txt
echo rc=$?
