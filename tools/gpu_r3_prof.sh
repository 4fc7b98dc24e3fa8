#!/bin/bash
# rocprofv3 kernel-trace summaries of the headline, config 2 (+FFT), config 4 (H=256x2 mv, layer-pipelined) and 5 on the round-3 tree
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
prof() { name=$1; shift; timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pr_$name -o $name -- "$@" > $R/gpurun_out/pr_$name.log 2>&1 || { echo "$name failed"; return 1; }; python3 $R/tools/prof_summary.py $R/gpurun_out/pr_$name > $R/gpurun_out/kernels_${name}_r3.txt; rm -rf $R/gpurun_out/pr_$name; }
prof bench python3 $R/bench.py --steps 20 --warmup 5 &&
prof c2 python3 $R/benchmarks/bench_configs.py --config 2 --steps 3 --warmup 1 &&
prof c2fft python3 $R/benchmarks/bench_configs.py --config 2 --detect-period --steps 3 --warmup 1 &&
prof c4mv python3 $R/benchmarks/bench_configs.py --config 4 --hidden 256 --layers 2 --multivariate --steps 3 --warmup 1 &&
prof c5 python3 $R/benchmarks/bench_configs.py --config 5 --steps 3 --warmup 1
echo rc=$?
