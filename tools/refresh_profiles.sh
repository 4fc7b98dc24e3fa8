#!/bin/bash
# Re-measure every benchmark config and collect rocprofv3 kernel-trace stats
# (run on the GPU box from the repo root).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
set -o pipefail
run() { name=$1; secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$R/gpurun_out/$name.log" 2>&1; rc=$?; echo "$name rc=$rc"; return $rc; }
run bench 200 python3 "$R/bench.py" --steps 50 --warmup 10 &&
run bench_serial 200 python3 "$R/bench.py" --steps 50 --warmup 10 --mode serial &&
run c1 300 python3 "$R/benchmarks/bench_configs.py" --config 1 --device cuda --jobs 200 --steps 5 --warmup 1 &&
run c1cpu 300 python3 "$R/benchmarks/bench_configs.py" --config 1 --device cpu --jobs 200 --steps 5 --warmup 1 &&
run c2 200 python3 "$R/benchmarks/bench_configs.py" --config 2 &&
run c2fft 200 python3 "$R/benchmarks/bench_configs.py" --config 2 --detect-period &&
run c2cached 200 python3 "$R/benchmarks/bench_configs.py" --config 2 --cached &&
run c3cpu 600 python3 "$R/benchmarks/bench_configs.py" --config 3 --device cpu --steps 2 --warmup 1 &&
run c4 200 python3 "$R/benchmarks/bench_configs.py" --config 4 &&
run c5 200 python3 "$R/benchmarks/bench_configs.py" --config 5 &&
cd /tmp && export TMPDIR=/tmp &&
run prof_bench 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_bench" -o bench -- python3 "$R/bench.py" --steps 20 --warmup 5 &&
run prof_c2 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c2" -o c2 -- python3 "$R/benchmarks/bench_configs.py" --config 2 --steps 5 --warmup 2 &&
run prof_c4 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c4" -o c4 -- python3 "$R/benchmarks/bench_configs.py" --config 4 --steps 5 --warmup 2 &&
run prof_c5 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c5" -o c5 -- python3 "$R/benchmarks/bench_configs.py" --config 5 --steps 5 --warmup 2
