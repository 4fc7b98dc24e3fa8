#!/bin/bash
# Re-measure the GPU configs 2, 4, 5 (bench JSON lines + rocprofv3 kernel stats);
# the CPU-path configs (1, 3 on CPU) are in tools/refresh_profiles.sh.
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
run() { name=$1; secs=$2; shift 2; timeout -k 10 "$secs" "$@" > "$R/gpurun_out/$name.log" 2>&1; rc=$?; echo "$name rc=$rc"; return $rc; }
run c2 200 python3 "$R/benchmarks/bench_configs.py" --config 2 &&
run c2fft 200 python3 "$R/benchmarks/bench_configs.py" --config 2 --detect-period &&
run c2cached 200 python3 "$R/benchmarks/bench_configs.py" --config 2 --cached &&
run c4 200 python3 "$R/benchmarks/bench_configs.py" --config 4 &&
run c5 200 python3 "$R/benchmarks/bench_configs.py" --config 5 &&
cd /tmp && export TMPDIR=/tmp &&
run prof_c2fft 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c2fft" -o c2fft -- python3 "$R/benchmarks/bench_configs.py" --config 2 --detect-period --steps 5 --warmup 2 &&
run prof_c4 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c4" -o c4 -- python3 "$R/benchmarks/bench_configs.py" --config 4 --steps 5 --warmup 2 &&
run prof_c5 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c5" -o c5 -- python3 "$R/benchmarks/bench_configs.py" --config 5 --steps 5 --warmup 2
