#!/bin/bash
# End-of-round sweep: every BASELINE config on the current tree, one JSON line each
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/bench_all_final.jsonl
rm -f $out
run() { name=$1; secs=$2; shift 2; echo "== $name" >&2; timeout -k 10 "$secs" "$@" 2>gpurun_out/final_$name.err | grep '^{' >> $out || { echo "$name failed" >&2; return 1; }; }
run bench 200 python bench.py --steps 300 --warmup 30 &&
run c1 300 python benchmarks/bench_configs.py --config 1 --device cuda --jobs 200 --steps 5 --warmup 1 &&
run c2 200 python benchmarks/bench_configs.py --config 2 &&
run c2fft 200 python benchmarks/bench_configs.py --config 2 --detect-period &&
run c2cached 200 python benchmarks/bench_configs.py --config 2 --cached &&
run c4 200 python benchmarks/bench_configs.py --config 4 &&
run c4mv 200 python benchmarks/bench_configs.py --config 4 --hidden 256 --layers 2 --multivariate &&
run c5 200 python benchmarks/bench_configs.py --config 5 &&
run c3e2e 600 python benchmarks/bench_configs.py --config 3e2e --steps 100 --warmup 5
echo rc=$?
wc -l $out
