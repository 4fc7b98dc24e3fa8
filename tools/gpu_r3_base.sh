#!/bin/bash
# Round-3 start: GPU tests, smoke, driver-shaped bench, every BASELINE config
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/r3_base.jsonl
rm -f $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_r3_base.log 2>&1 || { tail -30 gpurun_out/gputests_r3_base.log; exit 1; }
tail -1 gpurun_out/gputests_r3_base.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_r3.log 2>&1 || exit 1
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 300 "$@" 2>gpurun_out/r3b_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b driver python bench.py --gpus 1 --steps 20 --warmup 5 &&
b c2 python benchmarks/bench_configs.py --config 2 &&
b c3e2e python benchmarks/bench_configs.py --config 3e2e &&
b c4 python benchmarks/bench_configs.py --config 4 &&
b c4mv python benchmarks/bench_configs.py --config 4 --hidden 256 --layers 2 --multivariate &&
b c5 python benchmarks/bench_configs.py --config 5
echo rc=$?
cat $out
