#!/bin/bash
# Driver-shaped headline runs (--steps 20 --warmup 5, as the round-end driver
# calls bench.py) next to a long run on the same box: does a short run pay
# for idle clocks / cold state?
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/short_vs_long.jsonl
rm -f $out
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 200 python bench.py "$@" 2>gpurun_out/short_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
b short1 --gpus 1 --steps 20 --warmup 5 &&
b long1 --steps 300 --warmup 30 &&
b short2 --gpus 1 --steps 20 --warmup 5 &&
b long2 --steps 300 --warmup 30 &&
b short3 --gpus 1 --steps 20 --warmup 5
echo rc=$?
cat $out
