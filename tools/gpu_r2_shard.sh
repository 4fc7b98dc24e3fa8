#!/bin/bash
# The per-rank shard of an 8-GPU strong-scaling run (1,250 services) on one
# GPU: pipeline depth 2 vs 3, with the publish going through a real world-1
# RCCL group (--rccl-self: the all_gather_into_tensor host path + kernel each
# step), at the driver's step count and at a long count.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
out=gpurun_out/shard_probe.jsonl
rm -f $out
b() { tag=$1; shift; echo "== $tag" >&2; timeout -k 10 200 python bench.py "$@" 2>gpurun_out/shard_$tag.err | grep '^{' | sed "s/^{/{\"tag\": \"$tag\", /" >> $out; }
S="--services 1250"
b d2 $S --steps 2000 --warmup 100 --pipeline 2 &&
b d2rccl $S --steps 2000 --warmup 100 --pipeline 2 --rccl-self &&
b d3rccl $S --steps 2000 --warmup 100 --pipeline 3 --rccl-self &&
b d4rccl $S --steps 2000 --warmup 100 --pipeline 4 --rccl-self &&
b d2rccl_short $S --steps 20 --warmup 5 --pipeline 2 --rccl-self &&
b d3rccl_short $S --steps 20 --warmup 5 --pipeline 3 --rccl-self
echo rc=$?
cat $out
