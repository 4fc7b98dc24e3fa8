#!/bin/bash
# Multi-rank main() path on one GPU (gloo between ranks sharing cuda:0): the
# warm-up step count every rank derives from MAX-reduced timings must agree,
# or the collectives of the extra warm-up steps would not pair up
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FOREMAST_DIST_BACKEND=gloo FOREMAST_DEVICE_INDEX=0 timeout -k 10 240 python bench.py --gpus 2 --steps 20 --warmup 5 > gpurun_out/rehearse2_warm.log 2>&1 &&
FOREMAST_DIST_BACKEND=gloo FOREMAST_DEVICE_INDEX=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 20 --warmup 5 > gpurun_out/rehearse4_warm.log 2>&1
echo rc=$?
grep '^{' gpurun_out/rehearse2_warm.log gpurun_out/rehearse4_warm.log | cut -c1-400
