set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
# multi-rank rehearsal on one GPU: bench.py spawns its own ranks (no launcher),
# gloo between ranks that share cuda:0 (RCCL refuses two ranks per device)
FOREMAST_DIST_BACKEND=gloo FOREMAST_DEVICE_INDEX=0 timeout -k 10 240 python bench.py --gpus 2 --steps 50 --warmup 5 > gpurun_out/rehearse2.log 2>&1
echo r2=$?
FOREMAST_DIST_BACKEND=gloo FOREMAST_DEVICE_INDEX=0 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 50 --warmup 5 > gpurun_out/rehearse4.log 2>&1
echo r4=$?
