set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u benchmarks/bench_configs.py --config 3e2e --steps 30 --warmup 3 > gpurun_out/c3e2e.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d gpurun_out/prof3e2e -o run -- python -u benchmarks/bench_configs.py --config 3e2e --steps 30 --warmup 3 > gpurun_out/c3e2e_prof.log 2>&1
echo exit=$?
