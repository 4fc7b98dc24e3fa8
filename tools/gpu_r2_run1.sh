set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 && \
timeout -k 10 120 python bench.py > gpurun_out/bench1.log 2>&1
echo exit=$?
