#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_fastpath_models.py -k "arrivals or fused or models_fast" > gpurun_out/r6_churn_tests.log 2>&1; rc=$?
tail -5 gpurun_out/r6_churn_tests.log
[ $rc -eq 0 ] && bash tools/gpu_r6_churn.sh
