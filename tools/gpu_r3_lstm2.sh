#!/bin/bash
# Round 3: LSTM flow-kernel numerics + A/B; config 4e2e kernel stats (rocprofv3) and host profile
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_model_ops.py -m gpu -k "lstm_stack" > gpurun_out/lstm_r3_tests.log 2>&1 || { tail -30 gpurun_out/lstm_r3_tests.log; exit 1; }
tail -2 gpurun_out/lstm_r3_tests.log
timeout -k 10 200 python -u tools/lstm_stack_ab.py --tilings 4:2,4:1p,4:1f,2:1f > gpurun_out/lstm_r3_ab3.jsonl 2> gpurun_out/lstm_r3_ab3.err || { tail -20 gpurun_out/lstm_r3_ab3.err; exit 1; }
tail -1 gpurun_out/lstm_r3_ab3.jsonl
timeout -k 10 600 python tools/profile_3e2e.py --config 4e2e --steps 8 --warmup 2 --hpa-log-interval 300 > gpurun_out/host_c4e2e.txt 2>&1 || { tail -20 gpurun_out/host_c4e2e.txt; exit 1; }
grep -o '"span_ms_median_rank0": {[^}]*}' gpurun_out/host_c4e2e.txt
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_c4e2e" -o c4e2e -- \
    python3 "$R/benchmarks/bench_configs.py" --config 4e2e --steps 5 --warmup 2 --hpa-log-interval 300 > "$R/gpurun_out/prof_c4e2e.log" 2>&1
echo "prof rc=$?"
