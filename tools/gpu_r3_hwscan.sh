#!/bin/bash
# Round 3: time-parallel Holt-Winters scan fit -- GPU tests, A/B vs the serial kernel, config 2, kernel table
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -k "es_fit or es_update or hw_scan" > gpurun_out/hwscan_tests.log 2>&1 || { tail -40 gpurun_out/hwscan_tests.log; exit 1; }
tail -3 gpurun_out/hwscan_tests.log
timeout -k 10 300 python tools/hw_scan_ab.py --rows 40000 10000 --m 1440 288 1008 --methods ${HWSCAN_METHODS:-scan,serial} > gpurun_out/hwscan_ab.jsonl 2>gpurun_out/hwscan_ab.err || { tail -20 gpurun_out/hwscan_ab.err; exit 1; }
cat gpurun_out/hwscan_ab.jsonl
timeout -k 10 300 python benchmarks/bench_configs.py --config 2 > gpurun_out/hwscan_c2.jsonl 2>gpurun_out/hwscan_c2.err || { tail -20 gpurun_out/hwscan_c2.err; exit 1; }
cut -c1-400 gpurun_out/hwscan_c2.jsonl
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_hwscan -o c2 -- python benchmarks/bench_configs.py --config 2 > gpurun_out/hwscan_prof.log 2>&1 || { tail -20 gpurun_out/hwscan_prof.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_hwscan > gpurun_out/kernels_c2_hwscan.txt 2>&1; head -20 gpurun_out/kernels_c2_hwscan.txt
