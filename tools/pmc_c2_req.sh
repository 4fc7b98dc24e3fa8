#!/bin/bash
# Config 2 HBM traffic by request counts: TCC->EA read / write requests of the
# Holt-Winters grid fit, calibrated against a device copy of known bytes
# (tools/copy_calib.py).  Summaries: gpurun_out/pmc_c2_req.txt.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
C="TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
timeout -k 10 120 rocprofv3 --kernel-trace --pmc $C -d "$R/gpurun_out/pmc_copy_req" -o r -- \
  python3 "$R/tools/copy_calib.py" > "$R/gpurun_out/pmc_copy_req.log" 2>&1 || exit 1
timeout -k 10 150 rocprofv3 --kernel-trace --pmc $C -d "$R/gpurun_out/pmc_c2_req" -o r -- \
  python3 "$R/benchmarks/bench_configs.py" --config 2 --steps 2 --warmup 1 > "$R/gpurun_out/pmc_c2_req.log" 2>&1 || exit 1
cd "$R"
{ python3 tools/pmc_summary.py gpurun_out/pmc_copy_req --kernel copy; python3 tools/pmc_summary.py gpurun_out/pmc_c2_req --kernel hw2; } > gpurun_out/pmc_c2_req.txt
rm -rf gpurun_out/pmc_copy_req gpurun_out/pmc_c2_req
cat gpurun_out/pmc_c2_req.txt
