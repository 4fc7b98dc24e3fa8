#!/bin/bash
# PMC counters of the Holt-Winters fits at the config-2 shape (tools/hw_scan_ab.py:
# hw_scan_fit_kernel = time-parallel scan, hw2_fit_kernel = serial packed fp16
# scratch), two passes of <= 8 SQ counters, kernel-trace + counters only.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
set -e
A="--rows 40000 --m ${PMC_M:-1440} --reps 2 --methods ${PMC_METHODS:-scan,serial}"
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM \
  SQ_BUSY_CYCLES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/pmc_hwscan_a" -o a -- python3 "$R/tools/hw_scan_ab.py" $A > "$R/gpurun_out/pmc_hwscan_a.log" 2>&1
timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_WAIT_ANY \
  SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_SALU \
  -d "$R/gpurun_out/pmc_hwscan_b" -o b -- python3 "$R/tools/hw_scan_ab.py" $A > "$R/gpurun_out/pmc_hwscan_b.log" 2>&1
cd "$R" && python3 tools/pmc_summary.py gpurun_out/pmc_hwscan_a gpurun_out/pmc_hwscan_b --kernel fit_kernel > gpurun_out/pmc_hwscan.txt
rm -rf gpurun_out/pmc_hwscan_a gpurun_out/pmc_hwscan_b
echo done
