set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c2 -o r -- python3 $R/benchmarks/bench_configs.py --config 2 --steps 3 --warmup 1 > $R/gpurun_out/prof_c2.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/prof_c2 > $R/gpurun_out/prof_c2.txt; \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $R/gpurun_out/pmc_c2i -o r -- python3 $R/benchmarks/bench_configs.py --config 2 --steps 1 --warmup 1 > $R/gpurun_out/pmc_c2i.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_c2i > $R/gpurun_out/pmc_c2i.txt && rm -rf $R/gpurun_out/pmc_c2i; \
timeout -k 10 200 rocprofv3 --kernel-trace --pmc SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE TCC_EA0_RDREQ_sum -d $R/gpurun_out/pmc_c2b -o r -- python3 $R/benchmarks/bench_configs.py --config 2 --steps 1 --warmup 1 > $R/gpurun_out/pmc_c2b.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_c2b > $R/gpurun_out/pmc_c2b.txt && rm -rf $R/gpurun_out/pmc_c2b
echo exit=$?
