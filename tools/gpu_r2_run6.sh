set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_model_ops.py tests/test_canary_ops.py tests/test_fastpath.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests_num.log 2>&1
echo tests=$?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $R/gpurun_out/pmc_calib_fetch -o r -- python3 $R/tools/fetch_calib.py > $R/gpurun_out/pmc_calib_fetch.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_calib_fetch > $R/gpurun_out/pmc_calib_fetch.txt && rm -rf $R/gpurun_out/pmc_calib_fetch && \
timeout -k 10 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_EA0_RDREQ_sum -d $R/gpurun_out/pmc_calib_rd -o r -- python3 $R/tools/fetch_calib.py > $R/gpurun_out/pmc_calib_rd.log 2>&1 && \
python3 $R/tools/pmc_summary.py $R/gpurun_out/pmc_calib_rd > $R/gpurun_out/pmc_calib_rd.txt && rm -rf $R/gpurun_out/pmc_calib_rd
echo exit=$?
