#!/bin/bash
# Round 6 evidence pass: (1) headline PMC with the TCC->EA read requests
# (bytes from TCC_EA0_RDREQ / _32B / TCC_BUBBLE = 128-B requests), (2) the
# H = 256 x 2 stacked-LSTM PMC passes, (3) a 2-rank 2e2e brain cycle with the
# ranks' exchange on the device board vs the TCPStore mailbox (two ranks on
# the box's one GPU, gloo world, HIP IPC board).
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > "$R/gpurun_out/ev_avail.txt" 2>&1 || true
C="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
grep -q "TCC_BUBBLE" "$R/gpurun_out/ev_avail.txt" && C="$C TCC_BUBBLE_sum"
echo "tcc counters: $C"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $C GRBM_GUI_ACTIVE -d "$R/gpurun_out/ev_pmc_tcc" -o r -- \
  python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/ev_pmc_tcc.log" 2>&1 || { echo tcc failed; tail -5 "$R/gpurun_out/ev_pmc_tcc.log"; exit 1; }
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/ev_pmc_tcc" > "$R/gpurun_out/ev_pmc_tcc.txt" && rm -rf "$R/gpurun_out/ev_pmc_tcc"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE \
  -d "$R/gpurun_out/ev_pmc_sq" -o r -- python3 "$R/bench.py" --steps 5 --warmup 2 > "$R/gpurun_out/ev_pmc_sq.log" 2>&1 || { echo sq failed; exit 1; }
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/ev_pmc_sq" > "$R/gpurun_out/ev_pmc_sq.txt" && rm -rf "$R/gpurun_out/ev_pmc_sq"
echo "headline pmc done"
cd "$R"
PMC_TILINGS=4:2p bash tools/pmc_lstm_stack.sh > gpurun_out/ev_lstm_pmc.log 2>&1 || { echo lstm pmc failed; tail -5 gpurun_out/ev_lstm_pmc.log; exit 1; }
rm -rf gpurun_out/pmc_lstm_stack_a gpurun_out/pmc_lstm_stack_b
timeout -k 10 120 python -u tools/lstm_stack_ab.py --tilings 4:2p > gpurun_out/ev_lstm_ab.log 2>&1 || { echo lstm ab failed; exit 1; }
echo "lstm done"
for ex in mailbox board; do
  B=""; [ $ex = board ] && B="--board"
  FOREMAST_DIST_BACKEND=gloo FOREMAST_SHARE_GPU=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $((29700 + RANDOM % 200)) \
    benchmarks/bench_configs.py --config 2e2e --store sqlite --steps 40 --warmup 5 $B > gpurun_out/ev_2r_$ex.log 2>&1 \
    || { echo "2-rank $ex failed"; tail -20 gpurun_out/ev_2r_$ex.log; exit 1; }
  grep '^{' gpurun_out/ev_2r_$ex.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$ex', d['rank_exchange'], round(d['ms_per_step'],3), d.get('span_ms_median_rank0'))"
done
