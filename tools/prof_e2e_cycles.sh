set -o pipefail
FOREMAST_PROFILE_CYCLES=gpurun_out/c2cyc.prof timeout -k 10 400 python -u benchmarks/bench_configs.py --config 2e2e --steps 20 --warmup 3 > gpurun_out/c2prof.log 2>&1 && \
FOREMAST_PROFILE_CYCLES=gpurun_out/c4cyc.prof timeout -k 10 400 python -u benchmarks/bench_configs.py --config 4e2e --steps 20 --warmup 3 > gpurun_out/c4prof.log 2>&1 && \
FOREMAST_PROFILE_RESTART=gpurun_out/rscyc.prof timeout -k 10 500 python -u benchmarks/bench_configs.py --config 3e2e --steps 3 --warmup 1 --restart > gpurun_out/rsprof.log 2>&1 && \
python - <<'PY'
import pstats, io
for n in ("c2", "c4", "rs"):
    s = io.StringIO()
    p = pstats.Stats(f"gpurun_out/{n}cyc.prof", stream=s); p.sort_stats("tottime"); p.print_stats(45)
    p.sort_stats("cumulative"); p.print_stats(60)
    open(f"gpurun_out/{n}cyc.txt", "w").write(s.getvalue())
PY
