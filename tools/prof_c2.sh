set -o pipefail
mkdir -p gpurun_out
FOREMAST_PROFILE_CYCLES=gpurun_out/c2cyc.prof timeout -k 10 400 python -u benchmarks/bench_configs.py --config 2e2e --steps 20 --warmup 3 > gpurun_out/c2prof.log 2>&1 && \
python - <<'PY'
import pstats, io
s = io.StringIO()
p = pstats.Stats("gpurun_out/c2cyc.prof", stream=s); p.sort_stats("tottime"); p.print_stats(60)
p.sort_stats("cumulative"); p.print_stats(80)
open("gpurun_out/c2cyc.txt", "w").write(s.getvalue())
PY
