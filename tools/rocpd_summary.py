"""Summarise a rocprofv3 ``*_results.db`` (rocpd SQLite) kernel trace: per-kernel
count / total / mean, and -- given a once-per-cycle marker kernel -- the
kernels and device time of each steady cycle (between consecutive markers).

    python tools/rocpd_summary.py gpurun_out/prof_c2e2e/c2e2e_results.db \
        --marker es_band_step --cycles 8 > profiles/kernels_2e2e_r5.txt
"""
from __future__ import annotations

import argparse
import sqlite3
from collections import defaultdict


def _table(c, prefix: str) -> str:
    return [r[0] for r in c.execute("select name from sqlite_master where type='table' and name like ?",
                                    (prefix + "%",))][0]


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--marker", default="es_band_step", help="substring of a kernel launched once per cycle")
    ap.add_argument("--cycles", type=int, default=8, help="steady cycles to break down (the last N)")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    kd, ks = _table(c, "rocpd_kernel_dispatch"), _table(c, "rocpd_info_kernel_symbol")
    rows = c.execute(f"select d.start, d.end, s.kernel_name from {kd} d join {ks} s on d.kernel_id = s.id "
                     f"order by d.start").fetchall()
    print(f"# {a.db}: {len(rows)} dispatches")
    agg: dict = defaultdict(lambda: [0, 0.0])
    for s, e, n in rows:
        agg[n][0] += 1
        agg[n][1] += (e - s) * 1e-3
    print(f"{'count':>7} {'total_us':>11} {'mean_us':>9}  kernel")
    for n, (k, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:a.top]:
        print(f"{k:7d} {t:11.1f} {t / k:9.2f}  {n[:110]}")
    marks = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(marks) < 2:
        print(f"# marker {a.marker!r}: {len(marks)} dispatches, no cycle breakdown")
        return
    marks = marks[-(a.cycles + 1):]
    print(f"\n# steady cycles between consecutive {a.marker!r} dispatches (last {len(marks) - 1})")
    per: dict = defaultdict(lambda: [0, 0.0])
    for i0, i1 in zip(marks, marks[1:]):
        seg = rows[i0:i1]
        busy = sum((e - s) for s, e, _ in seg) * 1e-3
        span = (rows[i1][0] - rows[i0][0]) * 1e-6
        print(f"cycle: {len(seg)} kernels, device busy {busy:8.1f} us, marker-to-marker {span:8.2f} ms")
        for s, e, n in seg:
            per[n][0] += 1
            per[n][1] += (e - s) * 1e-3
    ncyc = len(marks) - 1
    print(f"\n{'per_cycle':>9} {'us/cycle':>9}  kernel")
    for n, (k, t) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"{k / ncyc:9.2f} {t / ncyc:9.1f}  {n[:110]}")


if __name__ == "__main__":
    main()
