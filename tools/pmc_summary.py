#!/usr/bin/env python3
"""Summarise rocprofv3 PMC databases: per kernel (name prefix), the mean
per-dispatch value of every collected counter (summed over the per-SE/XCD
instances of one dispatch) and the mean dispatch duration.

usage: tools/pmc_summary.py <dir-with-*_results.db> [...] [--kernel SUBSTR]
"""
from __future__ import annotations

import sqlite3
import sys
from collections import defaultdict
from pathlib import Path


def main() -> None:
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    want = ""
    if "--kernel" in sys.argv:
        want = sys.argv[sys.argv.index("--kernel") + 1]
        args = [a for a in args if a != want]
    per = defaultdict(lambda: defaultdict(float))     # (kernel, dispatch) -> counter -> value
    dur = {}
    for a in args:
        for db in Path(a).rglob("*_results.db"):
            c = sqlite3.connect(str(db))
            for name, disp, cnt, val, d in c.execute(
                    "select kernel_name, dispatch_id, counter_name, value, duration from counters_collection"):
                if want and want not in name:
                    continue
                nm = name.replace("(anonymous namespace)::", "")
                k = (nm.split("(")[0][:60], f"{db}:{disp}")
                per[k][cnt] += val
                dur[k] = d
    agg = defaultdict(lambda: defaultdict(list))
    for (kern, _), cs in per.items():
        for cnt, v in cs.items():
            agg[kern][cnt].append(v)
        agg[kern]["duration_us"].append(dur[(kern, _)] / 1e3)
    for kern, cs in agg.items():
        print(kern)
        for cnt, vs in sorted(cs.items()):
            print(f"    {cnt:28s} {sum(vs) / len(vs):16.4g}   (n={len(vs)})")


if __name__ == "__main__":
    main()
