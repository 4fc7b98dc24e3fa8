#!/usr/bin/env python3
"""Summarise a rocprofv3 kernel trace (rocpd SQLite .db or kernel_trace.csv)
into a per-kernel table: calls, total/avg/min us, share of GPU time."""
from __future__ import annotations

import csv
import sqlite3
import sys
from collections import defaultdict
from pathlib import Path


def rows_from_db(p: Path):
    c = sqlite3.connect(str(p))
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name_col = "kernel_name" if "kernel_name" in cols else "name"
    for name, s, e in c.execute(f"select {name_col}, start, end from kernels"):
        yield name, (e - s) / 1e3


def rows_from_csv(p: Path):
    with open(p) as f:
        for r in csv.DictReader(f):
            yield r["Kernel_Name"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


def main() -> None:
    agg = defaultdict(list)
    for arg in sys.argv[1:]:
        root = Path(arg)
        for p in ([root] if root.is_file() else root.rglob("*")):
            if p.suffix == ".db":
                it = rows_from_db(p)
            elif p.name.endswith("kernel_trace.csv"):
                it = rows_from_csv(p)
            else:
                continue
            for n, us in it:
                agg[n].append(us)
    tot = sum(sum(v) for v in agg.values()) or 1.0
    print(f"{'kernel':70s} {'calls':>6s} {'total_us':>10s} {'avg_us':>9s} {'min_us':>9s} {'share':>6s}")
    for n, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        short = n if len(n) <= 70 else n[:67] + "..."
        print(f"{short:70s} {len(v):6d} {sum(v):10.1f} {sum(v)/len(v):9.1f} {min(v):9.1f} {100*sum(v)/tot:5.1f}%")


if __name__ == "__main__":
    main()
