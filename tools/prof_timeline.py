#!/usr/bin/env python3
"""Raw kernel / memory-copy timeline of the last events of a rocprofv3 trace
(``--kernel-trace [--memory-copy-trace] --output-format csv``): start, end and
duration of each event in microseconds relative to the first one printed.
Shows which stream is the critical path of a tick and how large the
inter-kernel and launch gaps are (profiles/tick_timeline_*.txt).

usage: prof_timeline.py <trace dir> [--last 16]
"""
from __future__ import annotations

import argparse
import csv
from pathlib import Path


def load(root: Path):
    ev = []
    for p in root.rglob("*.csv"):
        if p.name.endswith("kernel_trace.csv"):
            with open(p) as f:
                ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0][-40:])
                       for r in csv.DictReader(f)]
        elif "memory_copy" in p.name:
            with open(p) as f:
                ev += [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "memcpy " + r.get("Direction", ""))
                       for r in csv.DictReader(f)]
    ev.sort()
    return ev


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--last", type=int, default=16)
    a = ap.parse_args()
    ev = load(Path(a.path))[-a.last:]
    if not ev:
        print("no events")
        return
    t0 = ev[0][0]
    print(f"{'event':44s} {'start_us':>9s} {'end_us':>9s} {'dur_us':>8s}")
    for s, e, n in ev:
        print(f"{n:44s} {(s - t0) / 1e3:9.1f} {(e - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f}")


if __name__ == "__main__":
    main()
