#!/usr/bin/env python3
"""Per-kernel dispatch statistics from a rocprofv3 --kernel-trace CSV
(<dir>/<name>_kernel_trace.csv): count, mean, median, min, max in us, and
the median over the last TAIL dispatches of each kernel (the interleaved /
steady part of a run whose first launches sit in the DVFS start-up window,
DESIGN.md §5.1). rocprofv3 --stats gives only mean/min/max per kernel.

  python scripts/trace_medians.py TRACE.csv [TAIL] > summary.json
"""
import csv
import json
import re
import sys

import numpy as np


def main():
    path = sys.argv[1]
    tail = int(sys.argv[2]) if len(sys.argv) > 2 else 48
    per = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            name = re.sub(r"\(.*", "", row["Kernel_Name"])  # drop the argument list
            us = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000.0
            per.setdefault(name, []).append((int(row["Start_Timestamp"]), us, row["Grid_Size_X"]))
    out = {}
    for name, rows in per.items():
        rows.sort()
        t = np.array([u for _, u, _ in rows])
        out[name] = {"count": len(t), "mean_us": round(float(t.mean()), 2), "median_us": round(float(np.median(t)), 2),
                     "min_us": round(float(t.min()), 2), "max_us": round(float(t.max()), 2),
                     f"median_last_{tail}_us": round(float(np.median(t[-tail:])), 2),
                     "grids": sorted({g for _, _, g in rows})[:4]}
    print(json.dumps({"trace": path, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
