#!/usr/bin/env python3
"""Kernel statistics from a rocprofv3 --kernel-trace --stats database (rocpd SQLite, the
default output format): the same columns as rocprofv3's kernel_stats.csv, plus, for the
render kernel of bench.py (which alternates scenes 1 and 8 every step), a per-scene split by
dispatch order.

    python tools/rocpd_stats.py gpurun_out/prof_bench/bench_results.db > profiles/r01_bench_kernel_stats.csv
"""
import csv
import sqlite3
import sys

import numpy as np


def main(db):
    c = sqlite3.connect(db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    by = {}
    for name, s, e in rows:
        by.setdefault(name, []).append((e - s) / 1e3)          # ns -> us
    w = csv.writer(sys.stdout)
    w.writerow(["Name", "Calls", "TotalDurationUs", "AverageUs", "MinUs", "MaxUs", "Percentage"])
    total = sum(sum(v) for v in by.values())
    for name, d in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        d = np.array(d)
        w.writerow([name, len(d), round(d.sum(), 3), round(d.mean(), 3), round(d.min(), 3), round(d.max(), 3),
                    round(100 * d.sum() / total, 2)])
    for name, d in by.items():
        if "k_render" in name and len(d) % 2 == 0:
            d = np.array(d)
            for i, sid in enumerate((1, 8)):
                part = d[i::2]
                w.writerow([f"{name} [scene {sid}]", len(part), round(part.sum(), 3), round(part.mean(), 3),
                            round(part.min(), 3), round(part.max(), 3), ""])


if __name__ == "__main__":
    main(sys.argv[1])
