"""Kernel time summary from a rocprofv3 rocpd database (ROCm 7 default output).

    python tools/rocpd_stats.py OUT/run_results.db [--runs R] [--top 30]

Per kernel: total us, calls, share; with --runs the totals are also divided by the number of
identical runs the traced program made (e.g. 1 warm-up + 2 timed = 3).
"""
import argparse
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument("db")
ap.add_argument("--runs", type=int, default=1)
ap.add_argument("--top", type=int, default=30)
a = ap.parse_args()
c = sqlite3.connect(a.db)
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
name = "kernel_name" if "kernel_name" in cols else ("name" if "name" in cols else None)
rows = c.execute(f"select {name}, start, end from kernels").fetchall()
tot, cnt = defaultdict(float), defaultdict(int)
for n, s, e in rows:
    tot[n] += (e - s) / 1e3
    cnt[n] += 1
allt = sum(tot.values())
print(f"{len(rows)} dispatches, {allt:.1f} us total ({allt / a.runs:.1f} us per run over {a.runs} runs)")
for n, t in sorted(tot.items(), key=lambda x: -x[1])[:a.top]:
    print(f"{t / a.runs:10.1f} us/run  x{cnt[n] / a.runs:6.1f}  {100 * t / allt:5.1f}%  {n[:110]}")
