"""Summarise a rocprofv3 kernel-trace CSV: mean / min duration per (kernel, grid size).

    python tools/ktrace_summary.py <kernel_trace.csv> [name-substring ...]
"""
import csv
import statistics
import sys
from collections import defaultdict


def main():
    path, keys = sys.argv[1], sys.argv[2:]
    rows = defaultdict(list)
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if keys and not any(k in name for k in keys):
                continue
            grid = r.get("Grid_Size_X") or r.get("Grid_Size")
            wg = r.get("Workgroup_Size_X") or r.get("Workgroup_Size")
            dur = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            short = name.replace("(anonymous namespace)::", "").replace("void ", "")
            rows[(short.split("(")[0][:60], grid, wg)].append(dur)
    for (name, grid, wg), ds in sorted(rows.items()):
        print(f"{name:60s} grid={grid:>8s} wg={wg:>4s} n={len(ds):4d} "
              f"median={statistics.median(ds):9.2f}us min={min(ds):9.2f}us")


if __name__ == "__main__":
    main()
