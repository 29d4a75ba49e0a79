"""Histogram of rocprofv3 kernel-trace durations by kernel and grid size (run on the GPU box; the raw trace has
one row per dispatch and is too large to bring back).

    python tools/trace_hist.py gpurun_out/prof/<name>_kernel_trace.csv > gpurun_out/trace_hist.txt
"""
import csv
import sys
from collections import defaultdict


def main():
    acc = defaultdict(lambda: [0, 0.0])
    for row in csv.DictReader(open(sys.argv[1])):
        name = row["Kernel_Name"].split("(")[0].replace("ccmi::", "")
        grid = int(row.get("Grid_Size") or row.get("Grid_Size_X") or 0)
        wg = int(row.get("Workgroup_Size") or row.get("Workgroup_Size_X") or 1)
        blocks = grid // max(1, wg)
        b = 1
        while b < blocks:
            b <<= 1
        dur = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) / 1000.0
        a = acc[(name, b)]
        a[0] += 1
        a[1] += dur
    print(f"{'kernel':20s} {'blocks<=':>8s} {'calls':>8s} {'avg us':>8s} {'total s':>8s}")
    for (name, b), (n, t) in sorted(acc.items()):
        print(f"{name:20s} {b:8d} {n:8d} {t / n:8.1f} {t / 1e6:8.3f}")


if __name__ == "__main__":
    main()
