"""Kernel durations from a rocprofv3 kernel trace, grouped by name, grid,
workgroup and LDS size: python tools/ktrace_stats.py run_kernel_trace.csv"""
import collections
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    d = collections.defaultdict(list)
    for r in rows:
        key = (r["Kernel_Name"][:40], r.get("Grid_Size_X", r.get("Grid_Size")),
               r.get("Workgroup_Size_X", r.get("Workgroup_Size")), r.get("LDS_Block_Size", r.get("Lds_Size")))
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
    for k, v in d.items():
        v = sorted(v)
        print(k, "p50 %.2f us  min %.2f" % (v[len(v) // 2], v[0]))


if __name__ == "__main__":
    main()
