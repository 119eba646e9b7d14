"""Per-kernel statistics of a bench window (between the two shm__mark
dispatches) in a rocprofv3 kernel trace: calls, average duration, and the
average start-to-start spacing per step of each kernel.
usage: python tools/window_stats.py run_kernel_trace.csv"""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Dispatch_Id"]))
m = [i for i, r in enumerate(rows) if "k_mark" in r["Kernel_Name"]]
w = rows[m[0] + 1:m[1]]
span = (max(int(r["End_Timestamp"]) for r in w) - min(int(r["Start_Timestamp"]) for r in w)) / 1e3
agg = collections.defaultdict(list)
for r in w:
    agg[r["Kernel_Name"].split("(")[0].replace("void ", "")].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
steps = max((len(v) for k, v in agg.items() if "k_upper" in k),
            default=max(len(v) for v in agg.values()))
print(f"window {span:.1f} us, {steps} steps, {span / steps:.1f} us/step")
for k, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
    print(f"{k[:44]:44s} {len(v):5d} {sum(v) / len(v):8.2f} us  {sum(v) / steps:8.2f} us/step")
