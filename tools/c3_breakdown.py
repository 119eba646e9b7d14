"""Per-step kernel breakdown of a kernel trace (tools/profile_c3.sh, or
tools/profile.sh for C2): kernels from the first get walk on, averaged per
get walk (or per ANCHOR kernel / PER_STEP).
usage: python tools/c3_breakdown.py OUTDIR [ANCHOR [PER_STEP]]
  (C5: ANCHOR=k_range PER_STEP=2)"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1] + "/trace/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
anchor = sys.argv[2] if len(sys.argv) > 2 else "k_get<4, 1, 4, false>"
per = int(sys.argv[3]) if len(sys.argv) > 3 else 1
is_get = lambda r: anchor in r["Kernel_Name"]
t0 = min(int(r["Start_Timestamp"]) for r in rows if is_get(r))
c3 = [r for r in rows if int(r["Start_Timestamp"]) >= t0]
steps = sum(1 for r in c3 if is_get(r)) / per
span = (int(c3[-1]["End_Timestamp"]) - t0) / 1e3
agg = collections.defaultdict(lambda: [0, 0.0])
for r in c3:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    agg[r["Kernel_Name"][:80]][0] += 1
    agg[r["Kernel_Name"][:80]][1] += d
tot = 0.0
for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:24]:
    tot += d
    print(f"{d / steps:8.1f} us/step {c / steps:5.1f} calls  {n}")
print(f"steps {steps}  kernel sum/step {tot / steps:.1f} us  span/step {span / steps:.1f} us")
