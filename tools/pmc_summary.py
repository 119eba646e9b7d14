"""Average each counter per dispatch for the kernels of a pmc.sh run (all
kernels the pass collected, keyed by name without the argument list).
env PMC_LAST=K: only each kernel's last K dispatches (the timed steps, not
the tree build)."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
last = int(os.environ.get("PMC_LAST", "0"))
agg = collections.defaultdict(list)
for p in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
    per = collections.defaultdict(list)  # (kernel, counter) -> [(dispatch, value)]
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].split("(")[0]
        per[(n, r["Counter_Name"])].append((int(r.get("Dispatch_Id", 0) or 0),
                                            float(r["Counter_Value"])))
    for key, v in per.items():
        # one row per dispatch after summing any per-instance rows
        byd = collections.defaultdict(float)
        for di, x in v:
            byd[di] += x
        vals = [byd[di] for di in sorted(byd)]
        agg[key].extend(vals[-last:] if last else vals)
out = collections.defaultdict(dict)
for (k, c), v in sorted(agg.items()):
    out[k][c] = sum(v) / len(v)
print(json.dumps(out, indent=1))
