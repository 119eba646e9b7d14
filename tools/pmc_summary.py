"""Average each counter per dispatch for the kernels of a pmc.sh run (all
kernels the pass collected, keyed by name without the argument list)."""
import collections
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
agg = collections.defaultdict(list)
for p in glob.glob(os.path.join(d, "p*", "run_counter_collection.csv")):
    for r in csv.DictReader(open(p)):
        n = r["Kernel_Name"].split("(")[0]
        agg[(n, r["Counter_Name"])].append(float(r["Counter_Value"]))
out = collections.defaultdict(dict)
for (k, c), v in sorted(agg.items()):
    out[k][c] = sum(v) / len(v)
print(json.dumps(out, indent=1))
