#!/bin/bash
# A/B of library variants (via gpurun): for each sherman_amd/exp_<V>.so, copy
# it over libsherman_amd.so, run a kernel-trace of bench.py and print the
# per-kernel averages.  usage: bash tools/ab_libs.sh TAG "bench args" V1 V2 ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ARGS=$2; shift 2
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
cp $R/sherman_amd/libsherman_amd.so $OUT/orig.so
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  cp $R/sherman_amd/exp_$V.so $R/sherman_amd/libsherman_amd.so
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$V -o run \
    -- python3 $R/bench.py --no-cpu-baseline --latency-steps 0 --profile-steps 5 $ARGS \
    > $OUT/$V.json 2> $OUT/$V.err || { tail -20 $OUT/$V.err; exit 1; }
  python3 - $OUT/$V $V $OUT/$V.json <<'PY'
import csv, json, sys
from collections import defaultdict
d = json.load(open(sys.argv[3]))
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "ins", d["roofline"].get("insert_ms_per_launch"))
# per kernel: the mean of its last 20 dispatches (the timed / profile steps,
# not the build); kernels launched twice per step also split by parity
ds = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1] + "/run_kernel_trace.csv")):
    ds[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
for k, v in sorted(ds.items(), key=lambda x: -sum(t for _, t in x[1][-20:])):
    v.sort()
    last = [t for _, t in v[-20:]]
    m = sum(last) / len(last) / 1e3
    if m * len(last) < 20:
        continue
    ev = [t for _, t in v[-20:]][0::2]; od = [t for _, t in v[-20:]][1::2]
    print("   %-45s %8.2f us (n=%d; alternate %.2f / %.2f)" % (k[:45], m, len(v), sum(ev) / max(len(ev), 1) / 1e3, sum(od) / max(len(od), 1) / 1e3))
PY
done
cp $OUT/orig.so $R/sherman_amd/libsherman_amd.so
