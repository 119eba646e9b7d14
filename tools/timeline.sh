#!/bin/bash
# Kernel timeline of one bench step: bash tools/timeline.sh TAG ANCHOR [bench args]
# (rocprofv3 kernel trace; prints the launches between two ANCHOR kernels
# with their gaps, then the per-step breakdown)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ANCHOR=$2; shift 2
bash $R/tools/profile_args.sh "$TAG" "$ANCHOR" "$@" > $R/gpurun_out/prof_$TAG.breakdown || exit $?
python3 - "$R/gpurun_out/prof_$TAG/trace/run_kernel_trace.csv" "$ANCHOR" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if sys.argv[2] in r["Kernel_Name"]]
i0, i1 = idx[-3], idx[-2]
t0 = int(rows[i0]["Start_Timestamp"]); prev = t0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print("%8.1f gap %6.1f dur %6.1f  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3,
                                            r["Kernel_Name"][:70]))
    prev = e
PY
cat $R/gpurun_out/prof_$TAG.breakdown
