#!/bin/bash
# Per-kernel average durations (rocprofv3 --kernel-trace --stats) of one bench
# line, for an A/B of builds or settings:
#   bash tools/kstats.sh TAG WORKLOAD [ENV=VAL ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; W=$2; shift 2
OUT=$R/gpurun_out/ks_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run \
  -- python3 $R/bench.py --workload $W --no-cpu-baseline --latency-steps 0 --profile-steps 0 \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/run_kernel_stats.csv", recursive=True)[0]
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%-40s calls %6s avg %8.1f us  total %8.1f ms" % (r["Name"].split("(")[0][-40:], r["Calls"],
          float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6))
PY
