#!/bin/bash
# Kernel-trace stats of a mixed workload: bash tools/profile_c3.sh TAG [c3|c5]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-c3}
WL=${2:-c3}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $R/bench.py --workload $WL --steps 20 --warmup 3 --no-cpu-baseline --profile-steps 0 \
  > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 - $OUT <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1] + "/trace/run_kernel_stats.csv")))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:25]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:90]}')
PY
