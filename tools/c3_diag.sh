#!/bin/bash
# C3 regression hunt: bench with each new default switched off, then a kernel
# trace of the default.  usage (via gpurun): bash tools/c3_diag.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-c3d}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
B="bench.py --workload c3 --no-cpu-baseline --steps 100 --latency-steps 0 --profile-steps 0"
for v in "X=1" "SHM_TILE_MODE=0" "SHM_DIR_READ_PHASE=0" "SHM_UPPER_PRELOCK=0"; do
  env $v timeout -k 10 300 python -u $B > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -20 $OUT/b_$v.err; exit 1; }
  python -c "import json; d=json.loads(open('$OUT/b_$v.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['ms_per_step'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $R/$B > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit 1
python3 - <<PY
import csv, collections
rows = list(csv.DictReader(open("$OUT/trace/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
last = rows[-400:]
for r in last[-40:]:
    print(r["Kernel_Name"][:50], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0, int(r["Start_Timestamp"]) // 1000 % 10000000)
PY
