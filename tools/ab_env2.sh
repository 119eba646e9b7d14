#!/bin/bash
# Same-box A/B of a library environment switch (run via gpurun):
#   bash tools/ab_env2.sh TAG VAR "v1 v2 ..." [workload] [reps]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abenv_${1:-r05}
VAR=$2
VALS=$3
W=${4:-c5}
REPS=${5:-2}
mkdir -p $OUT
cd $R
for i in $(seq 1 $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline --latency-steps 0 \
      > $OUT/${W}_${v}_$i.json 2> $OUT/${W}_${v}_$i.err || { tail -20 $OUT/${W}_${v}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${W}_${v}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$W $VAR=$v $i', d['value'], d['ms_per_step'], r.get('range_ms_per_launch'))"
  done
done
