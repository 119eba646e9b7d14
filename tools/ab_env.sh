#!/bin/bash
# Generic A/B of environment settings on one workload, alternating:
#   bash tools/ab_env.sh TAG WORKLOAD REPS "ENV_A" "ENV_B" ...  (each ENV_x: VAR=v[,VAR=v])
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; W=$2; REPS=$3; shift 3
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
cd $R
for r in $(seq 1 $REPS); do
  for e in "$@"; do
    name=$(echo "$e" | tr ',=/.' '____')
    env $(echo "$e" | tr ',' ' ') timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline $B_ARGS \
      > $OUT/${name}_$r.json 2> $OUT/${name}_$r.err || { tail -20 $OUT/${name}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/${name}_$r.json').read().strip().splitlines()[-1]); print('$e', $r, d['value'], d['ms_per_step'])"
  done
done
