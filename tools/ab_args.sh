#!/bin/bash
# Generic A/B of bench.py argument sets on one workload, alternating:
#   bash tools/ab_args.sh TAG REPS "ARGS_A" "ARGS_B" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; REPS=$2; shift 2
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
cd $R
for r in $(seq 1 $REPS); do
  i=0
  for a in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python -u bench.py --no-cpu-baseline $a > $OUT/v${i}_$r.json 2> $OUT/v${i}_$r.err \
      || { tail -20 $OUT/v${i}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$OUT/v${i}_$r.json').read().strip().splitlines()[-1]); print('$a', $r, d['value'], d['ms_per_step'])"
  done
done
