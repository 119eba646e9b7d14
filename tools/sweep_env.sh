#!/bin/bash
# Run the C2 bench once per environment setting and print the walk timing.
# usage: [SWEEP_ARGS="--workload c3"] bash tools/sweep_env.sh TAG "VAR=a" "VAR=b" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/sweep_$TAG
mkdir -p $OUT
cd $R
i=0
for setting in "$@"; do
  i=$((i+1))
  env $setting timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 $SWEEP_ARGS \
    > $OUT/s$i.json 2> $OUT/s$i.err || { tail -20 $OUT/s$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/s$i.json')); r=d['roofline']; print('$setting', d['value'], d['ms_per_step'], r['walk_ms_per_launch'], r['order_ms_per_launch'], r['frac'])"
done
