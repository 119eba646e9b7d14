#!/bin/bash
# Run the C2 bench once per argument set and print the walk timing.
# usage: bash tools/sweep_args.sh TAG "--batch-log2 21" "--keys-log2 24" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/sweepa_$TAG
mkdir -p $OUT
cd $R
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 30 --warmup 5 $args \
    > $OUT/s$i.json 2> $OUT/s$i.err || { tail -20 $OUT/s$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/s$i.json')); r=d['roofline']; print('$args', d['value'], d['ms_per_step'], r['walk_ms_per_launch'], r['order_ms_per_launch'], r['frac'])"
done
