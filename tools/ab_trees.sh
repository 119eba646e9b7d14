#!/bin/bash
# Same-box A/B of worktrees (built in place) and this tree (run via gpurun):
#   bash tools/ab_trees.sh TAG "c5 c3" . _ab/base _ab/v77
# two alternating runs per tree and workload; one JSON line each under
# gpurun_out/abt_TAG/
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abt_${1:-x}
WLS=${2:-c5}
shift 2
mkdir -p $OUT
for i in 1 2; do
  for W in $WLS; do
    for T in "$@"; do
      n=$(echo $T | tr '/.' '__')
      (cd $R/$T && timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline --latency-steps 0) \
        > $OUT/${W}_${n}_$i.json 2> $OUT/${W}_${n}_$i.err || { tail -20 $OUT/${W}_${n}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${W}_${n}_$i.json').read().strip().splitlines()[-1]); print('${W} $T $i', d['value'], d['ms_per_step'], d['roofline'].get('range_ms_per_launch'))"
    done
  done
done
