#!/bin/bash
# Same-box A/B of the round-4 tree (worktree _ab/r04, built in place) against
# this one (run via gpurun): bash tools/ab_r04_r05.sh TAG [workloads]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abr_${1:-r05}
WLS=${2:-c5 c2 c3}
mkdir -p $OUT
for i in 1 2; do
  for W in $WLS; do
    for side in r04 r05; do
      D=$R; [ $side = r04 ] && D=$R/_ab/r04
      (cd $D && timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline --latency-steps 0) \
        > $OUT/${W}_${side}_$i.json 2> $OUT/${W}_${side}_$i.err || { tail -20 $OUT/${W}_${side}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${W}_${side}_$i.json').read().strip().splitlines()[-1]); print('${W} ${side} $i', d['value'], d['ms_per_step'])"
    done
  done
done
