#!/bin/bash
# Same-box A/B of another tree (a worktree, built in place: _ab/r04 by
# default) against this one (run via gpurun):
#   bash tools/ab_r04_r05.sh TAG [workloads] [worktree]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abr_${1:-r05}
WLS=${2:-c5 c2 c3}
ALT=${3:-_ab/r04}
mkdir -p $OUT
for i in 1 2; do
  for W in $WLS; do
    for side in r04 r05; do
      D=$R; [ $side = r04 ] && D=$R/$ALT
      (cd $D && timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline --latency-steps 0) \
        > $OUT/${W}_${side}_$i.json 2> $OUT/${W}_${side}_$i.err || { tail -20 $OUT/${W}_${side}_$i.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${W}_${side}_$i.json').read().strip().splitlines()[-1]); print('${W} ${side} $i', d['value'], d['ms_per_step'])"
    done
  done
done
