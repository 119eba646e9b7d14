#!/bin/bash
# C5 / C3 with the insert ordering confined to N CUs (run via gpurun):
#   bash tools/ab_cus.sh TAG "N ..." [workloads]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/cus_${1:-r05}
NS=${2:-"0 32 64 128"}
WLS=${3:-c5}
mkdir -p $OUT
cd $R
for W in $WLS; do
  for N in $NS; do
    for M in spread low; do
      [ $N = 0 ] && [ $M = low ] && continue
      timeout -k 10 300 python3 bench.py --workload $W --no-cpu-baseline --latency-steps 0 \
        --order-cus $N --order-cu-mode $M > $OUT/${W}_${N}_$M.json 2> $OUT/${W}_${N}_$M.err \
        || { tail -20 $OUT/${W}_${N}_$M.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$OUT/${W}_${N}_$M.json').read().strip().splitlines()[-1]); print('$W $N $M', d['value'], d['ms_per_step'])"
    done
  done
done
