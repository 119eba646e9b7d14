#!/bin/bash
# A/B (run via gpurun): bash tools/r05_ab2.sh TAG
#   C5 order-first 0/1 and C3/C5 with 4 vs 8 directory entries per page
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab2_${1:-r05}
mkdir -p $OUT
cd $R
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --latency-steps 0 "$@" > $OUT/$n.json 2> $OUT/$n.err \
    || { tail -20 $OUT/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'])"
}
for i in 1 2; do
  run c5_of0_$i --workload c5 --order-first 0
  run c5_of1_$i --workload c5 --order-first 1
done
for i in 1 2; do
  run c5_x2_$i --workload c5 --dir-extra-bits 2
  run c5_x3_$i --workload c5 --dir-extra-bits 3
  run c3_x2_$i --workload c3 --dir-extra-bits 2
  run c3_x3_$i --workload c3 --dir-extra-bits 3
done
