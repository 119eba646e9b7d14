#!/bin/bash
# Early splits (upsert.hip) on vs off: GPU tests, then C5 and C3 bench lines
# with SHM_EARLY_SPLIT=1 (default) and 0, alternating.
# usage (via gpurun): bash tools/ab_early.sh TAG [reps] [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-early}
REPS=${2:-2}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
cd $R
if [ "$3" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
run() {  # name workload rep env...
  local name=$1 w=$2 r=$3; shift 3
  env "$@" timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline \
    > $OUT/${name}_$r.json 2> $OUT/${name}_$r.err || { tail -20 $OUT/${name}_$r.err; return 1; }
  python -c "import json; d=json.loads(open('$OUT/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', $r, d['value'], d['ms_per_step'], d.get('parity_vs_oracle'))"
}
for r in $(seq 1 $REPS); do
  run c5_early c5 $r SHM_EARLY_SPLIT=1 && run c5_late c5 $r SHM_EARLY_SPLIT=0 || exit 1
done
run c3_early c3 1 SHM_EARLY_SPLIT=1 && run c3_late c3 1 SHM_EARLY_SPLIT=0
