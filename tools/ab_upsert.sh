#!/bin/bash
# Upsert kernel variants (SHM_UPSERT_IL=0/1/2) on C5, against SHM_EARLY_SPLIT=0,
# then the early-split GPU tests under each variant.
# usage (via gpurun): bash tools/ab_upsert.sh TAG [reps] [workload]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-il}
REPS=${2:-2}
W=${3:-c5}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
cd $R
run() {  # name rep env...
  local name=$1 r=$2; shift 2
  env "$@" timeout -k 10 300 python -u bench.py --workload $W --no-cpu-baseline \
    > $OUT/${name}_$r.json 2> $OUT/${name}_$r.err || { tail -20 $OUT/${name}_$r.err; return 1; }
  python -c "import json; d=json.loads(open('$OUT/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', $r, d['value'], d['ms_per_step'])"
}
for m in 0 1 2; do
  SHM_UPSERT_IL=$m timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 \
    --timeout-method thread -k "early or random_batches or mixed_zipf" > $OUT/pytest_il$m.log 2>&1 \
    || { tail -40 $OUT/pytest_il$m.log; exit 1; }
  echo "il$m tests: $(tail -1 $OUT/pytest_il$m.log)"
done
for r in $(seq 1 $REPS); do
  run il0 $r SHM_UPSERT_IL=0 && run il1 $r SHM_UPSERT_IL=1 && run il2 $r SHM_UPSERT_IL=2 &&
  run late $r SHM_EARLY_SPLIT=0 || exit 1
done
for m in 0 1 2; do
  SHM_UPSERT_IL=$m timeout -k 10 300 python -u tools/upper_stamps.py 26 1 > $OUT/stamps_il$m.log 2>&1 \
    || { tail -20 $OUT/stamps_il$m.log; exit 1; }
  echo "il$m: $(grep -m1 'upsert blocks' $OUT/stamps_il$m.log)"
done
