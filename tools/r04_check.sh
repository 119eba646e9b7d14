#!/bin/bash
# Round-4 GPU pass: GPU tests + smoke, then the three bench lines.
# usage (via gpurun): bash tools/r04_check.sh TAG [skip-tests] [pytest -k expr]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r04}
OUT=$R/gpurun_out/check_$TAG
mkdir -p $OUT
cd $R
if [ "$2" != "skip-tests" ]; then
  K=()
  [ -n "$3" ] && K=(-k "$3")
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { cat $OUT/smoke.log; exit 1; }
  tail -2 $OUT/smoke.log
fi
for w in c2 c3 c5; do
  timeout -k 10 400 python -u bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err \
    || { tail -30 $OUT/bench_$w.err; exit 1; }
  python -c "import json,sys; d=json.loads(open('$OUT/bench_$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d.get('parity_vs_oracle'), d['roofline'].get('frac'), d['roofline'].get('request_frac'))"
done
