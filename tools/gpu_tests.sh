#!/bin/bash
# GPU tests + smoke on the box (run via gpurun): bash tools/gpu_tests.sh TAG [pytest -k expr]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out/tests_$TAG
mkdir -p $OUT
cd $R
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
  > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -5 $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
