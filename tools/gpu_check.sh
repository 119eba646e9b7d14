#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke, C2 and C3 bench lines.
# usage (via gpurun): bash tools/gpu_check.sh TAG [skip-tests]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/check_$TAG
mkdir -p $OUT
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { cat $OUT/smoke.log; exit 1; }
  cat $OUT/smoke.log
fi
timeout -k 10 400 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
  || { tail -30 $OUT/bench_c2.err; exit 1; }
cat $OUT/bench_c2.json
timeout -k 10 400 python -u bench.py --workload c3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err \
  || { tail -30 $OUT/bench_c3.err; exit 1; }
cat $OUT/bench_c3.json
timeout -k 10 400 python -u bench.py --workload c5 > $OUT/bench_c5.json 2> $OUT/bench_c5.err \
  || { tail -30 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
