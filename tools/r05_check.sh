#!/bin/bash
# Round-5 GPU pass (run via gpurun): GPU tests + smoke, the roofline pass of
# the three workloads, and the routed C2 get at world 1 over RCCL.
#   bash tools/r05_check.sh TAG [skip-tests] [skip-route]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05}
OUT=$R/gpurun_out/check_$TAG
mkdir -p $OUT
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
    > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
    || { cat $OUT/smoke.log; exit 1; }
  tail -1 $OUT/smoke.log
fi
if [ "$3" != "skip-route" ]; then
  timeout -k 10 300 python -u tools/route_c2.py 27 200 > $OUT/route_c2_27.log 2>&1 \
    || { tail -20 $OUT/route_c2_27.log; exit 1; }
  cat $OUT/route_c2_27.log
fi
bash tools/roofline_pass.sh $TAG c2 c3 c5 > $OUT/roofline.log 2>&1 || { tail -30 $OUT/roofline.log; exit 1; }
tail -8 $OUT/roofline.log
