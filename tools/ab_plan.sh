#!/bin/bash
# Range-scan plan check and A/B (run via gpurun): bash tools/ab_plan.sh TAG
# 1. the range / stale-directory / C5 GPU tests; 2. k_upper's phase and
# per-block clocks; 3. the C5 timeline with the directory plan on and off
# (SHM_RANGE_PLAN=0), same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-plan}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_c5.py -m gpu -x -v \
  -k "range or stale or c5" --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 \
  || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u tools/upper_stamps.py 26 3 > $OUT/upper_stamps.txt 2>&1 \
  || { cat $OUT/upper_stamps.txt; exit 1; }
cat $OUT/upper_stamps.txt
bash tools/c5_trace.sh $TAG/on || exit 1
SHM_RANGE_PLAN=0 bash tools/c5_trace.sh $TAG/off || exit 1
echo ab_plan done
