#!/bin/bash
# GPU tests + k_upper stamps + a bench A/B of command-line variants (via gpurun):
#   bash tools/gpu_ab.sh TAG ROUNDS "common args" "variant 1" "variant 2" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1
OUT=$R/gpurun_out/gab_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u tools/upper_stamps.py 26 3 > $OUT/upper_stamps.txt 2>&1 || { cat $OUT/upper_stamps.txt; exit 1; }
grep -v "^   " $OUT/upper_stamps.txt
shift
bash tools/ab_args.sh $TAG "$@"
