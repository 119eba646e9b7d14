#!/bin/bash
# tests + quick benches (run via gpurun): bash tools/gpu_quick.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out/quick_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -80 $OUT/pytest_gpu.log; exit 1; }
tail -5 $OUT/pytest_gpu.log
timeout -k 10 300 python3 -u tools/upper_stamps.py 26 3 > $OUT/upper_stamps.txt 2>&1 || { cat $OUT/upper_stamps.txt; exit 1; }
cat $OUT/upper_stamps.txt
for W in c2 c5; do
  timeout -k 10 300 python3 -u bench.py --workload $W --no-cpu-baseline > $OUT/bench_$W.json 2> $OUT/bench_$W.err \
    || { tail -30 $OUT/bench_$W.err; exit 1; }
  cat $OUT/bench_$W.json
done
