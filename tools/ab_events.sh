#!/bin/bash
# Ordering events without system-scope fences (run via gpurun):
#   bash tools/ab_events.sh TAG
# 1. the GPU tests and 2. the C5 kernel timeline, both with device-scope events
# (SHM_EVENT_SYSFENCE=0; the library default is HIP's events); 3. C2 / C3 / C5 bench lines with device-scope events and
# with the default HIP events (SHM_EVENT_SYSFENCE=1), alternating, same box.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ev}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
SHM_EVENT_SYSFENCE=0 timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
SHM_EVENT_SYSFENCE=0 bash tools/c5_trace.sh $TAG/dev || exit 1
for W in c5 c3 c2; do
  for F in 0 1; do
    SHM_EVENT_SYSFENCE=$F timeout -k 10 300 python3 -u bench.py --workload $W --no-cpu-baseline \
      --latency-steps 0 > $OUT/bench_${W}_sys$F.json 2> $OUT/bench_${W}_sys$F.err \
      || { tail -30 $OUT/bench_${W}_sys$F.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      $OUT/bench_${W}_sys$F.json "$W sysfence=$F"
  done
done
echo ab_events done
