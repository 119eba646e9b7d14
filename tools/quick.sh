#!/bin/bash
# Quick GPU pass after a kernel change (via gpurun): GPU parity tests, then
# bench lines without the CPU baseline.  usage: bash tools/quick.sh TAG [wl ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-q}
shift
OUT=$R/gpurun_out/quick_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
for wl in "${@:-c2 c3 c5}"; do
  timeout -k 10 300 python -u bench.py --workload $wl --no-cpu-baseline --latency-steps 0 \
    > $OUT/bench_$wl.json 2> $OUT/bench_$wl.err || { tail -30 $OUT/bench_$wl.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], d['ms_per_step'], d['host_issue_ms_per_step'], r['frac'], r.get('insert_ms_per_launch'), r.get('upsert_ms_per_launch'), r.get('range_ms_per_launch'), r.get('walk_ms_per_launch'))" $OUT/bench_$wl.json $wl
done
