#!/bin/bash
# C5 step timeline under the timed condition + the request-ceiling
# calibration (run via gpurun): bash tools/diag_c5.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out/diag_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
STEPS=40
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run \
  -- python3 $R/bench.py --workload c5 --no-cpu-baseline --latency-steps 0 --profile-steps 0 \
  --steps $STEPS > $OUT/c5_trace.json 2> $OUT/c5_trace.err || exit $?
python3 $R/tools/c5_timeline.py $OUT/trace/run_kernel_trace.csv $STEPS $OUT/c5_trace.json \
  > $OUT/c5_timeline.json || exit $?
cat $OUT/c5_timeline.json
if [ "$2" = "cal" ]; then
  timeout -k 10 120 $R/tools/_build/cal_fetch > $OUT/cal.jsonl 2> $OUT/cal.err || exit $?
  cat $OUT/cal.jsonl
fi
cd $R
for W in c2 c3; do
  timeout -k 10 300 python3 -u bench.py --workload $W --no-cpu-baseline > $OUT/bench_$W.json 2> $OUT/bench_$W.err \
    || { tail -30 $OUT/bench_$W.err; exit 1; }
  cat $OUT/bench_$W.json
done
