#!/bin/bash
# C2 roofline evidence under the timed condition (run via gpurun):
#   bash tools/measure_c2.sh TAG
# 1. tools/cal_fetch: known counts of random 16 B / 64 B reads (HBM- and
#    Infinity-Cache-resident buffers): timings, then a FETCH_SIZE pass and a
#    TCC request pass over the same binary (calibration of the counters for
#    the summary walk's access shape);
# 2. the default bench (two streams, two walks in flight) under a kernel
#    trace, no CPU baseline / latency / profile passes, so the last STEPS
#    k_get_sum launches are the timed steps (tools/step_timeline.py);
# 3. FETCH_SIZE and TCC request passes over k_get_sum in the same command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out/mc2_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
CAL=$R/tools/_build/cal_fetch
STEPS=50
B="$R/bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --profile-steps 0 --latency-steps 0"
timeout -k 10 120 $CAL > $OUT/cal.jsonl 2> $OUT/cal.err || exit $?
cat $OUT/cal.jsonl
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/cal_fetch -o run \
  -- $CAL > /dev/null 2> $OUT/cal_fetch.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --output-format csv \
  -d $OUT/cal_req -o run -- $CAL > /dev/null 2> $OUT/cal_req.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $B > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit $?
cat $OUT/trace_bench.json
python3 $R/tools/step_timeline.py $OUT/trace/run_kernel_trace.csv $STEPS k_get_sum \
  $OUT/trace_bench.json > $OUT/step_timeline.json || exit $?
cat $OUT/step_timeline.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_get_sum" --output-format csv \
  -d $OUT/pmc_fetch -o run -- python3 $B > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit $?
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex "k_get_sum" \
  --output-format csv -d $OUT/pmc_req -o run -- python3 $B > $OUT/pmc_req.json 2> $OUT/pmc_req.err || exit $?
find $OUT -name "*.csv" | head -40
timeout -k 10 300 python3 $R/tools/upper_stamps.py 26 4 > $OUT/upper_stamps.txt 2>&1 || exit $?
cat $OUT/upper_stamps.txt
