#!/bin/bash
# One GPU-box pass for a round's record (run via gpurun):
#   bash tools/final_check.sh TAG
# 1. GPU tests + smoke; 2. the three bench lines with the CPU baseline;
# 3. C2 under the timed condition: kernel trace of the default two-stream
#    run (tools/step_timeline.py) and the walk's FETCH / TCC request passes;
# 4. C3 and C5: kernel trace + FETCH_SIZE / WRITE_SIZE passes
#    (tools/profile_write.sh, folded by tools/write_summary.py).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r03}
OUT=$R/gpurun_out/final_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -60 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
  || { cat $OUT/smoke.log; exit 1; }
cat $OUT/smoke.log
for W in c2 c3 c5; do
  timeout -k 10 500 python -u bench.py --workload $W > $OUT/bench_$W.json 2> $OUT/bench_$W.err \
    || { tail -30 $OUT/bench_$W.err; exit 1; }
  cat $OUT/bench_$W.json
done
cd /tmp && export TMPDIR=/tmp
STEPS=50
B="$R/bench.py --steps $STEPS --warmup 5 --no-cpu-baseline --profile-steps 0 --latency-steps 0"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c2_trace -o run \
  -- python3 $B > $OUT/c2_trace_bench.json 2> $OUT/c2_trace_bench.err || exit $?
python3 $R/tools/step_timeline.py $OUT/c2_trace/run_kernel_trace.csv $STEPS k_get_sum \
  $OUT/c2_trace_bench.json > $OUT/c2_step_timeline.json || exit $?
cat $OUT/c2_step_timeline.json
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_get_sum" --output-format csv \
  -d $OUT/c2_pmc_fetch -o run -- python3 $B > /dev/null 2> $OUT/c2_pmc_fetch.err || exit $?
timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-include-regex "k_get_sum" \
  --output-format csv -d $OUT/c2_pmc_req -o run -- python3 $B > /dev/null 2> $OUT/c2_pmc_req.err || exit $?
cd $R
bash tools/profile_write.sh $TAG c5 > $OUT/pw_c5.log 2>&1 || { tail -20 $OUT/pw_c5.log; exit 1; }
bash tools/profile_write.sh $TAG c3 > $OUT/pw_c3.log 2>&1 || { tail -20 $OUT/pw_c3.log; exit 1; }
echo final_check done
