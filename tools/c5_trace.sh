#!/bin/bash
# C5 timed-step kernel timeline (run via gpurun):
#   bash tools/c5_trace.sh TAG [extra bench args...]
# A plain bench line first (no profiler), then a kernel trace of the same
# command folded by tools/c5_timeline.py (per-kernel time per step, the
# scan / ordering / tree chain, device idle).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-c5t}
shift
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
STEPS=40
B="$R/bench.py --workload c5 --no-cpu-baseline --latency-steps 0 --profile-steps 0 --steps $STEPS $*"
timeout -k 10 300 python3 -u $B > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run \
  -- python3 $B > $OUT/trace_bench.json 2> $OUT/trace_bench.err || { tail -30 $OUT/trace_bench.err; exit 1; }
python3 $R/tools/c5_timeline.py $OUT/trace/run_kernel_trace.csv $STEPS $OUT/trace_bench.json \
  | tee $OUT/timeline.json
rm -f $OUT/trace/run_kernel_trace.csv.gz
