#!/bin/bash
# Kernel trace of C5's timed window (run via gpurun): bash tools/c5_window.sh TAG [bench args]
# then: python3 tools/window_stats.py gpurun_out/c5w_TAG/trace/run_kernel_trace.csv
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05}
shift
OUT=$R/gpurun_out/c5w_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
export SHM_BENCH_REGION=timed
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $R/bench.py --workload c5 --no-cpu-baseline --latency-steps 0 --profile-steps 0 "$@" \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 $R/tools/window_stats.py $OUT/trace/run_kernel_trace.csv
