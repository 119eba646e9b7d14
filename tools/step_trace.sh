#!/bin/bash
# Kernel trace of one bench line and its per-step timeline (tools/step_gaps.py):
#   bash tools/step_trace.sh TAG WORKLOAD MARKER [ENV=VAL ...]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; W=$2; M=$3; shift 3
OUT=$R/gpurun_out/st_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run \
  -- python3 $R/bench.py --workload $W --no-cpu-baseline --latency-steps 0 --profile-steps 0 --steps 60 \
  > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 $R/tools/step_gaps.py $OUT/trace/run_kernel_trace.csv 1 $M 40
rm -f $OUT/trace/run_kernel_trace.csv.gz
