#!/bin/bash
# Kernel-trace stats of one bench configuration:
#   bash tools/profile_args.sh TAG ANCHOR_KERNEL [bench args...]
# prints the per-step kernel breakdown (tools/c3_breakdown.py, anchored on
# ANCHOR_KERNEL, one anchor launch per step)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ANCHOR=$2; shift 2
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --profile-steps 0 "$@" \
  > $OUT/bench.json 2> $OUT/bench.err || exit $?
python3 $R/tools/c3_breakdown.py $OUT "$ANCHOR" 1
