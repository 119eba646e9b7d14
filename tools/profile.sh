#!/bin/bash
# Kernel-trace + PMC passes over bench.py on the GPU box (run via gpurun).
# Each rocprofv3 pass is its own process; counters are collected in separate
# passes (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass on gfx950).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
# one stream: every walk launch runs alone, so the trace's per-launch average
# is the kernel's own duration, the one bench.py's roofline uses (the timed
# steps of the default run overlap two walks on two streams)
ARGS="--no-cpu-baseline --streams 1"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $R/bench.py --steps 20 --warmup 5 $ARGS > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "k_get|k_part|k_unpart" --output-format csv -d $OUT/pmc_fetch -o run \
  -- python3 $R/bench.py --steps 5 --warmup 1 --profile-steps 0 $ARGS > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "k_get|k_part|k_unpart" --output-format csv -d $OUT/pmc_write -o run \
  -- python3 $R/bench.py --steps 5 --warmup 1 --profile-steps 0 $ARGS > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit $?
find $OUT -name "*.csv" | head -50
