#!/bin/bash
# Alternating bench A/B of command-line variants on one box (via gpurun):
#   bash tools/ab_args.sh TAG ROUNDS "common args" "variant args 1" "variant args 2" ...
# prints value / ms_per_step per run (no profiler, no CPU baseline).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ROUNDS=$2; COMMON=$3; shift 3
OUT=$R/gpurun_out/aba_$TAG
mkdir -p $OUT
cd $R
for r in $(seq 1 $ROUNDS); do
  i=0
  for V in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-steps 0 $COMMON $V \
      > $OUT/v${i}_$r.json 2> $OUT/v${i}_$r.err || { tail -20 $OUT/v${i}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      $OUT/v${i}_$r.json "[$V] r$r"
  done
done
