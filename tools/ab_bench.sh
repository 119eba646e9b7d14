#!/bin/bash
# Alternating bench A/B of library variants on one box (via gpurun):
#   bash tools/ab_bench.sh TAG ROUNDS "bench args" V1 V2 ...
# copies sherman_amd/exp_<V>.so over libsherman_amd.so for each run and
# prints value / ms_per_step per run (no profiler).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
OUT=$R/gpurun_out/abb_$TAG
mkdir -p $OUT
cp $R/sherman_amd/libsherman_amd.so $OUT/orig.so
cd $R
for r in $(seq 1 $ROUNDS); do
  for V in "$@"; do
    cp $R/sherman_amd/exp_$V.so $R/sherman_amd/libsherman_amd.so
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-steps 0 $ARGS \
      > $OUT/${V}_$r.json 2> $OUT/${V}_$r.err || { tail -20 $OUT/${V}_$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" $OUT/${V}_$r.json "$V r$r"
  done
done
cp $OUT/orig.so $R/sherman_amd/libsherman_amd.so
