#!/bin/bash
# Alternating bench A/B of (library, arguments) variants on one box (via gpurun):
#   bash tools/ab_mixed.sh TAG ROUNDS "common args" "LIB|variant args" ...
# LIB names sherman_amd/exp_LIB.so (copied over libsherman_amd.so for the run).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; ROUNDS=$2; COMMON=$3; shift 3
OUT=$R/gpurun_out/abm_$TAG
mkdir -p $OUT
cp $R/sherman_amd/libsherman_amd.so $OUT/orig.so
cd $R
for r in $(seq 1 $ROUNDS); do
  i=0
  for V in "$@"; do
    i=$((i + 1))
    LIBV=${V%%|*}; ARGS=${V#*|}
    cp $R/sherman_amd/exp_$LIBV.so $R/sherman_amd/libsherman_amd.so
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-steps 0 $COMMON $ARGS \
      > $OUT/v${i}_$r.json 2> $OUT/v${i}_$r.err || { tail -20 $OUT/v${i}_$r.err; cp $OUT/orig.so $R/sherman_amd/libsherman_amd.so; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'])" \
      $OUT/v${i}_$r.json "[$V] r$r"
  done
done
cp $OUT/orig.so $R/sherman_amd/libsherman_amd.so
