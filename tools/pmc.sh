#!/bin/bash
# One rocprofv3 --pmc pass per argument group over a short bench run.
# usage: tools/pmc.sh TAG "CTR1 CTR2 ..." ["CTR ..."] ...
# env: PMC_REGEX (kernels, default the get path), BENCH_ARGS (default C2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmc_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --kernel-include-regex "${PMC_REGEX:-k_get|k_part|k_unpart}" --output-format csv -d $OUT/p$i -o run \
    -- python3 $R/bench.py --steps 3 --warmup 1 --profile-steps 0 --no-cpu-baseline $BENCH_ARGS \
    > $OUT/p$i.json 2> $OUT/p$i.err || exit $?
done
python3 $R/tools/pmc_summary.py $OUT > $OUT/summary.json
cat $OUT/summary.json
