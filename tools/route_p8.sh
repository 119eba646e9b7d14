#!/bin/bash
# tools/route_p8.py on the box, plain and under a kernel trace:  bash tools/route_p8.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
OUT=$R/gpurun_out/route_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 $R/tools/route_p8.py > $OUT/route.json 2> $OUT/route.err || { tail -20 $OUT/route.err; exit 1; }
cat $OUT/route.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- \
  python3 $R/tools/route_p8.py 27 20 > $OUT/route_trace.json 2> $OUT/route_trace.err || { tail -20 $OUT/route_trace.err; exit 1; }
cut -d, -f1-4 $OUT/trace/run_kernel_stats.csv | head -14 | cut -c1-140
echo route_p8 done
