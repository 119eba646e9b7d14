#!/bin/bash
# Round-5 A/B and trace pass (run via gpurun): bash tools/r05_ab.sh TAG
#   1. C2 with 4 vs 8 directory entries per tree page (two runs each, alternating)
#   2. kernel trace of C5's timed window (SHM_BENCH_REGION=timed)
#   3. the C2 roofline pass (device-clock walk time against the trace)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
cd $R
for i in 1 2; do
  for x in 2 3; do
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --latency-steps 0 --dir-extra-bits $x \
      > $OUT/c2_x${x}_$i.json 2> $OUT/c2_x${x}_$i.err || { tail -20 $OUT/c2_x${x}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/c2_x${x}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('x$x', d['value'], r['frac'], r.get('request_frac'), r.get('dir_fp_frac'), r['walk_ms_per_launch'], r.get('walk_event_ms_per_launch'))"
  done
done
cd /tmp && export TMPDIR=/tmp
export SHM_BENCH_REGION=timed
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c5_timed -o run \
  -- python3 $R/bench.py --workload c5 --no-cpu-baseline --latency-steps 0 --profile-steps 0 \
  > $OUT/c5_timed.json 2> $OUT/c5_timed.err || { tail -20 $OUT/c5_timed.err; exit 1; }
unset SHM_BENCH_REGION
echo "c5 timed trace done"
cd $R
bash tools/roofline_pass.sh ${TAG} c2 > $OUT/roof.log 2>&1 || { tail -20 $OUT/roof.log; exit 1; }
tail -3 $OUT/roof.log
