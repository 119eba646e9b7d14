#!/bin/bash
# The roofline evidence of one round (run via gpurun):
#   bash tools/roofline_pass.sh TAG [c2 c3 c5]
# For each workload, every profiler run marks the bench's roofline window with
# an empty kernel at each edge (bench.py Region, SHM_BENCH_REGION = "profile":
# the pass whose HIP-event times give roofline.achieved), and the fold keeps
# only the dispatches between the marks:
#   1. the bench line itself (no profiler);
#   2. kernel trace + stats of the profile window;
#   3. FETCH_SIZE, WRITE_SIZE (and for C2 the TCC read requests) passes of
#      the same window, one counter group per run;
#   4. C2 also a kernel trace of the timed window (SHM_BENCH_REGION=timed);
# then tools/fold_roofline.py writes profiles/pmc_walk.json,
# profiles/pmc_steps.json and gpurun_out/roof_TAG/roofline_W.json (the
# recomputation of each bench line's frac from the profile files).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r05}
shift
WLS=${@:-c2 c3 c5}
OUT=$R/gpurun_out/roof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for W in $WLS; do
  B="$R/bench.py --workload $W --no-cpu-baseline --latency-steps 0"
  S="--steps 20 --warmup 3"
  [ $W = c5 ] && S="--steps 10 --warmup 3"
  timeout -k 10 400 python3 $B > $OUT/bench_$W.json 2> $OUT/bench_$W.err || { tail -20 $OUT/bench_$W.err; exit 1; }
  echo "$W bench: $(tail -c 300 $OUT/bench_$W.json)"
  export SHM_BENCH_REGION=profile
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
    -d $OUT/${W}_trace -o run -- python3 $B $S > $OUT/${W}_trace.json 2> $OUT/${W}_trace.err \
    || { tail -20 $OUT/${W}_trace.err; exit 1; }
  echo "$W trace done"
  timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --output-format csv \
    -d $OUT/${W}_fetch -o run -- python3 $B $S > $OUT/${W}_fetch.json 2> $OUT/${W}_fetch.err \
    || { tail -20 $OUT/${W}_fetch.err; exit 1; }
  echo "$W FETCH_SIZE done"
  timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --output-format csv \
    -d $OUT/${W}_write -o run -- python3 $B $S > $OUT/${W}_write.json 2> $OUT/${W}_write.err \
    || { tail -20 $OUT/${W}_write.err; exit 1; }
  echo "$W WRITE_SIZE done"
  if [ $W = c2 ]; then
    timeout -s KILL 400 rocprofv3 --pmc TCC_EA0_RDREQ_sum --output-format csv \
      -d $OUT/${W}_req -o run -- python3 $B $S > $OUT/${W}_req.json 2> $OUT/${W}_req.err \
      || { tail -20 $OUT/${W}_req.err; exit 1; }
    echo "$W requests done"
    export SHM_BENCH_REGION=timed
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $OUT/${W}_timed -o run -- python3 $B --steps 50 --warmup 5 > $OUT/${W}_timed.json \
      2> $OUT/${W}_timed.err || { tail -20 $OUT/${W}_timed.err; exit 1; }
    echo "$W timed trace done"
  fi
  unset SHM_BENCH_REGION
done
cd $R
python3 tools/fold_roofline.py $OUT $TAG $WLS || exit 1
echo roofline_pass done
