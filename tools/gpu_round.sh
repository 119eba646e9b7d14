#!/bin/bash
# One GPU-box pass (run via gpurun):  bash tools/gpu_round.sh TAG [what...]
#   what: dir full tests bench ie (default: all, in that order)
# Each step under its own time limit; the first failure ends the call.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
shift
WHAT=${*:-dir full tests bench ie}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd $R
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for w in $WHAT; do
  case $w in
    dir) timeout -k 10 600 $PYT tests/test_gpu_dir.py > $OUT/dir.log 2>&1 || { tail -60 $OUT/dir.log; exit 1; }
         tail -3 $OUT/dir.log ;;
    full) timeout -k 10 600 $PYT tests/test_gpu_fullsize.py > $OUT/full.log 2>&1 || { tail -60 $OUT/full.log; exit 1; }
         tail -3 $OUT/full.log ;;
    tests) timeout -k 10 900 $PYT -m gpu tests > $OUT/tests.log 2>&1 || { tail -60 $OUT/tests.log; exit 1; }
         tail -3 $OUT/tests.log
         timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 \
           || { cat $OUT/smoke.log; exit 1; }
         cat $OUT/smoke.log ;;
    bench) timeout -k 10 500 python -u bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err \
           || { tail -30 $OUT/bench_c2.err; exit 1; }
         cat $OUT/bench_c2.json ;;
    ie) timeout -k 10 500 python -u bench.py --insert-every 8 > $OUT/bench_ie.json 2> $OUT/bench_ie.err \
           || { tail -30 $OUT/bench_ie.err; exit 1; }
         cat $OUT/bench_ie.json ;;
    pchk) timeout -k 10 500 python -u bench.py --page-check 1 --no-cpu-baseline > $OUT/bench_pchk.json 2> $OUT/bench_pchk.err \
           || { tail -30 $OUT/bench_pchk.err; exit 1; }
         cat $OUT/bench_pchk.json ;;
    c3|c5) timeout -k 10 500 python -u bench.py --workload $w > $OUT/bench_$w.json 2> $OUT/bench_$w.err \
           || { tail -30 $OUT/bench_$w.err; exit 1; }
         cat $OUT/bench_$w.json ;;
  esac
done
echo gpu_round done
