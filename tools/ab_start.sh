#!/bin/bash
# A/B of the get walk's start: leaf directory, LDS replica of the
# top levels, root descent; C2 (2^26 keys) and the C4 shard size (2^27 keys
# of an 8-way partition); each line with the index statistics pass.
#   bash tools/ab_start.sh TAG        (via gpurun)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abstart_${1:-r03}
mkdir -p $OUT
cd $R
for CFG in "c2:" "c4:--keys-log2 27 --sim-world 8 --sim-rank 3"; do
  N=${CFG%%:*}; A=${CFG#*:}
  for S in dir lds root; do
    timeout -k 10 400 python3 -u bench.py --no-cpu-baseline --index-stats --latency-steps 0 \
      --start $S $A > $OUT/${N}_$S.json 2> $OUT/${N}_$S.err || { tail -20 $OUT/${N}_$S.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[1].split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['walk_ms_per_launch'], json.dumps(d.get('index_stats')))" $OUT/${N}_$S.json
  done
done
