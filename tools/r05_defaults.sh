#!/bin/bash
# The default bench lines (CPU baseline included), twice each, plus the C4
# shard's start-mode A/B (run via gpurun): bash tools/r05_defaults.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/def_${1:-r05}
mkdir -p $OUT
cd $R
for i in 1 2; do
  for W in c2 c5 c3; do
    timeout -k 10 400 python3 bench.py --workload $W > $OUT/${W}_$i.json 2> $OUT/${W}_$i.err \
      || { tail -20 $OUT/${W}_$i.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$OUT/${W}_$i.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$W $i', d['value'], d['ms_per_step'], d.get('parity_vs_oracle'), r.get('frac'), r.get('step_frac'), r.get('dir_fp_frac'))"
  done
done
for S in dir lds root; do
  timeout -k 10 400 python3 bench.py --keys-log2 27 --sim-world 8 --sim-rank 3 --start $S --index-stats \
    --no-cpu-baseline --latency-steps 0 > $OUT/c4_$S.json 2> $OUT/c4_$S.err || { tail -20 $OUT/c4_$S.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$OUT/c4_$S.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c4 $S', d['value'], d['ms_per_step'], r['walk_ms_per_launch'], d.get('index_stats',{}).get('start_internal_per_get'), d.get('index_stats',{}).get('right_moves_per_get'))"
done
