#!/bin/bash
# Round-4 A/B of the new defaults against their switches, same box:
#   C2: SHM_DIR_READ_PHASE=1 (default) vs 0
#   C3/C5: SHM_TILE_MODE=1 (default) vs 0;  C5: SHM_UPPER_PRELOCK=1 vs 0
# usage (via gpurun): bash tools/ab_r04.sh TAG [reps]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-ab}
REPS=${2:-2}
OUT=$R/gpurun_out/ab_$TAG
mkdir -p $OUT
cd $R
run() {  # name workload env...
  local name=$1 w=$2; shift 2
  for r in $(seq 1 $REPS); do
    env "$@" timeout -k 10 300 python -u bench.py --workload $w --no-cpu-baseline \
      > $OUT/${name}_$r.json 2> $OUT/${name}_$r.err || { tail -20 $OUT/${name}_$r.err; return 1; }
    python -c "import json; d=json.loads(open('$OUT/${name}_$r.json').read().strip().splitlines()[-1]); print('$name', $r, d['value'], d['ms_per_step'])"
  done
}
run c2_new c2 SHM_DIR_READ_PHASE=1 && run c2_old c2 SHM_DIR_READ_PHASE=0 &&
run c3_new c3 SHM_TILE_MODE=1 && run c3_old c3 SHM_TILE_MODE=0 &&
run c5_new c5 SHM_TILE_MODE=1 SHM_UPPER_PRELOCK=1 && run c5_tile0 c5 SHM_TILE_MODE=0 &&
run c5_pre0 c5 SHM_UPPER_PRELOCK=0
