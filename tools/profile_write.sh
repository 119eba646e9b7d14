#!/bin/bash
# Write-path evidence for one workload (run via gpurun):
#   bash tools/profile_write.sh TAG c3|c5
# 1. rocprofv3 kernel trace + stats of a short bench run;
# 2. FETCH_SIZE and WRITE_SIZE passes (separate runs: they do not fit one TCC
#    pass) over every kernel of the step (gets, ordering, locate, segmentation,
#    upsert, split levels, range scans);
# 3. tools/write_summary.py folds them into OUT/summary.json (per kernel:
#    calls per step, avg us, HBM bytes per launch with the gfx950 FETCH x2
#    correction).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r02}
WL=${2:-c3}
OUT=$R/gpurun_out/pw_${TAG}_$WL
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
RX="k_tile_dedup|k_part_|k_bin_|k_locate|k_seg_|k_leaf_|k_tile_s|k_int_|k_new_root|k_readback|k_write_super|k_get|k_range|k_upper|k_split|k_alloc|k_publish|k_unpart"
B="$R/bench.py --workload $WL --no-cpu-baseline"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run \
  -- python3 $B --steps 20 --warmup 3 --profile-steps 0 > $OUT/trace_bench.json 2> $OUT/trace_bench.err || exit $?
echo "profile_write $WL: trace done"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_fetch -o run \
  -- python3 $B --steps 4 --warmup 1 --profile-steps 0 > $OUT/pmc_fetch.json 2> $OUT/pmc_fetch.err || exit $?
echo "profile_write $WL: FETCH_SIZE done"
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RX" --output-format csv -d $OUT/pmc_write -o run \
  -- python3 $B --steps 4 --warmup 1 --profile-steps 0 > $OUT/pmc_write.json 2> $OUT/pmc_write.err || exit $?
python3 $R/tools/write_summary.py $OUT $WL > $OUT/summary.json || exit $?
cat $OUT/summary.json | head -80
