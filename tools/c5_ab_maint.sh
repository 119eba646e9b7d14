#!/bin/bash
# C5's timed window with the directory upkeep on and off (run via gpurun):
#   bash tools/c5_ab_maint.sh TAG
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r06}
for M in 1 0; do
  SHM_DIR_MAINT=$M bash $R/tools/c5_window.sh ${TAG}_m$M > $R/gpurun_out/c5w_${TAG}_m$M.txt 2>&1 || { cat $R/gpurun_out/c5w_${TAG}_m$M.txt; exit 1; }
  echo "== SHM_DIR_MAINT=$M"; cat $R/gpurun_out/c5w_${TAG}_m$M.txt
  tail -c 400 $R/gpurun_out/c5w_${TAG}_m$M/bench.json | head -c 200; echo
done
