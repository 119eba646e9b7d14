#!/bin/bash
# FETCH_SIZE / WRITE_SIZE of the get walk under two environment settings.
# usage: bash tools/pmc_ab.sh TAG "VAR=a" "VAR=b"
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/pmcab_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for setting in "$@"; do
  i=$((i+1))
  for ctr in FETCH_SIZE WRITE_SIZE; do
    env $setting timeout -k 10 300 rocprofv3 --pmc $ctr --kernel-include-regex "k_get" --output-format csv \
      -d $OUT/s${i}_$ctr -o run -- python3 $R/bench.py --steps 3 --warmup 1 --profile-steps 0 --no-cpu-baseline \
      > $OUT/s${i}_$ctr.json 2> $OUT/s${i}_$ctr.err || exit $?
  done
  python3 - $OUT $i "$setting" <<'PY'
import csv, glob, sys
out, i, setting = sys.argv[1], sys.argv[2], sys.argv[3]
res = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    v = [float(r["Counter_Value"]) for r in csv.DictReader(open(glob.glob(f"{out}/s{i}_{ctr}/run_counter_collection.csv")[0]))
         if r["Counter_Name"] == ctr]
    res[ctr] = sum(v) / len(v)
print(setting, "FETCH_KB", round(res["FETCH_SIZE"]), "WRITE_KB", round(res["WRITE_SIZE"]),
      "hbm_MB", round((2 * res["FETCH_SIZE"] + res["WRITE_SIZE"]) / 1024, 1))
PY
done
