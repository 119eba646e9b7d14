set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/t60
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/bench.py --workload c5 --no-cpu-baseline --latency-steps 0 --profile-steps 0 --steps 60 > $OUT/b.json 2> $OUT/b.err || exit 1
python3 - $OUT <<'PY'
import csv, sys, json
from collections import defaultdict
rows = list(csv.DictReader(open(sys.argv[1] + "/trace/run_kernel_trace.csv")))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
# per k_upper launch index: durations of the chain's kernels in order
names = ["k_tile_dedup", "k_part_coarse", "k_bin_unique", "k_leaf_dir", "k_locate", "k_seg_fill", "k_leaf_upsert", "k_upper", "k_range", "k_scan_u64"]
seq = [r for r in rows if any(n in r["Kernel_Name"] for n in names)]
steps = []
cur = defaultdict(float)
for r in seq:
    n = [x for x in names if x in r["Kernel_Name"]][0]
    cur[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    if n == "k_upper":
        steps.append(dict(cur)); cur = defaultdict(float)
for i in range(60, len(steps), 5):
    print(i, {k: round(v, 1) for k, v in steps[i].items()})
print(json.load(open(sys.argv[1] + "/b.json"))["value"])
PY
