"""Per-step kernel timeline of the timed C5 steps, from a rocprofv3 kernel
trace of `bench.py --workload c5 --no-cpu-baseline --latency-steps 0
--profile-steps 0 --steps STEPS`:

    python tools/c5_timeline.py TRACE.csv STEPS [bench.json]

A step ends with its chunk's k_upper; the last STEPS steps are the timed
ones.  Prints per kernel family the mean duration per step, the step's span
(previous k_upper end -> this k_upper end), the device-busy union and the
idle gaps, and the critical chain: scans (k_range x2 + scan) then the
chunk's tree phase (locate .. k_upper), with the ordering kernels that ran
beside the scans."""
import csv
import json
import sys
from collections import defaultdict

FAMILIES = ["k_tile_dedup", "k_part_coarse", "k_bin_unique", "k_leaf_dir", "k_locate",
            "k_seg_fill", "k_leaf_upsert", "k_upper", "k_range", "k_scan_u64", "k_readback"]


def fam(name):
    for f in FAMILIES:
        if f in name:
            return f
    return name.split("(")[0][-40:]


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), fam(r["Kernel_Name"]))
                 for r in rows), key=lambda x: x[0])
    ups = [i for i, k in enumerate(ks) if k[2] == "k_upper"]
    ups = ups[-(steps + 1):]
    per = defaultdict(float)
    span = busy = 0.0
    chain = defaultdict(float)
    for a, b in zip(ups[:-1], ups[1:]):
        t0, t1 = ks[a][1], ks[b][1]
        inside = [k for k in ks[a + 1:b + 1]]
        for s, e, f in inside:
            per[f] += (e - s) / 1e3
        ev = sorted([(max(s, t0), 1) for s, e, _ in inside] + [(e, -1) for s, e, _ in inside])
        depth, last, bz = 0, t0, 0
        for t, d in ev:
            if depth > 0:
                bz += t - last
            depth += d
            last = t
        busy += bz / 1e3
        span += (t1 - t0) / 1e3
        # the chain: first scan start -> last scan end; then locate start -> k_upper end
        rs = [k for k in inside if k[2] in ("k_range", "k_scan_u64")]
        tr = [k for k in inside if k[2] in ("k_locate", "k_seg_fill", "k_leaf_upsert", "k_upper",
                                            "k_leaf_dir")]
        od = [k for k in inside if k[2] in ("k_tile_dedup", "k_part_coarse", "k_bin_unique")]
        if rs:
            chain["scans_span"] += (max(e for _, e, _ in rs) - min(s for s, _, _ in rs)) / 1e3
        if tr:
            chain["tree_span"] += (max(e for _, e, _ in tr) - min(s for s, _, _ in tr)) / 1e3
        if od:
            chain["ordering_span"] += (max(e for _, e, _ in od) - min(s for s, _, _ in od)) / 1e3
        if rs and tr:
            chain["scans_end_to_tree_start"] += (min(s for s, _, _ in tr) -
                                                 max(e for _, e, _ in rs)) / 1e3
        if rs and od:
            chain["ordering_end_after_scans_end"] += (max(e for _, e, _ in od) -
                                                      max(e for _, e, _ in rs)) / 1e3
    n = len(ups) - 1
    out = {
        "steps": n,
        "span_us_per_step": round(span / n, 2),
        "busy_us_per_step": round(busy / n, 2),
        "idle_us_per_step": round((span - busy) / n, 2),
        "kernel_us_per_step": {k: round(v / n, 2) for k, v in sorted(per.items(),
                                                                     key=lambda x: -x[1])},
        "chain_us_per_step": {k: round(v / n, 2) for k, v in chain.items()},
    }
    if len(sys.argv) > 3:
        b = json.load(open(sys.argv[3]))
        out["bench_value"] = b["value"]
        out["bench_ms_per_step"] = b["ms_per_step"]
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
