"""Summarise a tools/profile.sh output directory: per-kernel stats from the
kernel trace and per-launch HBM bytes from the FETCH_SIZE / WRITE_SIZE passes
(FETCH_SIZE doubled: gfx950 reports half of a wide coalesced read,
MI355X_MICROARCH.md §HBM)."""
import collections
import csv
import json
import os
import sys


def main(d, match=("k_get", "k_walk", "k_part", "k_unpart", "k_gather")):
    stats = list(csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))))
    out = {"kernels": {}, "pmc": {}}
    for r in stats:
        name = r["Name"]
        if any(m in name for m in match):
            out["kernels"][name] = {"calls": int(r["Calls"]),
                                    "avg_us": float(r["AverageNs"]) / 1e3,
                                    "min_us": float(r["MinNs"]) / 1e3,
                                    "max_us": float(r["MaxNs"]) / 1e3}
    for ctr, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(p)):
            if r["Counter_Name"] == ctr and any(m in r["Kernel_Name"] for m in match):
                agg[r["Kernel_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            kb = sum(v) / len(v)
            out["pmc"].setdefault(k, {})[ctr + "_KB"] = kb
    for k, v in out["pmc"].items():
        f = v.get("FETCH_SIZE_KB", 0.0) * 1024 * 2
        w = v.get("WRITE_SIZE_KB", 0.0) * 1024
        v["hbm_bytes_per_launch"] = f + w
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
