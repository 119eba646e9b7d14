"""Fold a tools/profile_write.sh directory into one JSON summary.

Per kernel over the timed steps only (everything from the first anchor
dispatch on: the first get walk for C3, the first range scan for C5; the
untimed C2 preload before it is dropped): calls per step, average and total
duration per step (kernel trace), and HBM bytes per launch from the
FETCH_SIZE / WRITE_SIZE passes (KB units; FETCH doubled, the gfx950
correction of MI355X_MICROARCH.md §HBM).  Also the step's kernel-time sum and
its span (first start .. last end), so the gaps between kernels are visible.
usage: python tools/write_summary.py OUTDIR c3|c5"""
import collections
import csv
import json
import os
import sys

INSERT_KERNELS = ("k_tile_dedup", "k_part_coarse", "k_bin_", "k_locate", "k_seg_",
                  "k_leaf_", "k_upper")
ANCHOR = {"c3": "k_get", "c5": "k_range", "c2": "k_get"}


def steps_of(rows, name, per):
    n = sum(1 for r in rows if name in r["Kernel_Name"])
    return n / per if per else n


def main(d, wl):
    anchor = ANCHOR[wl]
    tr = list(csv.DictReader(open(os.path.join(d, "trace", "run_kernel_trace.csv"))))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    i0 = next(i for i, r in enumerate(tr) if anchor in r["Kernel_Name"])
    # drop the trailing torch / readback-only tail after the last anchor step
    run = tr[i0:]
    # one insert chunk (one k_upper) per step in C3 and C5
    steps = steps_of(run, "k_upper", 1)
    agg = collections.defaultdict(lambda: {"calls": 0, "ns": 0})
    for r in run:
        name = r["Kernel_Name"].split("(")[0]
        a = agg[name]
        a["calls"] += 1
        a["ns"] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    span = int(run[-1]["End_Timestamp"]) - int(run[0]["Start_Timestamp"])
    pmc = collections.defaultdict(dict)
    for ctr, sub in (("FETCH_SIZE", "pmc_fetch"), ("WRITE_SIZE", "pmc_write")):
        p = os.path.join(d, sub, "run_counter_collection.csv")
        if not os.path.exists(p):
            continue
        rows = [r for r in csv.DictReader(open(p)) if r["Counter_Name"] == ctr]
        rows.sort(key=lambda r: int(r["Dispatch_Id"]))
        j0 = next((i for i, r in enumerate(rows) if anchor in r["Kernel_Name"]), None)
        if j0 is None:
            continue
        vals = collections.defaultdict(list)
        for r in rows[j0:]:
            vals[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
        for k, v in vals.items():
            pmc[k][ctr + "_KB"] = sum(v) / len(v)
    out = {"workload": wl, "steps": steps, "span_us_per_step": span / 1e3 / steps,
           "kernel_us_per_step": sum(a["ns"] for a in agg.values()) / 1e3 / steps,
           "kernels": {}}
    for k, a in sorted(agg.items(), key=lambda x: -x[1]["ns"]):
        e = {"calls_per_step": round(a["calls"] / steps, 2),
             "avg_us": round(a["ns"] / a["calls"] / 1e3, 2),
             "us_per_step": round(a["ns"] / 1e3 / steps, 2)}
        if k in pmc:
            f = pmc[k].get("FETCH_SIZE_KB", 0.0) * 1024 * 2
            w = pmc[k].get("WRITE_SIZE_KB", 0.0) * 1024
            e["hbm_bytes_per_launch"] = round(f + w)
            e["fetch_bytes_x2"] = round(f)
            e["write_bytes"] = round(w)
        out["kernels"][k] = e
    # the insert chunk's kernels (ordering, locate, segmentation, upsert,
    # split levels): HBM bytes and kernel time per step
    ins = {k: e for k, e in out["kernels"].items() if any(p in k for p in INSERT_KERNELS)}
    out["insert_chunk"] = {
        "kernels": sorted(ins),
        "kernel_us_per_step": round(sum(e["us_per_step"] for e in ins.values()), 2),
        "hbm_bytes_per_step": round(sum(e.get("hbm_bytes_per_launch", 0) * e["calls_per_step"]
                                        for e in ins.values())),
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
