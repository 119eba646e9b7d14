"""Fold a tools/roofline_pass.sh directory into the committed roofline inputs.

  profiles/pmc_walk.json    C2: the get walk's HBM bytes and TCC read
                            requests per launch, and its kernel-trace average,
                            all over the bench's profile window
  profiles/pmc_steps.json   C3 / C5: per kernel of the profile window (calls
                            per chunk, average us, HBM bytes per launch) and
                            the per-chunk sums bench.py reads: the tree
                            phase's kernels (apply), the ordering's, the step
  OUTDIR/roofline_W.json    the recomputation of each bench line's roofline
                            fractions from these files (every
                            frac reproducible from profiles/, none above 1)

HBM bytes = FETCH_SIZE x 2 + WRITE_SIZE (KB as reported; the gfx950 FETCH
correction of MI355X_MICROARCH.md §HBM).
usage: python tools/fold_roofline.py OUTDIR TAG W [W ...]"""
import collections
import csv
import json
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(R, "profiles")
PEAK = 8000.0  # GB/s
APPLY = ("k_locate", "k_seg_fill", "k_leaf_upsert", "k_upper", "k_leaf_dir", "k_sum_rebuild",
         "k_dir_")
ORDER = ("k_tile_dedup", "k_part_coarse", "k_bin_unique")
CORR = ("FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads, MI355X_MICROARCH.md HBM "
        "section) + WRITE_SIZE as reported")


def kname(n):
    n = n.split("(")[0]
    return n[5:] if n.startswith("void ") else n


def window(rows):
    """The rows dispatched between the bench's two k_mark dispatches (its
    Region edges, tag 1 then tag 2), in dispatch order."""
    rows = sorted(rows, key=lambda r: int(r["Dispatch_Id"]))
    marks = [i for i, r in enumerate(rows) if "k_mark" in r["Kernel_Name"]]
    assert len(marks) >= 2, "no marked window (SHM_BENCH_REGION unset?)"
    return rows[marks[0] + 1:marks[1]]


def trace(d):
    p = os.path.join(d, "run_kernel_trace.csv")
    agg = collections.defaultdict(lambda: [0, 0])
    for r in window(list(csv.DictReader(open(p)))):
        a = agg[kname(r["Kernel_Name"])]
        a[0] += 1
        a[1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return {k: {"calls": c, "avg_us": ns / c / 1e3} for k, (c, ns) in agg.items()}


def counter(d, name):
    p = os.path.join(d, "run_counter_collection.csv")
    v = collections.defaultdict(list)
    rows = [r for r in csv.DictReader(open(p)) if r["Counter_Name"] == name]
    for r in window(rows):
        v[kname(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: (sum(x) / len(x), len(x)) for k, x in v.items()}


def line(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


def kernels(out, w):
    tr = trace(os.path.join(out, w + "_trace"))
    fe = counter(os.path.join(out, w + "_fetch"), "FETCH_SIZE")
    wr = counter(os.path.join(out, w + "_write"), "WRITE_SIZE")
    ks = {}
    for k, t in tr.items():
        e = {"calls": t["calls"], "avg_us": round(t["avg_us"], 3)}
        if k in fe:
            e["fetch_kb"] = round(fe[k][0], 2)
            e["write_kb"] = round(wr.get(k, (0.0, 0))[0], 2)
            e["hbm_bytes_per_launch"] = round(e["fetch_kb"] * 1024 * 2 + e["write_kb"] * 1024)
            e["pmc_dispatches"] = fe[k][1]
        ks[k] = e
    return ks


def main(out, tag, wls):
    res = {}
    steps_doc = {}
    try:
        steps_doc = json.load(open(os.path.join(P, "pmc_steps.json")))
    except (OSError, ValueError):
        pass
    for w in wls:
        bl = line(os.path.join(out, "bench_%s.json" % w))       # the plain bench run
        tl = line(os.path.join(out, "%s_trace.json" % w))       # the traced run's line
        rf, rft = bl["roofline"], tl["roofline"]
        ks = kernels(out, w)
        batch = bl["config"]["batch_per_gpu"]
        keys_log2 = bl["config"]["keys_per_gpu"].bit_length() - 1
        src = "tools/roofline_pass.sh %s (rocprofv3, the bench's marked profile window)" % tag
        if w == "c2":
            k = next(n for n in ks if "k_get_sum" in n)
            e = ks[k]
            req = counter(os.path.join(out, "c2_req"), "TCC_EA0_RDREQ_sum")
            rq = req.get(k, (None, 0))[0]
            walk = {"kernel": k, "batch": batch, "keys_log2": keys_log2, "source": src,
                    "fetch_size_kb": e["fetch_kb"], "write_size_kb": e["write_kb"],
                    "correction": CORR, "hbm_bytes_per_launch": e["hbm_bytes_per_launch"],
                    "tcc_ea_rdreq_per_launch": rq, "kernel_trace_avg_us": e["avg_us"],
                    "launches_in_window": e["calls"]}
            json.dump(walk, open(os.path.join(P, "pmc_walk.json"), "w"), indent=1)
            q = rf["queries_per_launch"]
            recomputed = rf["alg_bytes_per_get"] * q / (e["avg_us"] * 1e-6) / 1e9 / PEAK
            timed = trace(os.path.join(out, "c2_timed"))
            tk = next(n for n in timed if "k_get_sum" in n)
            res[w] = {
                "bench_frac": rf["frac"], "bench_walk_ms_per_launch": rf["walk_ms_per_launch"],
                "alg_bytes_per_get": rf["alg_bytes_per_get"], "queries_per_launch": q,
                "trace_avg_us_profile_window": e["avg_us"],
                "frac_recomputed_from_trace": round(recomputed, 4),
                "agreement": round(recomputed / rf["frac"] - 1, 4) if rf["frac"] else None,
                "traffic_per_launch": e["hbm_bytes_per_launch"],
                "traffic_frac": round(e["hbm_bytes_per_launch"] / (e["avg_us"] * 1e-6) / 1e9 / PEAK, 4),
                "requests_per_get": round(rq / q, 4) if rq else None,
                "timed_window": {"k_get_sum_launches": timed[tk]["calls"],
                                 "k_get_sum_avg_us": round(timed[tk]["avg_us"], 3),
                                 "bench_ms_per_step": tl["ms_per_step"],
                                 "note": "two walks in flight on two streams: each walk's "
                                         "duration spans its overlap with the other"},
                "kernels": ks,
            }
        else:
            chunks = max(ks.get(next((n for n in ks if "k_upper" in n), ""), {}).get("calls", 0), 1)

            def by(pred):
                return sum(e.get("hbm_bytes_per_launch", 0) * e["calls"] for n, e in ks.items()
                           if pred(n)) / chunks

            apply_b = by(lambda n: any(p in n for p in APPLY))
            order_b = by(lambda n: any(p in n for p in ORDER))
            step_b = by(lambda n: True)
            steps_doc[w] = {"batch": batch, "keys_log2": keys_log2, "source": src,
                            "correction": CORR, "chunks_in_window": chunks,
                            "apply_kernels": sorted(n for n in ks if any(p in n for p in APPLY)),
                            "order_kernels": sorted(n for n in ks if any(p in n for p in ORDER)),
                            "apply_bytes_per_chunk": round(apply_b),
                            "order_bytes_per_chunk": round(order_b),
                            "step_bytes": round(step_b),
                            "kernels": {n: dict(e, calls_per_chunk=round(e["calls"] / chunks, 3))
                                        for n, e in ks.items()}}
            ins = rf.get("insert") or rf
            r = {"bench_frac": rf["frac"], "bench_insert_ms_per_launch": ins["insert_ms_per_launch"],
                 "apply_bytes_per_chunk": round(apply_b), "order_bytes_per_chunk": round(order_b),
                 "step_bytes": round(step_b), "alg_bytes_per_chunk": ins["alg_bytes_per_chunk"],
                 "apply_kernel_us_per_chunk": round(sum(e["avg_us"] * e["calls"] for n, e in ks.items()
                                                        if any(p in n for p in APPLY)) / chunks, 2)}
            win_b = apply_b + (0 if "ordering runs" in ins["window"] else order_b)
            r["traffic_frac_recomputed"] = round(
                win_b / (ins["insert_ms_per_launch"] * 1e-3) / 1e9 / PEAK, 4)
            r["alg_frac_recomputed"] = round(
                ins["alg_bytes_per_chunk"] / (ins["insert_ms_per_launch"] * 1e-3) / 1e9 / PEAK, 4)
            if w == "c3":
                r["step_traffic_frac_recomputed"] = round(
                    step_b / (bl["ms_per_step"] * 1e-3) / 1e9 / PEAK, 4)
            r["kernels"] = ks
            res[w] = r
    json.dump(steps_doc, open(os.path.join(P, "pmc_steps.json"), "w"), indent=1)
    for w, r in res.items():
        json.dump(r, open(os.path.join(out, "roofline_%s.json" % w), "w"), indent=1)
        print(w, json.dumps({k: v for k, v in r.items() if k != "kernels"}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3:])
