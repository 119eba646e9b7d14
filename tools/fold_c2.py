"""Fold one tools/measure_c2.sh pass (gpurun_out/mc2_TAG) into profiles/:

  profiles/rRR_c2_timed.json          the timed C2 steps (two walks in flight):
                                      per-step kernel timeline from the kernel
                                      trace, the bench line of that run, the
                                      walk's PMC counters per launch, and the
                                      request roofline recomputed from them
  profiles/rRR_c2_timed_kernel_stats.csv   rocprofv3 --stats of that run
  profiles/cal_fetch.json             the counter calibration for random small
                                      reads (tools/cal_fetch.hip): bytes
                                      FETCH_SIZE counts per read, TCC read
                                      requests per read, reads/s ceilings
  profiles/pmc_walk.json              + the walk's TCC read requests per launch
                                      (bench.py's request roofline input)

usage: python tools/fold_c2.py RR TAG"""
import collections
import csv
import json
import os
import shutil
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counters(path):
    """{kernel name: {counter: [values per dispatch]}} of a PMC pass."""
    out = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        out[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return out


def short(name):
    return name.split("(")[0].replace("void ", "")


def main():
    rnd, tag = sys.argv[1], sys.argv[2]
    src = os.path.join(R, "gpurun_out", "mc2_" + tag)
    P = os.path.join(R, "profiles")
    # ---- calibration: known reads per launch; the last 3 dispatches are warm
    cal_runs = [json.loads(l) for l in open(os.path.join(src, "cal.jsonl")) if l.strip()]
    fetch = counters(os.path.join(src, "cal_fetch", "run_counter_collection.csv"))
    req = counters(os.path.join(src, "cal_req", "run_counter_collection.csv"))
    cal = {"source": "tools/cal_fetch.hip under rocprofv3 --pmc FETCH_SIZE, then "
                     "TCC_EA0_RDREQ_sum TCC_MISS_sum TCC_HIT_sum (tools/measure_c2.sh %s)" % tag,
           "kernels": []}
    seen = collections.Counter()  # runs of one kernel so far: 4 dispatches each
    for run in cal_runs:
        key = run["kernel"].split(" ")[0]
        ix = seen[key]
        seen[key] += 1
        warm = slice(4 * ix + 1, 4 * ix + 4)  # a cold launch, then 3 timed ones
        fk = [k for k in fetch if short(k).startswith(key.split("<")[0]) and
              short(k).replace(" ", "") == key.replace(" ", "")] or \
             [k for k in fetch if short(k).replace(" ", "").startswith(key.replace(" ", ""))]
        row = dict(run)
        if fk:
            f = fetch[fk[0]]["FETCH_SIZE"][warm]
            q = req[fk[0]]
            reads = run["reads_per_launch"]
            row["fetch_size_bytes_per_read"] = round(sum(f) / len(f) * 1024 / reads, 2)
            for c in ("TCC_EA0_RDREQ_sum", "TCC_MISS_sum", "TCC_HIT_sum"):
                v = q[c][warm]
                row[c + "_per_read"] = round(sum(v) / len(v) / reads, 4)
            row["G_requests_per_s"] = round(row["G_reads_per_s"] * row["TCC_EA0_RDREQ_sum_per_read"],
                                            2)
        cal["kernels"].append(row)
    # the ceiling: the highest request rate any calibration kernel sustained
    # over a long launch (steady state), and the walk-shaped mix's
    longs = [k for k in cal["kernels"] if "short" not in k["kernel"] and "G_requests_per_s" in k]
    cal["random_request_ceiling_G_per_s"] = max(k["G_requests_per_s"] for k in longs)
    mixk = [k for k in longs if k["kernel"].startswith("k_mix")]
    if mixk:
        cal["walk_mix_ceiling_G_per_s"] = mixk[0]["G_requests_per_s"]
    open(os.path.join(P, "cal_fetch.json"), "w").write(json.dumps(cal, indent=1) + "\n")

    # ---- the timed steps
    tl = json.load(open(os.path.join(src, "step_timeline.json")))
    bench = json.loads(open(os.path.join(src, "trace_bench.json")).read().strip().splitlines()[-1])
    wf = counters(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    wr = counters(os.path.join(src, "pmc_req", "run_counter_collection.csv"))
    wk = [k for k in wf if "k_get_sum" in k][0]
    steps = tl["steps"]
    batch = bench["config"]["batch_per_gpu"]
    last = lambda v: v[-steps:]  # the timed steps' launches (the last ones)
    avg = lambda v: sum(v) / len(v)
    fetch_kb = avg(last(wf[wk]["FETCH_SIZE"]))
    rdreq = avg(last(wr[wk]["TCC_EA0_RDREQ_sum"]))
    hit = avg(last(wr[wk]["TCC_HIT_sum"]))
    miss = avg(last(wr[wk]["TCC_MISS_sum"]))
    step_s = tl["span_us_per_step"] * 1e-6
    rpg = rdreq / batch
    req_rate = rdreq / step_s / 1e9
    # the highest request rate any calibration kernel sustained (the walk-shaped
    # mix, MALL-resident and HBM-resident random reads, more reads in flight)
    ceil = cal["random_request_ceiling_G_per_s"]
    # the bench line's own accounting: 128 B per random line the walk must
    # touch (two or three, by the measured directory-fingerprint share) + 16 B
    bpg = bench["roofline"].get("alg_bytes_per_get") or 400
    out = {
        "what": "C2 timed steps (bench.py default: two HIP streams, two k_get_sum walks in "
                "flight) under rocprofv3 --kernel-trace; PMC passes of the same command",
        "bench_line": {k: bench[k] for k in ("value", "unit", "ms_per_step", "steps")},
        "step_timeline": tl,
        "pmc_per_launch": {
            "kernel": short(wk),
            "FETCH_SIZE_KB": round(fetch_kb, 1),
            "TCC_EA0_RDREQ": round(rdreq),
            "TCC_HIT": round(hit),
            "TCC_MISS": round(miss),
            "fetch_bytes_per_get_counted": round(fetch_kb * 1024 / batch, 1),
            "requests_per_get": round(rpg, 3),
            "l2_hits_per_get": round(hit / batch, 3),
        },
        "byte_roofline": {
            "alg_bytes_per_get": bpg,
            "note": bench["roofline"].get("alg_bytes_note",
                                          "%s B/get (bench.py roofline.alg_bytes_per_get)" % bpg),
            "alg_GBps_over_step": round(batch * bpg / step_s / 1e9, 1),
            "frac": round(batch * bpg / step_s / 1e9 / 8000.0, 4),
            "reference_1040B_frac": round(batch * 1040 / step_s / 1e9 / 8000.0, 4),
        },
        "request_roofline": {
            "requests_per_get": round(rpg, 3),
            "G_requests_per_s": round(req_rate, 2),
            "ceiling_G_per_s": ceil,
            "ceiling_source": "profiles/cal_fetch.json: the highest TCC read-request rate of "
                              "the calibration kernels (random 16 B / 64 B reads over HBM- and "
                              "Infinity-Cache-resident buffers, the walk's three-request mix "
                              "independent and chained; 16 Mi lanes per launch)",
            "request_frac": round(req_rate / ceil, 4),
        },
    }
    open(os.path.join(P, "r%s_c2_timed.json" % rnd), "w").write(json.dumps(out, indent=1) + "\n")
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                os.path.join(P, "r%s_c2_timed_kernel_stats.csv" % rnd))
    pw = json.load(open(os.path.join(P, "pmc_walk.json")))
    pw["tcc_ea_rdreq_per_launch"] = round(rdreq)
    pw["requests_source"] = "profiles/r%s_c2_timed.json (TCC_EA0_RDREQ_sum pass)" % rnd
    # the walk's FETCH_SIZE from this pass (its writes, 8 B value + found
    # byte per get, are unchanged: WRITE_SIZE kept from the earlier pass)
    pw["fetch_size_kb"] = round(fetch_kb, 2)
    pw["hbm_bytes_per_launch"] = fetch_kb * 1024 * 2 + pw["write_size_kb"] * 1024
    pw.setdefault("write_source", pw.get("source", "earlier pass"))
    pw["source"] = ("FETCH_SIZE: profiles/r%s_c2_timed.json (tools/measure_c2.sh %s); "
                    "WRITE_SIZE: write_source" % (rnd, tag))
    open(os.path.join(P, "pmc_walk.json"), "w").write(json.dumps(pw, indent=1) + "\n")
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
