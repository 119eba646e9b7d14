"""Per-step kernel timeline of the timed C2 steps, from a rocprofv3 kernel
trace of `bench.py --profile-steps 0 --latency-steps 0 --no-cpu-baseline`
(the default two-stream run, i.e. the timed condition):

    python tools/step_timeline.py TRACE.csv STEPS [KERNEL] [bench.json] [pmc_fetch.csv]

The last STEPS launches of KERNEL (default k_get_sum) are the timed steps (the
warmup steps come before them; no profile or latency pass after).  Prints one
JSON object: per-launch duration (two walks overlap, so each is longer than
alone), the steps' span per step, the union of busy time per step, the
overlap, and — with the bench line — the rates recomputed from the trace.
With a FETCH_SIZE pass of the same command it adds the per-launch counted
bytes and TCC requests."""
import csv
import json
import sys

ALG_BYTES_PER_GET_SUM = 3 * 128 + 16


def main():
    path, steps = sys.argv[1], int(sys.argv[2])
    kern = sys.argv[3] if len(sys.argv) > 3 else "k_get_sum"
    bench = json.load(open(sys.argv[4])) if len(sys.argv) > 4 else None
    rows = [r for r in csv.DictReader(open(path))]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    walks = [r for r in rows if kern in r["Kernel_Name"]][-steps:]
    iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in walks]
    t0, t1 = iv[0][0], max(e for _, e in iv)
    # every kernel launched inside the timed window (gets only in C2)
    inside = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in rows if t0 <= int(r["Start_Timestamp"]) <= t1]
    ev = sorted([(s, 1) for s, e, _ in inside] + [(e, -1) for s, e, _ in inside])
    busy, depth, last = 0, 0, t0
    two = 0
    for t, d in ev:
        if depth > 0:
            busy += t - last
        if depth > 1:
            two += t - last
        depth += d
        last = t
    durs = [(e - s) / 1e3 for s, e in iv]
    names = {}
    for _, _, n in inside:
        names[n.split("(")[0][:40]] = names.get(n.split("(")[0][:40], 0) + 1
    out = {
        "kernel": kern,
        "steps": steps,
        "launches_in_window": len(inside),
        "kernels_in_window": names,
        "launch_us_avg": round(sum(durs) / len(durs), 2),
        "launch_us_min": round(min(durs), 2),
        "launch_us_max": round(max(durs), 2),
        "span_us_per_step": round((t1 - t0) / 1e3 / steps, 2),
        "busy_us_per_step": round(busy / 1e3 / steps, 2),
        "two_in_flight_frac": round(two / max(busy, 1), 3),
    }
    if bench is not None:
        q = bench["config"]["batch_per_gpu"]
        out["bench_ms_per_step"] = bench["ms_per_step"]
        step_us = (t1 - t0) / 1e3 / steps
        out["alg_GBps_over_span"] = round(q * ALG_BYTES_PER_GET_SUM / (step_us * 1e-6) / 1e9, 1)
        out["alg_frac_over_span"] = round(out["alg_GBps_over_span"] / 8000.0, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
