"""Copy one GPU check + profile pass into profiles/ for round RR:
  tools/gpu_check.sh TAG       -> profiles/rRR/{bench_c2,bench_c3,bench_c5}.json,
                                  pytest_gpu.log, smoke.log
  tools/profile.sh TAG         -> profiles/rRR_c2_kernel_stats.csv, rRR_c2_summary.json,
                                  profiles/pmc_walk.json (the walk's per-launch HBM
                                  bytes that bench.py reports as C2 roofline.traffic)
  tools/profile_write.sh TAG c3|c5
                               -> profiles/rRR_{c3,c5}_kernel_stats.csv,
                                  rRR_{c3,c5}_summary.json, profiles/pmc_insert.json
                                  (the C5 insert chunk's HBM bytes per step that
                                  bench.py reports as C5 roofline.traffic)
The copied C2 / C5 bench lines get the traffic measured in the same call.
usage: python tools/refresh_profiles.py RR TAG"""
import json
import os
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd, tag = sys.argv[1], sys.argv[2]
P = os.path.join(R, "profiles")
chk = os.path.join(R, "gpurun_out", "check_" + tag)
prof = os.path.join(R, "gpurun_out", "prof_" + tag)
dst = os.path.join(P, "r" + rnd)
os.makedirs(dst, exist_ok=True)
FETCH_NOTE = ("FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads, "
              "MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported")

pmc = None
if os.path.isdir(prof):
    s = json.loads(subprocess.check_output(
        [sys.executable, os.path.join(R, "tools", "prof_summary.py"), prof]))
    open(os.path.join(P, "r%s_c2_summary.json" % rnd), "w").write(json.dumps(s, indent=1) + "\n")
    shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"),
                os.path.join(P, "r%s_c2_kernel_stats.csv" % rnd))
    k = [n for n in s["pmc"] if "k_get" in n][0]
    p = s["pmc"][k]
    pmc = {"kernel": k, "batch": 1 << 20, "keys_log2": 26,
           "source": "profiles/r%s_c2_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                     "passes, tools/profile.sh %s)" % (rnd, tag),
           "fetch_size_kb": p["FETCH_SIZE_KB"], "write_size_kb": p["WRITE_SIZE_KB"],
           "correction": FETCH_NOTE,
           "hbm_bytes_per_launch": p["hbm_bytes_per_launch"],
           "kernel_trace_avg_us": s["kernels"][k]["avg_us"]}
    open(os.path.join(P, "pmc_walk.json"), "w").write(json.dumps(pmc, indent=1) + "\n")

ins = None
for wl in ("c3", "c5"):
    d = os.path.join(R, "gpurun_out", "pw_%s_%s" % (tag, wl))
    if not os.path.isdir(d):
        continue
    s = json.loads(subprocess.check_output(
        [sys.executable, os.path.join(R, "tools", "write_summary.py"), d, wl]))
    s["source"] = "tools/profile_write.sh %s %s (kernel trace + FETCH_SIZE / WRITE_SIZE passes)" % (
        tag, wl)
    s["correction"] = FETCH_NOTE
    open(os.path.join(P, "r%s_%s_summary.json" % (rnd, wl)), "w").write(
        json.dumps(s, indent=1) + "\n")
    shutil.copy(os.path.join(d, "trace", "run_kernel_stats.csv"),
                os.path.join(P, "r%s_%s_kernel_stats.csv" % (rnd, wl)))
    if wl == "c5":
        bl = json.loads(open(os.path.join(d, "trace_bench.json")).read())
        ins = {"workload": "c5", "batch": bl["config"]["batch_per_gpu"],
               "keys_log2": (bl["config"]["keys_per_gpu"]).bit_length() - 1,
               "source": "profiles/r%s_c5_summary.json insert_chunk" % rnd,
               "correction": FETCH_NOTE,
               "kernels": s["insert_chunk"]["kernels"],
               "hbm_bytes_per_chunk": s["insert_chunk"]["hbm_bytes_per_step"],
               "kernel_us_per_chunk": s["insert_chunk"]["kernel_us_per_step"]}
        open(os.path.join(P, "pmc_insert.json"), "w").write(json.dumps(ins, indent=1) + "\n")

for f in ("bench_c2.json", "bench_c3.json", "bench_c5.json", "pytest_gpu.log", "smoke.log"):
    src = os.path.join(chk, f)
    if not os.path.exists(src):
        continue
    if f in ("bench_c2.json", "bench_c5.json"):
        d = json.loads(open(src).read())
        r = d["roofline"]
        if f == "bench_c2.json" and pmc:
            r["traffic"] = pmc["hbm_bytes_per_launch"]
            if r.get("queries_per_launch") and r.get("walk_ms_per_launch"):
                r["traffic_per_get"] = round(r["traffic"] / r["queries_per_launch"], 1)
                r["traffic_GBps"] = round(r["traffic"] / (r["walk_ms_per_launch"] * 1e-3) / 1e9, 1)
        if f == "bench_c5.json" and ins:
            r["traffic"] = ins["hbm_bytes_per_chunk"]
        open(os.path.join(dst, f), "w").write(json.dumps(d) + "\n")
    else:
        shutil.copy(src, os.path.join(dst, f))
print(json.dumps({"pmc_walk": pmc, "pmc_insert": ins}, indent=1))
