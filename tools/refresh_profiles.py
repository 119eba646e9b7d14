"""Copy one GPU check + profile pass (tools/gpu_check.sh TAG, tools/profile.sh
TAG) into profiles/: bench lines, pytest log, kernel stats, PMC summary, and
profiles/pmc_walk.json (the walk's per-launch HBM bytes that bench.py reports
as roofline.traffic).  The C2 bench line's traffic is replaced by the value
measured in the same gpurun call.
usage: python tools/refresh_profiles.py TAG"""
import json
import os
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
chk = os.path.join(R, "gpurun_out", "check_" + tag)
prof = os.path.join(R, "gpurun_out", "prof_" + tag)
dst = os.path.join(R, "profiles", "r01")
summ = subprocess.check_output([sys.executable, os.path.join(R, "tools", "prof_summary.py"), prof])
s = json.loads(summ)
open(os.path.join(R, "profiles", "r01_summary.json"), "w").write(json.dumps(s, indent=1) + "\n")
shutil.copy(os.path.join(prof, "trace", "run_kernel_stats.csv"),
            os.path.join(R, "profiles", "r01_kernel_stats.csv"))
k = [n for n in s["pmc"] if "k_get" in n][0]
p = s["pmc"][k]
pmc = {"kernel": k, "batch": 1 << 20, "keys_log2": 26,
       "source": "profiles/r01_summary.json (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, "
                 "tools/profile.sh %s)" % tag,
       "fetch_size_kb": p["FETCH_SIZE_KB"], "write_size_kb": p["WRITE_SIZE_KB"],
       "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads, "
                     "MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported",
       "hbm_bytes_per_launch": p["hbm_bytes_per_launch"],
       "kernel_trace_avg_us": s["kernels"][k]["avg_us"]}
open(os.path.join(R, "profiles", "pmc_walk.json"), "w").write(json.dumps(pmc, indent=1) + "\n")
for f in ("bench_c2.json", "bench_c3.json", "bench_c5.json", "pytest_gpu.log", "smoke.log"):
    src = os.path.join(chk, f)
    if not os.path.exists(src):
        continue
    if f == "bench_c2.json":
        d = json.loads(open(src).read())
        r = d["roofline"]
        r["traffic"] = pmc["hbm_bytes_per_launch"]
        if r.get("queries_per_launch") and r.get("walk_ms_per_launch"):
            r["traffic_per_get"] = round(r["traffic"] / r["queries_per_launch"], 1)
            r["traffic_GBps"] = round(r["traffic"] / (r["walk_ms_per_launch"] * 1e-3) / 1e9, 1)
        open(os.path.join(dst, f), "w").write(json.dumps(d) + "\n")
    else:
        shutil.copy(src, os.path.join(dst, f))
print(json.dumps(pmc, indent=1))
