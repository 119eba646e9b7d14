"""Copy a merged tools/roofline_pass.sh directory into profiles/rRR/ and
refresh the committed roofline inputs (run in the build container after the
gpurun call; the GPU box's own profiles/ writes are not merged back):
  python tools/commit_roofline.py RR TAG
-> profiles/pmc_walk.json, profiles/pmc_steps.json (tools/fold_roofline.py),
   profiles/rRR/roofline_{c2,c3,c5}.json (each bench line's fractions
   recomputed from them), bench_W.json (the plain bench line),
   W_kernel_stats.csv (rocprofv3 --kernel-trace --stats of the profiled
   command) and W_window.txt (per-kernel statistics of the marked window)."""
import os
import shutil
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
rnd, tag = sys.argv[1], sys.argv[2]
src = os.path.join(R, "gpurun_out", "roof_" + tag)
dst = os.path.join(R, "profiles", "r" + rnd)
os.makedirs(dst, exist_ok=True)
wls = [w for w in ("c2", "c3", "c5") if os.path.exists(os.path.join(src, "bench_%s.json" % w))]
subprocess.check_call([sys.executable, os.path.join(R, "tools", "fold_roofline.py"), src, tag] + wls,
                      stdout=subprocess.DEVNULL)
for w in wls:
    shutil.copy(os.path.join(src, "roofline_%s.json" % w), os.path.join(dst, "roofline_%s.json" % w))
    shutil.copy(os.path.join(src, "bench_%s.json" % w), os.path.join(dst, "bench_%s.json" % w))
    shutil.copy(os.path.join(src, "%s_trace" % w, "run_kernel_stats.csv"),
                os.path.join(dst, "%s_kernel_stats.csv" % w))
    out = subprocess.check_output([sys.executable, os.path.join(R, "tools", "window_stats.py"),
                                   os.path.join(src, "%s_trace" % w, "run_kernel_trace.csv")])
    open(os.path.join(dst, "%s_window.txt" % w), "wb").write(out)
    if w == "c2":
        out = subprocess.check_output([sys.executable, os.path.join(R, "tools", "window_stats.py"),
                                       os.path.join(src, "c2_timed", "run_kernel_trace.csv")])
        open(os.path.join(dst, "c2_timed_window.txt"), "wb").write(out)
print("profiles/r%s: %s" % (rnd, ", ".join(sorted(os.listdir(dst)))))
