"""Write profiles/pmc_walk.json (read by bench.py for roofline.traffic) from a
prof_summary.py output: the get walk kernel's per-launch HBM bytes
(FETCH_SIZE x 2 + WRITE_SIZE, gfx950 correction) and its kernel-trace
average duration.  usage: python tools/pmc_json.py SUMMARY.json TAG"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main(path, tag):
    d = json.load(open(path))
    pk = [k for k in d["pmc"] if k.startswith("void shm::dev::k_get<")]
    kk = [k for k in d["kernels"] if k.startswith("void shm::dev::k_get<")]
    assert len(pk) == 1 and len(kk) == 1, (pk, kk)
    p = d["pmc"][pk[0]]
    out = {
        "kernel": pk[0],
        "batch": 1 << 20,
        "keys_log2": 26,
        "source": f"profiles/{os.path.basename(path)} (rocprofv3 --pmc FETCH_SIZE / "
                  f"WRITE_SIZE passes, tools/profile.sh {tag})",
        "fetch_size_kb": p["FETCH_SIZE_KB"],
        "write_size_kb": p["WRITE_SIZE_KB"],
        "correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads, "
                      "MI355X_MICROARCH.md HBM section); WRITE_SIZE as reported",
        "hbm_bytes_per_launch": p["hbm_bytes_per_launch"],
        "kernel_trace_avg_us": d["kernels"][kk[0]]["avg_us"],
    }
    json.dump(out, open(os.path.join(ROOT, "profiles", "pmc_walk.json"), "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
