"""Gaps between k_spin's end and the next k_mark's start, per mode (the
k_mark's argument order: modes 1..7 of tools/event_gap.hip in launch order).
    python tools/event_gap.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    spins = [e for e in ev if "k_spin" in e[2]]
    marks = [e for e in ev if "k_mark" in e[2]]
    names = {1: "back to back", 2: "device-scope event record", 3: "default event record",
             4: "same-stream wait", 5: "cross-stream record+wait", 6: "cross-stream wait, done",
             7: "timing event record", 8: "write-value packet", 9: "write-value + wait-value",
             10: "kernel flag + wait-value"}
    gaps = defaultdict(list)
    # the spin that precedes each mark in time (mode 6 has two spins: the later one)
    spins += [e for e in ev if "k_spin_flag" in e[2] and e not in spins]
    for m in marks:
        prev = max((s for s in spins if s[1] <= m[0]), key=lambda s: s[1], default=None)
        if prev is None:
            continue
        mode = len(gaps) and 0
        gaps[m].append((m[0] - prev[1]) / 1000)
    seq = [g[0] for m, g in sorted(gaps.items())]
    for i, v in enumerate(seq):
        gaps_by = i % 10 + 1
        names.setdefault(gaps_by, str(gaps_by))
    out = defaultdict(list)
    for i, v in enumerate(seq):
        out[i % 10 + 1].append(v)
    for k in sorted(out):
        v = sorted(out[k])
        print(f"mode {k} {names[k]:30s} gap p50 {v[len(v) // 2]:6.1f} us  min {v[0]:6.1f}  max {v[-1]:6.1f}")


if __name__ == "__main__":
    main()
