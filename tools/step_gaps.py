"""Per-step kernel timeline with gaps from a rocprofv3 kernel trace:
    python tools/step_gaps.py run_kernel_trace.csv [steps_to_show] [marker] [avg_steps]
(the last steps, each starting at a `marker` kernel, default k_range), then
each kernel's mean duration and the mean step span over the last avg_steps."""
import csv
import sys
from collections import defaultdict


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    show = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    marker = sys.argv[3] if len(sys.argv) > 3 else "k_range"
    navg = int(sys.argv[4]) if len(sys.argv) > 4 else 20
    ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                 r['Kernel_Name'].split('(')[0].split('::')[-1][:28]) for r in rows)
    idx = [i for i, e in enumerate(ev) if marker in e[2]]
    start, end = idx[-(show + 2)], idx[-2]
    t0 = ev[start][0]
    busy = ev[start][1]
    for s, e, n in ev[start:end]:
        print(f"{(s - t0) / 1000:8.1f} {(e - t0) / 1000:8.1f} dur {(e - s) / 1000:6.1f} "
              f"gap {(s - busy) / 1000:6.1f} {n}")
        busy = max(busy, e)
    a, b = idx[-(navg + 2)], idx[-2]
    dur = defaultdict(float)
    for s, e, n in ev[a:b]:
        dur[n] += (e - s) / 1000
    span = (ev[b][0] - ev[a][0]) / 1000 / navg
    print(f"mean over {navg} steps: span {span:.1f} us; " +
          ", ".join(f"{n} {d / navg:.1f}" for n, d in sorted(dur.items(), key=lambda x: -x[1])))


if __name__ == "__main__":
    main()
