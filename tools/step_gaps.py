"""Per-step kernel timeline with gaps from a rocprofv3 kernel trace:
    python tools/step_gaps.py run_kernel_trace.csv [steps_to_show]
(the last steps, each starting at a k_range)."""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    show = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    ev = sorted((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                 r['Kernel_Name'].split('(')[0].split('::')[-1][:28]) for r in rows)
    idx = [i for i, e in enumerate(ev) if 'k_range' in e[2]]
    start, end = idx[-(show + 2)], idx[-2]
    t0 = ev[start][0]
    busy = ev[start][1]
    for s, e, n in ev[start:end]:
        print(f"{(s - t0) / 1000:8.1f} {(e - t0) / 1000:8.1f} dur {(e - s) / 1000:6.1f} "
              f"gap {(s - busy) / 1000:6.1f} {n}")
        busy = max(busy, e)


if __name__ == "__main__":
    main()
