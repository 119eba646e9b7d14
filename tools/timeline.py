"""Print the tail of a rocprofv3 kernel trace as a timeline (duration and gap
before each kernel, µs) for the get-path kernels."""
import csv
import sys

MATCH = ("k_walk<false", "k_part", "k_unpart", "k_gather")


def main(path, last=12):
    rows = [r for r in csv.DictReader(open(path))
            if any(m in r["Kernel_Name"] for m in MATCH)]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    prev = None
    for r in rows[-last:]:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        gap = (s - prev) / 1e3 if prev else 0.0
        print(f"{r['Kernel_Name'][:48]:48s} {((e - s) / 1e3):9.2f} gap {gap:7.2f}")
        prev = e


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 12)
