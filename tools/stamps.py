"""Summarise SHM_GET_STAMPS dumps: per launch, kernel span, wave lifetime and
the occupancy profile (waves alive per 5 % of the span)."""
import json
import sys

import numpy as np


def main(path):
    raw = np.fromfile(path, dtype=np.uint64)
    i, out = 0, []
    while i < raw.size:
        n = int(raw[i]); st = raw[i + 1:i + 1 + n].reshape(-1, 2).astype(np.int64)
        i += 1 + n
        t0 = st[:, 0].min(); s = (st[:, 0] - t0) / 100.0; e = (st[:, 1] - t0) / 100.0
        span = e.max()
        grid = np.linspace(0, span, 21)
        alive = [int(((s <= g) & (e > g)).sum()) for g in grid[:-1] + span / 40]
        out.append({"waves": len(s), "span_us": round(float(span), 2),
                    "life_us_mean": round(float((e - s).mean()), 2),
                    "life_us_p50": round(float(np.median(e - s)), 2),
                    "start_us_p90": round(float(np.percentile(s, 90)), 2),
                    "end_us_p10": round(float(np.percentile(e, 10)), 2),
                    "alive_per_5pct": alive})
    print(json.dumps(out[-3:], indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
