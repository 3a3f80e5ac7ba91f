#!/usr/bin/env python3
"""A readable excerpt of a rocprofv3 kernel trace (``--kernel-trace``, CSV):
a window of ``--ms`` milliseconds starting ``--at`` (a fraction of the
trace), printed per stream as runs of back-to-back kernels.  Each run is one
line: start / end in ms from the window start, kernel count, and the first
and most frequent kernel names -- enough to see where a realtime
micro-forward lands between (or inside) the big serving steps
(profiles/r6_realtime_modes.md).

    python scripts/timeline_excerpt.py <run_kernel_trace.csv> [--at 0.5] [--ms 120] [--gap-us 40]
"""
from __future__ import annotations

import argparse
import collections
import csv
import re
import sys


def short(n: str) -> str:
    n = re.sub(r"\(.*", "", n)
    n = re.sub(r"<.*", "", n)
    return n.replace("void ", "").split("::")[-1][:40]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--at", type=float, default=0.5, help="window start as a fraction of the trace")
    ap.add_argument("--ms", type=float, default=120.0)
    ap.add_argument("--gap-us", type=float, default=40.0, help="a longer idle gap on a stream starts a new run")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    if not rows:
        print("empty trace", file=sys.stderr)
        return 1
    key = "Stream_Id" if "Stream_Id" in rows[0] else ("Queue_Id" if "Queue_Id" in rows[0] else None)
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    w0 = t0 + a.at * (t1 - t0)
    w1 = w0 + a.ms * 1e6
    by = collections.defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if e >= w0 and s <= w1:
            by[r.get(key, "?") if key else "?"].append((s, e, short(r["Kernel_Name"])))
    print(f"window {a.ms:.0f} ms at {a.at:.2f} of a {(t1 - t0) / 1e6:.0f} ms trace; runs split at idle gaps > "
          f"{a.gap_us:.0f} us")
    for sid, ks in sorted(by.items()):
        ks.sort()
        print(f"\n{key or 'stream'} {sid}: {len(ks)} kernels")
        run = [ks[0]]
        for k in ks[1:] + [None]:
            if k is not None and k[0] - run[-1][1] <= a.gap_us * 1e3:
                run.append(k)
                continue
            names = collections.Counter(x[2] for x in run)
            top = ", ".join(f"{n} x{c}" for n, c in names.most_common(3))
            print(f"  {(run[0][0] - w0) / 1e6:8.2f} .. {(run[-1][1] - w0) / 1e6:8.2f} ms  "
                  f"{len(run):4d} kernels  [{top}]")
            if k is not None:
                run = [k]
    return 0


if __name__ == "__main__":
    sys.exit(main())
