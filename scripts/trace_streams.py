#!/usr/bin/env python3
"""Per-stream view of a rocprofv3 kernel trace (``--kernel-trace``, CSV):
for each stream / queue, kernel count, summed kernel time, the span from its
first kernel to its last, busy fraction (union of its kernel intervals over
the span), and its top kernels.  Used for the realtime micro-forward
analysis (profiles/r6_realtime_modes.md): is a stream waiting for the GPU or
for the host that feeds it?

    python scripts/trace_streams.py gpurun_out/r6_prof_micro/<host>/<pid>_kernel_trace.csv [--from 0.3]
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import sys


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--from", dest="frac", type=float, default=0.3, help="skip this leading fraction of the trace")
    ap.add_argument("--top", type=int, default=8)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    if not rows:
        print("empty trace", file=sys.stderr)
        return 1
    key = "Stream_Id" if "Stream_Id" in rows[0] else ("Queue_Id" if "Queue_Id" in rows[0] else None)
    t0 = min(int(r["Start_Timestamp"]) for r in rows)
    t1 = max(int(r["End_Timestamp"]) for r in rows)
    cut = t0 + a.frac * (t1 - t0)
    by = collections.defaultdict(list)
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if s < cut:
            continue
        by[r.get(key, "?") if key else "?"].append((s, e, r["Kernel_Name"]))
    out = {"stream_key": key, "window_ms": round((t1 - cut) / 1e6, 2), "streams": {}}
    for sid, ks in sorted(by.items(), key=lambda kv: -len(kv[1])):
        ks.sort()
        span = ks[-1][1] - ks[0][0]
        busy, cur_s, cur_e = 0, ks[0][0], ks[0][1]
        for s, e, _ in ks[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        busy += cur_e - cur_s
        tot = collections.Counter()
        cnt = collections.Counter()
        for s, e, n in ks:
            short = n.split("(")[0][:90]
            tot[short] += e - s
            cnt[short] += 1
        out["streams"][str(sid)] = {
            "kernels": len(ks), "kernel_ms": round(sum(e - s for s, e, _ in ks) / 1e6, 2),
            "span_ms": round(span / 1e6, 2), "busy_frac": round(busy / max(1, span), 4),
            "top": [{"kernel": n, "calls": cnt[n], "ms": round(t / 1e6, 2), "avg_us": round(t / cnt[n] / 1e3, 1)}
                    for n, t in tot.most_common(a.top)]}
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
