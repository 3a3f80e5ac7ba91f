"""Idle gaps between consecutive kernels of a rocprofv3 kernel trace.

    python scripts/gap_histogram.py gpurun_out/prof/run_kernel_trace.csv [--tail 0.6]

Splits GPU idle time into inter-kernel bubbles (launch latency, < 20 us) and
host stalls (>= 20 us), over the last ``--tail`` fraction of the trace (the
serving loop), to tell whether HIP-graph capture (removes bubbles) or host
work (removes stalls) is the lever.
"""
from __future__ import annotations

import argparse
import csv


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("trace", nargs="?", default="gpurun_out/prof/run_kernel_trace.csv")
    ap.add_argument("--tail", type=float, default=0.6)
    a = ap.parse_args()
    iv = []
    with open(a.trace) as f:
        for r in csv.DictReader(f):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
    t0 = iv[0][0] + (1 - a.tail) * (iv[-1][1] - iv[0][0])
    iv = [x for x in iv if x[0] >= t0]
    span = iv[-1][1] - iv[0][0]
    edges = [0, 2_000, 5_000, 20_000, 100_000, 1_000_000, 10**12]
    hist = [[0, 0] for _ in edges[:-1]]
    end = iv[0][1]
    for s, e in iv[1:]:
        g = s - end
        if g > 0:
            for i in range(len(edges) - 1):
                if edges[i] <= g < edges[i + 1]:
                    hist[i][0] += 1
                    hist[i][1] += g
                    break
        end = max(end, e)
    idle = sum(h[1] for h in hist)
    print(f"window {span / 1e6:.1f} ms, idle {idle / 1e6:.1f} ms ({100 * idle / span:.1f}%)")
    for i, (n, tot) in enumerate(hist):
        lo, hi = edges[i] / 1e3, edges[i + 1] / 1e3
        print(f"  gaps [{lo:>7.0f}, {hi:>9.0f}) us: {n:7d}  {tot / 1e6:8.2f} ms  {100 * tot / span:5.2f}%")


if __name__ == "__main__":
    main()
