"""Break the library-GEMM time of a rocprofv3 kernel trace down by layer role.

    python scripts/gemm_roles.py gpurun_out/prof/run_kernel_trace.csv

A GEMM's role is read from the kernel that ran just before it in the serving
forward (rmsnorm -> qkv or gate_up, attention -> o, silu_mul -> down); the
grid size tells qkv and gate_up apart.
"""
from __future__ import annotations

import collections
import csv
import sys


def main(path: str) -> None:
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                         int(r["Grid_Size_X"]), int(r["Grid_Size_Y"])))
    rows.sort()
    prev = ""
    stats = collections.defaultdict(list)
    for s, e, n, gx, gy in rows:
        short = n.split("(")[0]
        is_gemm = n.startswith("Cijk") or n.startswith("Custom_Cijk")
        if is_gemm:
            role = {"llmq::rmsnorm_kernel": "qkv|gate_up", "llmq::attention_dec_kernel": "o",
                    "llmq::attention_seg_kernel": "o", "llmq::silu_mul_kernel": "down"}.get(prev, "other")
            mt = n.split("_MT")[1].split("_")[0] if "_MT" in n else "?"
            stats[(role, mt, gx, gy)].append(e - s)
            prev = "gemm"
        else:
            prev = short
    tot = sum(sum(v) for v in stats.values())
    print(f"{'role':12s} {'tile':12s} {'grid':>14s} {'calls':>6s} {'avg us':>8s} {'%':>6s}")
    for k, v in sorted(stats.items(), key=lambda kv: -sum(kv[1]))[:20]:
        print(f"{k[0]:12s} {k[1]:12s} {str(k[2]) + 'x' + str(k[3]):>14s} {len(v):6d} "
              f"{sum(v) / len(v) / 1e3:8.1f} {100 * sum(v) / tot:6.1f}")


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv")
