"""Summarise a rocprofv3 ``--kernel-trace --stats --output-format csv`` run into
a short markdown report (for ``profiles/``).

    python scripts/prof_summary.py gpurun_out/prof/run > profiles/bench_kernels.md

Reports the top kernels by total time, a per-category roll-up (library GEMM,
our HIP kernels, PyTorch elementwise), and GPU busy fraction / per-step
statistics over the densest window of the trace (the serving loop).
"""
from __future__ import annotations

import csv
import re
import sys
from collections import defaultdict

CATEGORIES = [
    ("gemm+swiglu (HIP)", re.compile(r"gemm_bf16_kernel")),
    ("skinny gemm (HIP)", re.compile(r"skinny_(partial|finalize)_kernel")),
    ("lm-head argmax (HIP)", re.compile(r"gemm_argmax_reduce_kernel")),
    ("gemm (hipBLASLt)", re.compile(r"^(Custom_)?Cijk_|gemm|Gemm")),
    ("attention (HIP)", re.compile(r"attention|attn")),
    ("rmsnorm (HIP)", re.compile(r"rmsnorm")),
    ("silu_mul (HIP)", re.compile(r"silu")),
    ("rope_kv (HIP)", re.compile(r"rope")),
    ("text/classifier/summary (HIP)", re.compile(r"text_analyze|scan_rows|embed_pool|classify|summarise|salient")),
    ("slot census (HIP)", re.compile(r"census")),
    ("host link copies (HIP)", re.compile(r"copy_bytes")),
    ("torch elementwise/index", re.compile(r"elementwise|index|gather|scatter|copy|fill|reduce|arange|cat")),
]


def short(name: str, n: int = 90) -> str:
    s = re.sub(r"\(.*", "", name)
    s = re.sub(r"<.*", "", s)
    s = s.replace("void ", "")
    return s if len(s) <= n else s[: n - 3] + "..."


def category(name: str) -> str:
    for cat, rx in CATEGORIES:
        if rx.search(name):
            return cat
    return "other"


def from_db(path: str, tail_frac: float = 1.0):
    """rocprofv3 SQLite output (``run_results.db``): per-kernel stats and
    the dispatch intervals, optionally only the last ``tail_frac`` of the
    trace (the serving loop after calibration)."""
    import sqlite3
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end from kernels"))
    if not rows:
        return [], []
    t_lo = min(r[1] for r in rows)
    t_hi = max(r[2] for r in rows)
    cut = t_hi - tail_frac * (t_hi - t_lo)
    rows = [r for r in rows if r[1] >= cut]
    agg = defaultdict(lambda: [0, 0])
    for n, a, b in rows:
        agg[n][0] += 1
        agg[n][1] += b - a
    total = sum(v[1] for v in agg.values()) or 1
    stats = [{"Name": n, "Calls": str(v[0]), "TotalDurationNs": str(v[1]), "AverageNs": str(v[1] / v[0]),
              "Percentage": str(100.0 * v[1] / total)} for n, v in sorted(agg.items(), key=lambda kv: -kv[1][1])]
    trace = [{"Start_Timestamp": str(a), "End_Timestamp": str(b)} for _, a, b in rows]
    return stats, trace


def main(prefix: str, tail_frac: float = 1.0) -> None:
    if prefix.endswith(".db"):
        stats, tr_db = from_db(prefix, tail_frac)
    else:
        stats, tr_db = list(csv.DictReader(open(prefix + "_kernel_stats.csv"))), None
    total = sum(int(r["TotalDurationNs"]) for r in stats) or 1
    print(f"# Kernel profile: `{prefix.split('/')[-1]}`\n")
    print(f"Total kernel time {total / 1e6:.1f} ms over {sum(int(r['Calls']) for r in stats)} dispatches.\n")
    print("## Top kernels\n\n| kernel | calls | total ms | avg us | % |\n|---|---:|---:|---:|---:|")
    for r in stats[:15]:
        print(f"| `{short(r['Name'])}` | {r['Calls']} | {int(r['TotalDurationNs']) / 1e6:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['Percentage']):.2f} |")
    cats = defaultdict(int)
    for r in stats:
        cats[category(r["Name"])] += int(r["TotalDurationNs"])
    print("\n## By category\n\n| category | total ms | % |\n|---|---:|---:|")
    for c, v in sorted(cats.items(), key=lambda kv: -kv[1]):
        print(f"| {c} | {v / 1e6:.1f} | {100 * v / total:.1f} |")
    if tr_db is not None:
        tr = tr_db
    else:
        try:
            tr = list(csv.DictReader(open(prefix + "_kernel_trace.csv")))
        except FileNotFoundError:
            return
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in tr)
    if not iv:
        return
    # busy fraction over the last 60% of the trace (serving loop, after load/warmup)
    t0 = iv[0][0] + int(0.4 * (iv[-1][1] - iv[0][0]))
    busy, cur_s, cur_e = 0, None, None
    for s, e in iv:
        if e <= t0:
            continue
        s = max(s, t0)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = iv[-1][1] - t0
    print(f"\n## Timeline (last 60% of trace)\n\nGPU busy {100 * busy / span:.1f}% of {span / 1e6:.1f} ms "
          f"(union of kernel intervals; gaps = host-side idle).")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 1.0)
