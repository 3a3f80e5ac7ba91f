"""Token-count padding for the serving GEMMs: a continuous-batching step has
an arbitrary token count T; hipBLASLt's kernel choice (and its stream-K tail)
depends on T.  Compare the four layer GEMMs at T against T rounded up to a
multiple of 64 / 128 / 256 (the padded rows cost nothing in tile count when
the rounding stays inside the last 256-row tile).

    python bench/gemm_pad.py [--tokens 1500,2222,...] [--iters 20]
"""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F

GEMMS = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}


def timeit(fn, iters):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def layer_ms(T, ws, xs, iters):
    return sum(timeit(lambda: F.linear(xs[K][:T], w), iters) for (N, K), w in ws.items())


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="1100,1517,1800,2049,2300,2611,2900,3100,3333,3600,3790,3900,3974,4000,4050")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    ws = {(N, K): torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02 for N, K in GEMMS.values()}
    xs = {K: torch.randn(8192, K, device=dev, dtype=torch.bfloat16) for K in (4096, 14336)}
    tot = {"raw": 0.0, "p64": 0.0, "p128": 0.0, "p256": 0.0}
    for T in [int(t) for t in a.tokens.split(",")]:
        row = {"T": T}
        for tag, m in (("raw", 1), ("p64", 64), ("p128", 128), ("p256", 256)):
            Tp = -(-T // m) * m
            row[tag] = round(layer_ms(Tp, ws, xs, a.iters), 4)
            tot[tag] += row[tag]
        print(json.dumps(row), flush=True)
    print(json.dumps({"sum_ms": {k: round(v, 3) for k, v in tot.items()}}), flush=True)


if __name__ == "__main__":
    main()
