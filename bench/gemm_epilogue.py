"""Residual-accumulating projections: does ``res.addmm_(x, W^T)`` (hipBLASLt
with beta = 1, the residual add folded into the GEMM epilogue) cost more than
the plain ``F.linear`` it would replace?  If not, the o / down projections can
write straight into the residual stream and the following RMSNorm only reads
it (half the RMSNorm traffic).

    python bench/gemm_epilogue.py [--tokens 3968,4096] [--iters 30]
"""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F

GEMMS = {"o": (4096, 4096), "down": (4096, 14336), "qkv": (6144, 4096), "gate_up": (28672, 4096)}


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="3968,4096")
    ap.add_argument("--iters", type=int, default=30)
    a = ap.parse_args()
    dev = torch.device("cuda")
    for T in [int(t) for t in a.tokens.split(",")]:
        for name, (N, K) in GEMMS.items():
            x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            w = (torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02)
            res = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
            fl = 2.0 * T * N * K
            row = {"gemm": name, "T": T}
            row["linear_ms"] = round(timeit(lambda: F.linear(x, w), a.iters), 4)
            if N == 4096:
                row["linear_plus_add_ms"] = round(timeit(lambda: res.add_(F.linear(x, w)), a.iters), 4)
                row["addmm_beta1_ms"] = round(timeit(lambda: res.addmm_(x, w.t()), a.iters), 4)
                ref = res.float() + F.linear(x, w).float()
                r2 = res.clone()
                r2.addmm_(x, w.t())
                row["addmm_max_err"] = round(float((r2.float() - ref).abs().max()), 4)
            row["tflops_linear"] = round(fl / row["linear_ms"] / 1e9, 1)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
