"""Does the library GEMM on the o / down projections (``res.addmm_(x, W^T)``,
hipBLASLt beta = 1) run faster when the token count M is rounded up to a
tile multiple?  The serving step's M is the step's token count (4041-4096 at
the bench's 4096-token budget); rows past M are scratch rows of the same
preallocated buffers.  Times each M as-is and rounded up to 64 / 256, plus
the hand-written residual-epilogue kernel at the same M.

    python bench/gemm_m_align.py [--tokens 4041,4064,...] [--iters 40]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

GEMMS = {"o": (4096, 4096), "down": (4096, 14336)}


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
    ap.add_argument("--tokens", default="3000,3900,4000,4032,4041,4064,4080,4088,4092,4095,4096")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--hip", action="store_true", help="also time ops.gemm.gemm_residual")
    a = ap.parse_args()
    dev = torch.device("cuda")
    G = None
    if a.hip:
        from llm_message_queue_amd.ops import gemm as G
    rows = 4352
    for name, (N, K) in GEMMS.items():
        x = torch.randn(rows, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
        res = torch.randn(rows, N, device=dev, dtype=torch.bfloat16)
        for T in [int(t) for t in a.tokens.split(",")]:
            row = {"gemm": name, "T": T}
            for al in (1, 64, 256):
                Mp = (T + al - 1) // al * al
                row[f"ms_m{al}"] = round(timeit(lambda: res[:Mp].addmm_(x[:Mp], w.t()), a.iters), 4)
            if G is not None:
                row["ms_hip_resid"] = round(timeit(lambda: G.gemm_residual(x[:T], w, res[:T]), a.iters), 4)
            print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
