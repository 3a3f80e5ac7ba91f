#!/usr/bin/env python3
"""Split-K factor of the skinny GEMM at 65-256 rows (128-row A chunks):
more splits fill more CUs but write S x M x N fp32 partials that the
finalize kernel re-reads.  Device time per (GEMM, M, S) next to hipBLASLt.

    python bench/skinny_splits_sweep.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import torch

    from llm_message_queue_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    cus = G._cu_count(dev)

    def timed(fn, reps=20):
        for _ in range(3):
            fn()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) / reps * 1e3

    only = os.environ.get("SWEEP_ONLY", "")
    shapes = {"qkv": (6144, 4096, G.SK_STORE), "o": (4096, 4096, G.SK_RESID), "down": (4096, 14336, G.SK_RESID),
              "gate_up": (28672, 4096, G.SK_SWIGLU)}
    if only:
        shapes = {k: v for k, v in shapes.items() if k in only.split(",")}
    for name, (N, K, epi) in shapes.items():
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        for M in (96, 128, 165, 200, 256):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            o = torch.zeros(M, N // 2 if epi == G.SK_SWIGLU else N, device=dev, dtype=torch.bfloat16)
            row = {"gemm": name, "M": M, "default_S": G.skinny_splits(N, K, cus, M)}
            for S in (1, 2, 4, 8, 16):
                if K % (128 * S) or K // S < 256:
                    continue
                row[f"S{S}_us"] = round(timed(lambda: G.skinny(x, w, o, epi, cus=cus, splits=S)), 1)
            if epi == G.SK_SWIGLU:
                wp = G.swiglu_permute(w)
                row["tiles_split_us"] = round(timed(lambda: G.gemm_swiglu(x, wp, o, split_cus=cus)), 1)
                big = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                row["hipblaslt_us"] = round(timed(lambda: torch.mm(x, w.t(), out=big)), 1)
            else:
                row["hipblaslt_us"] = round(timed(lambda: o.addmm_(x, w.t()) if epi == G.SK_RESID
                                                  else torch.mm(x, w.t(), out=o)), 1)
            print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
