#!/usr/bin/env python3
"""Small-step GEMMs at 65-256 rows, the library-free path's weak spot at low
load (a ~165-token step at 30 % load): the skinny kernel with 64-row A
chunks (``G.skinny``) vs the 256x256-tile kernel with split-K
(``split_cus``, today's library-free route) vs hipBLASLt, for the four layer
GEMMs of Llama-3-8B; plus the fp32 check of the chunked skinny output.
Device time from events around 20 repeats.

    python bench/skinny_chunked.py
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

    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    only = os.environ.get("SK_GEMMS", "")
    if only:
        shapes = {k: v for k, v in shapes.items() if k in only.split(",")}
    ms = tuple(int(m) for m in os.environ.get("SK_MS", "48,65,128,165,200,256").split(","))
    for name, (N, K) in shapes.items():
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        for M in ms:
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            row = {"gemm": name, "M": M, "N": N, "K": K}
            if name == "o" or name == "down":
                res = torch.randn(M, N, device=dev).to(torch.bfloat16)
                want = res.float() + x.float() @ w.float().t()
                got = res.clone()
                G.skinny(x, w, got, G.SK_RESID, cus=cus)
                torch.cuda.synchronize()
                row["skinny_max_err_rel"] = round(((got.float() - want).abs().max() / want.abs().max()).item(), 5)
                r2 = res.clone()
                row["skinny_us"] = round(timed(lambda: G.skinny(x, w, r2, G.SK_RESID, cus=cus)), 1)
                row["tiles_split_us"] = round(timed(lambda: G.gemm_residual(x, w, r2, split_cus=cus)), 1)
                row["hipblaslt_us"] = round(timed(lambda: r2.addmm_(x, w.t())), 1)
            else:
                out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
                G.skinny(x, w, out, G.SK_STORE, cus=cus)
                torch.cuda.synchronize()
                want = x.float() @ w.float().t()
                row["skinny_max_err_rel"] = round(((out.float() - want).abs().max() / want.abs().max()).item(), 5)
                row["skinny_us"] = round(timed(lambda: G.skinny(x, w, out, G.SK_STORE, cus=cus)), 1)
                row["tiles_split_us"] = round(timed(lambda: G.gemm(x, w, out, split_cus=cus)), 1)
                row["hipblaslt_us"] = round(timed(lambda: torch.mm(x, w.t(), out=out)), 1)
            print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
