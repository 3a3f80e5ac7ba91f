#!/usr/bin/env python3
"""o / down projections into the residual at the row counts the serving
steps give the library today: the pruned last layer's
sampled rows (~900-1,100) and sub-wave steps.  Times, per (M, K):

* hipBLASLt ``res.addmm_(x, w.t())`` (beta = 1, what ``residual_tiles_ok``
  routes these shapes to);
* the hand-written residual GEMM, whole tiles;
* the same with every tile split over two K-halves (``split_cus``);
* the skinny kernel where M <= 64.

One JSON line per shape; device time from events around 20 repeats.

    python bench/resid_small_m.py
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
    N = 4096

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
        return a.elapsed_time(b) / reps * 1e3          # us

    for K in (4096, 14336):
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        for M in (16, 64, 300, 700, 900, 1000, 1100, 2000, 3000, 3500):
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            res = torch.randn(M, N, device=dev).to(torch.bfloat16)
            row = {"M": M, "K": K, "N": N, "tiles": -(-M // 256) * (N // 256), "cus": cus}
            row["hipblaslt_us"] = round(timed(lambda: res.addmm_(x, w.t())), 1)
            row["hip_whole_us"] = round(timed(lambda: G.gemm_residual(x, w, res)), 1)
            if G.split_all(M, N, K, cus) is not None:
                row["hip_split2_us"] = round(timed(lambda: G.gemm_residual(x, w, res, split_cus=cus)), 1)
            if M <= G.SKINNY_MAX_M:
                row["skinny_us"] = round(timed(lambda: G.skinny(x, w, res, G.SK_RESID, cus=cus)), 1)
            print(json.dumps(row), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
