#!/usr/bin/env python3
"""Fixed per-tile cost of the hand-written 256x256 GEMM: device time of one
and of several full waves of tiles at K = 1024 ... 8192, fitted as
t = a + b * K per wave.  ``a`` is what a tile pays outside its K-loop
(launch / pipeline fill, epilogue, block turnover); it bounds what a
persistent kernel overlapping one tile's epilogue with the next tile's
prologue could recover.

    python bench/gemm_fixed_overhead.py
"""
from __future__ import annotations

import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    import numpy as np
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

    M = 4096
    for waves, epi in ((1, "store"), (7, "store"), (7, "swiglu"), (1, "resid")):
        N = 256 * (cus * waves // 16)                 # 16 row tiles x N/256 column tiles = waves x CUs
        pts = []
        for K in (1024, 2048, 4096, 8192):
            x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            if epi == "store":
                us = timed(lambda: G.gemm(x, w))
            elif epi == "swiglu":
                wp = G.swiglu_permute(w)
                us = timed(lambda: G.gemm_swiglu(x, wp))
            else:
                res = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
                us = timed(lambda: G.gemm_residual(x, w, res))
            pts.append((K, us))
            del x, w
        k = np.array([p[0] for p in pts], dtype=np.float64)
        t = np.array([p[1] for p in pts], dtype=np.float64)
        b, a = np.polyfit(k, t, 1)
        per_wave_a = a / waves
        print(json.dumps({"epi": epi, "M": M, "N": N, "waves": waves, "cus": cus,
                          "us_by_K": {int(K): round(us, 1) for K, us in pts},
                          "fit_fixed_us": round(a, 2), "fit_fixed_us_per_wave": round(per_wave_a, 2),
                          "fit_us_per_1k_K_per_wave": round(b * 1024 / waves, 2),
                          "fixed_share_at_K4096": round(a / (a + b * 4096), 4),
                          "pflops_at_K4096": round(2 * M * N * 4096 / dict(pts)[4096] / 1e9, 3)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
