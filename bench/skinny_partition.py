#!/usr/bin/env python3
"""The skinny GEMM (M <= 64) on a CU partition vs the whole chip: device
time and weight bandwidth of the Llama-3-8B layer GEMMs (qkv, o, gate/up,
down) at a micro-forward's row counts, alone on the GPU (no serving steps
next to it).  The bound a realtime micro-forward on ``--micro-cus`` CUs can
reach (docs/performance.md "Realtime modes").

    python bench/skinny_partition.py [--micro-cus 32]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--micro-cus", type=int, default=32)
    a = ap.parse_args()
    import torch

    from llm_message_queue_amd.backend.cu_partition import partition_streams
    from llm_message_queue_amd.ops import gemm as G
    dev = torch.device("cuda", 0)
    big, micro, _n = partition_streams(dev, a.micro_cus)
    shapes = {"qkv": (6144, 4096, G.SK_STORE), "o": (4096, 4096, G.SK_RESID),
              "gate_up": (28672, 4096, G.SK_SWIGLU), "down": (4096, 14336, G.SK_RESID)}
    ws = {k: (torch.randn(n, kk, device=dev) * 0.02).to(torch.bfloat16) for k, (n, kk, _e) in shapes.items()}

    def run(stream, cus, M, reps=10):
        out = {}
        with torch.cuda.stream(stream):
            for name, (N, K, epi) in shapes.items():
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                o = torch.zeros(M, N // 2 if epi == G.SK_SWIGLU else N, device=dev, dtype=torch.bfloat16)
                r = torch.ones(M, device=dev)
                f = lambda: G.skinny(x, ws[name], o, epi, row_scale=r if epi != G.SK_RESID else None, cus=cus)
                for _ in range(2):
                    f()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(reps):
                    f()
                e1.record()
                e1.synchronize()
                us = e0.elapsed_time(e1) / reps * 1e3
                out[name] = {"us": round(us, 1), "weight_TBps": round(N * K * 2 / us / 1e6, 3),
                             "splits": G.skinny_splits(N, K, cus)}
        return out

    full = G._cu_count_idx(0)
    for M in (8, 32, 64):
        for label, st, cus in (("partition", micro, a.micro_cus), ("chip", torch.cuda.current_stream(dev), full)):
            res = run(st, cus, M)
            layer_us = sum(v["us"] for v in res.values())
            print(json.dumps({"M": M, "where": label, "cus": cus, "gemms": res,
                              "layer_gemm_us": round(layer_us, 1),
                              "forward_gemm_ms_32_layers": round(layer_us * 32 / 1e3, 2)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
