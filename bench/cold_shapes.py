#!/usr/bin/env python3
"""First-use cost of forward shapes the saturated warm-up never ran.

The headline bench calibrates in saturation (every step ~token_budget
tokens) and then starts the timed window from an empty system, whose first
steps are small (T = tens..hundreds of tokens).  This probe measures, for a
Llama-3-8B-shaped stub already warmed at T = token_budget, the host wall time
of the FIRST forward at each new T and of a repeat at the same T.  A large
first/repeat gap means per-shape one-time work (GEMM heuristics / kernel code
object loading) lands on live requests.

    python bench/cold_shapes.py [--budget 4096] [--ts 1,7,33,...]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=1536)
    ap.add_argument("--ts", default="1,7,19,33,64,100,161,250,384,511,777,1000,1500,2000,3000,3500")
    ap.add_argument("--bucket", type=int, default=0, help="pad T up to a multiple of this (0 = off)")
    ap.add_argument("--json-out", default="")
    a = ap.parse_args()
    import torch
    from llm_message_queue_amd.models.llama_stub import LlamaConfig, LlamaStub

    dev = torch.device("cuda", 0)
    m = LlamaStub(LlamaConfig.llama3_8b(), a.slots, 512, device=dev, impl="hip")

    def fwd(T):
        Tp = -(-T // a.bucket) * a.bucket if a.bucket else T
        tok = torch.randint(0, 1000, (Tp,), device=dev, dtype=torch.long)
        pos = (torch.arange(Tp, device=dev, dtype=torch.int32) % 64)
        slot = (torch.arange(Tp, device=dev, dtype=torch.int32) // 64) % a.slots
        # tiles: 16-token segments of consecutive positions (prefill-like)
        n = (Tp + 15) // 16
        t0 = torch.arange(n, device=dev, dtype=torch.int32) * 16
        tiles = torch.stack([t0, torch.clamp(Tp - t0, max=16), (t0 // 64) % a.slots, t0 % 64], 1).contiguous()
        samp = torch.arange(min(Tp, 64), device=dev, dtype=torch.long)
        torch.cuda.synchronize()
        h0 = time.perf_counter()
        m.forward(tok, pos, slot, samp, tiles=tiles, n_dec=0)
        torch.cuda.synchronize()
        return (time.perf_counter() - h0) * 1e3

    for _ in range(5):
        fwd(a.budget)
    warm_full = fwd(a.budget)
    rows = []
    for T in [int(x) for x in a.ts.split(",")]:
        c = fwd(T)
        w = fwd(T)
        rows.append({"T": T, "first_ms": round(c, 2), "repeat_ms": round(w, 2), "extra_ms": round(c - w, 2)})
        print(json.dumps(rows[-1]), flush=True)
    out = {"budget": a.budget, "bucket": a.bucket, "warm_full_ms": round(warm_full, 2), "rows": rows,
           "sum_extra_ms": round(sum(r["extra_ms"] for r in rows), 1)}
    print(json.dumps(out), flush=True)
    if a.json_out:
        with open(a.json_out, "w") as fh:
            json.dump(out, fh, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
