#!/usr/bin/env python3
"""A/B of the persistent form of the hand-written GEMM (one block per CU
walking the tiles, ``GM_PERSIST_FLAG``) against one block per tile, at the
serving step's shapes (T ~ 4,091 tokens of Llama-3-8B).  Alternating rounds,
device time from events around ``--reps`` launches; the outputs of the two
forms must be bitwise equal (same tiles, same K order).

    python bench/gemm_persist_ab.py [--rounds 3] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PERSIST = 256


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--M", type=int, default=4091)
    a = ap.parse_args()
    import torch

    from llm_message_queue_amd import _native
    from llm_message_queue_amd.ops import gemm as G
    k = _native.require_hipops()
    dev = torch.device("cuda", 0)
    M = a.M
    shapes = [("qkv_store", 6144, 4096, G.EPI_STORE), ("gate_up", 28672, 4096, G.EPI_SWIGLU),
              ("o", 4096, 4096, G.EPI_RESID_LDS), ("down", 4096, 14336, G.EPI_RESID_LDS),
              ("head_store", 16384, 4096, G.EPI_STORE)]

    def launch(x, w, out, epi):
        st = torch.cuda.current_stream(dev).cuda_stream
        k.gemm_bf16(x.data_ptr(), w.data_ptr(), out.data_ptr(), x.shape[0], w.shape[0], x.shape[1], epi, st, 8,
                    0, 0, 0, 0)

    def timed(fn, reps):
        for _ in range(2):
            fn()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3

    for name, N, K, epi in shapes:
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        if epi == G.EPI_SWIGLU:
            w = G.swiglu_permute(w)
        ncol = N // 2 if epi == G.EPI_SWIGLU else N
        base = torch.randn(M, ncol, device=dev).to(torch.bfloat16)
        outs = {}
        for tag, e in (("plain", epi), ("persist", epi | PERSIST)):
            o = base.clone()
            launch(x, w, o, e)
            torch.cuda.synchronize()
            outs[tag] = o
        equal = bool(torch.equal(outs["plain"], outs["persist"]))
        times = {"plain": [], "persist": []}
        for _ in range(a.rounds):
            for tag, e in (("plain", epi), ("persist", epi | PERSIST)):
                o = base.clone()
                times[tag].append(timed(lambda: launch(x, w, o, e), a.reps))
        tp, tq = statistics.median(times["plain"]), statistics.median(times["persist"])
        flop = 2.0 * M * N * K
        print(json.dumps({"gemm": name, "M": M, "N": N, "K": K, "epi": epi, "bitwise_equal": equal,
                          "plain_us": round(tp, 1), "persist_us": round(tq, 1),
                          "speedup": round(tp / tq, 4), "persist_pflops": round(flop / tq / 1e9, 3),
                          "plain_runs": [round(t, 1) for t in times["plain"]],
                          "persist_runs": [round(t, 1) for t in times["persist"]]}), flush=True)
        del x, w, base, outs
    return 0


if __name__ == "__main__":
    sys.exit(main())
