"""The residual GEMM with the fused RMSNorm row-scale epilogue against the
plain residual GEMM followed by the separate ``row_rms`` pass it replaces
(o: K = 4096, down: K = 14336, N = 4096), at serving token counts.  Median
of ``--iters`` event-timed calls per variant, ``--rounds`` alternating
rounds; one JSON line per (T, shape)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_message_queue_amd.ops import gemm as G
from llm_message_queue_amd.ops.llama_ops import HipOps


def timed(fn, iters):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for _ in range(3):
        fn()
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in ev)
    return ms[len(ms) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="4041,4091,4096")
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda")
    ops = HipOps()
    for T in [int(t) for t in a.tokens.split(",")]:
        for name, K in (("o", 4096), ("down", 14336)):
            x = ((torch.rand(T, K, device=dev) * 2 - 1)).to(torch.bfloat16)
            w = ((torch.rand(4096, K, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16)
            res = torch.randn(T, 4096, device=dev).to(torch.bfloat16)
            r = {"T": T, "gemm": name, "plain_ms": [], "row_rms_ms": [], "plain_plus_row_rms_ms": [], "fused_ms": []}
            for _ in range(a.rounds):
                r["plain_ms"].append(timed(lambda: G._launch(x, w, res, G.EPI_RESID_LDS), a.iters))
                r["row_rms_ms"].append(timed(lambda: ops.row_rms(res, 1e-5), a.iters))
                r["plain_plus_row_rms_ms"].append(
                    timed(lambda: (G._launch(x, w, res, G.EPI_RESID_LDS), ops.row_rms(res, 1e-5)), a.iters))
                r["fused_ms"].append(timed(lambda: G.gemm_residual_rms(x, w, res, 1e-5), a.iters))
            for k in list(r):
                if k.endswith("_ms"):
                    r[k] = round(sorted(r[k])[len(r[k]) // 2], 4)
            r["saved_us"] = round((r["plain_plus_row_rms_ms"] - r["fused_ms"]) * 1e3, 2)
            print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
