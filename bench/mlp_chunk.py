"""MLP block in row chunks: does splitting the step's tokens so one chunk's
gate_up output (T/c x 28672 bf16) stays in the 256 MB Infinity Cache make
the SiLU-mul and the down GEMM read it from the cache instead of HBM?

    python bench/mlp_chunk.py [--tokens 4096] [--chunks 1,2,4] [--iters 20]

Prints one JSON line per chunk count: MLP-block ms (gate_up -> silu_mul ->
down with the residual accumulated in the GEMM, as ``LlamaStub.hidden``) and
the split into its three ops measured at chunk count 1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


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
    ap.add_argument("--tokens", type=int, default=4096)
    ap.add_argument("--chunks", default="1,2,4")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from llm_message_queue_amd.ops.llama_ops import get_ops
    ops = get_ops("hip")
    dev = torch.device("cuda")
    T, d, f = a.tokens, 4096, 14336
    # 4 layers' worth of distinct weights so the chunked run cannot keep one
    # layer's weights cache-resident across iterations any more than the model does
    Ws = [((torch.randn(2 * f, d, device=dev, dtype=torch.bfloat16) * 0.02),
           (torch.randn(d, f, device=dev, dtype=torch.bfloat16) * 0.02)) for _ in range(4)]
    x2 = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
    res = torch.randn(T, d, device=dev, dtype=torch.bfloat16)

    def mlp(c):
        def run():
            step = T // c
            for wgu, wd in Ws:
                for r0 in range(0, T, step):
                    gu = F.linear(x2[r0:r0 + step], wgu)
                    act = ops.silu_mul(gu)
                    res[r0:r0 + step].addmm_(act, wd.t())
        return run

    # numerics: chunking is row-separable, results must match bitwise-closely
    r_save = res.clone()
    mlp(1)()
    one = res.clone()
    res.copy_(r_save)
    mlp(2)()
    diff = float((res.float() - one.float()).abs().max())
    res.copy_(r_save)

    gu = F.linear(x2, Ws[0][0])
    act = ops.silu_mul(gu)
    split = {"gate_up_ms": timeit(lambda: F.linear(x2, Ws[0][0]), a.iters),
             "silu_mul_ms": timeit(lambda: ops.silu_mul(gu), a.iters),
             "down_ms": timeit(lambda: res.addmm_(act, Ws[0][1].t()), a.iters)}
    for c in [int(x) for x in a.chunks.split(",")]:
        ms = timeit(mlp(c), a.iters) / len(Ws)
        print(json.dumps({"tokens": T, "chunks": c, "mlp_ms_per_layer": round(ms, 4),
                          "max_abs_diff_vs_1chunk": diff if c == 2 else None,
                          **({k: round(v, 4) for k, v in split.items()} if c == 1 else {})}), flush=True)


if __name__ == "__main__":
    main()
