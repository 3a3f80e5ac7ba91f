"""QKV projection at T = 4096: the fused 4096 x 6144 GEMM runs ~15% below the
other layer GEMMs (384 256x256 tiles = 1.5 rounds over 256 CUs).  Does
splitting it into q (4096 x 4096 = 256 tiles, one round) and kv (4096 x 2048)
GEMMs -- written into column slices of one qkv buffer so the RoPE kernel is
unchanged -- beat it?

    python bench/qkv_split.py [--tokens 4096] [--iters 50]
"""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F


def timeit(fn, iters):
    for _ in range(5):
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
    ap.add_argument("--tokens", default="3968,4096")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda")
    d, nq, nkv = 4096, 4096, 2048
    w = torch.randn(nq + nkv, d, device=dev, dtype=torch.bfloat16) * 0.02
    wq, wkv = w[:nq].contiguous(), w[nq:].contiguous()
    for T in [int(t) for t in a.tokens.split(",")]:
        x = torch.randn(T, d, device=dev, dtype=torch.bfloat16)
        out = torch.empty(T, nq + nkv, device=dev, dtype=torch.bfloat16)
        fused = timeit(lambda: F.linear(x, w), a.iters)

        def split_slices():
            torch.mm(x, wq.t(), out=out[:, :nq])
            torch.mm(x, wkv.t(), out=out[:, nq:])

        def split_separate():
            F.linear(x, wq)
            F.linear(x, wkv)

        t_slices = timeit(split_slices, a.iters)
        t_sep = timeit(split_separate, a.iters)
        split_slices()
        err = float((out.float() - F.linear(x, w).float()).abs().max())
        fl = 2.0 * T * (nq + nkv) * d
        print(json.dumps({"T": T, "fused_ms": round(fused, 4), "fused_tflops": round(fl / fused / 1e9, 1),
                          "split_into_slices_ms": round(t_slices, 4), "split_separate_ms": round(t_sep, 4),
                          "slices_max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
