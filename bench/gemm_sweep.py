"""Backend GEMM roofline check: the four per-layer GEMMs of the Llama-3-8B stub
at the token counts a serving step sees, through ``F.linear`` (hipBLASLt).

    python bench/gemm_sweep.py [--tokens 1024,2048,4096,8192] [--iters 20]

Prints one JSON line per (gemm, T) with achieved TFLOP/s.  Run once plain and
once with ``PYTORCH_TUNABLEOP_ENABLED=1`` to see what per-shape tuning buys.
"""
from __future__ import annotations

import argparse
import json

import torch
import torch.nn.functional as F

GEMMS = {  # name: (N, K)
    "qkv": (6144, 4096),
    "o": (4096, 4096),
    "gate_up": (28672, 4096),
    "down": (4096, 14336),
    "lm_head": (128256, 4096),
}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", default="1024,2048,3072,4096,6144,8192")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--blas", default="", help="hipblaslt | rocblas (default: torch's choice)")
    a = ap.parse_args()
    if a.blas:
        torch.backends.cuda.preferred_blas_library("cublaslt" if a.blas == "hipblaslt" else "cublas")
    dev = torch.device("cuda")
    tot_t = tot_f = 0.0
    for T in [int(x) for x in a.tokens.split(",")]:
        for name, (N, K) in GEMMS.items():
            if name == "lm_head" and T > 2048:
                continue
            x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16)
            for _ in range(3):
                F.linear(x, w)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(a.iters):
                F.linear(x, w)
            e.record()
            e.synchronize()
            ms = s.elapsed_time(e) / a.iters
            fl = 2.0 * T * N * K
            if name != "lm_head":
                tot_t += ms
                tot_f += fl
            print(json.dumps({"gemm": name, "T": T, "N": N, "K": K, "ms": round(ms, 4),
                              "tflops": round(fl / ms / 1e9, 1)}), flush=True)
    print(json.dumps({"layer_gemms_tflops": round(tot_f / tot_t / 1e9, 1)}), flush=True)


if __name__ == "__main__":
    main()
