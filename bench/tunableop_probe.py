"""Would a searched hipBLASLt / rocBLAS solution beat the default heuristic on
the two projections still on the library (o and down, ``res.addmm_(x, W^T)``
with beta = 1)?  PyTorch's TunableOp times every candidate solution for a
shape on first use; this probe times the serving shapes with the default
pick and with the tuned pick (``--tunable``) in separate processes.

    python bench/tunableop_probe.py [--tunable] [--tokens 4041,4096] [--iters 40]
"""
from __future__ import annotations

import argparse
import json
import os

import torch

GEMMS = {"o": (4096, 4096), "down": (4096, 14336)}


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
    ap.add_argument("--tokens", default="4041,4096")
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--tunable", action="store_true")
    ap.add_argument("--results", default="gpurun_out/tunableop_results.csv")
    a = ap.parse_args()
    if a.tunable:
        os.makedirs(os.path.dirname(a.results) or ".", exist_ok=True)
        torch.cuda.tunable.enable(True)
        torch.cuda.tunable.tuning_enable(True)
        torch.cuda.tunable.set_filename(a.results)
        torch.cuda.tunable.set_max_tuning_duration(200)
    dev = torch.device("cuda")
    for T in [int(t) for t in a.tokens.split(",")]:
        for name, (N, K) in GEMMS.items():
            x = torch.randn(T, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.02
            res = torch.randn(T, N, device=dev, dtype=torch.bfloat16)
            ms = timeit(lambda: res.addmm_(x, w.t()), a.iters)
            print(json.dumps({"gemm": name, "T": T, "tunable": a.tunable, "addmm_beta1_ms": round(ms, 4),
                              "tflops": round(2.0 * T * N * K / ms / 1e9, 1)}), flush=True)
    if a.tunable:
        torch.cuda.tunable.write_file()


if __name__ == "__main__":
    main()
