"""A/B of the hand-written gfx950 GEMMs against hipBLASLt (F.linear).

  python bench/gemm_fused.py [--rounds 7] [--tokens 37,1024,2048,4041,4096]

* swiglu: F.linear(x, W_gu) + silu_mul (the model's unfused MLP front half)
  vs gemm_swiglu(x, W_perm) (one launch, SwiGLU epilogue).
* plain:  F.linear(x, W) vs gemm(x, W) for the qkv / o / gate_up / down shapes.

Numerics against an fp32 reference are printed first.  Timings are
interleaved rounds in one process (median of per-round means), random
normal activations and std-0.02 weights as in the model.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch
import torch.nn.functional as F

from llm_message_queue_amd.ops import gemm as G
from llm_message_queue_amd.ops.llama_ops import HipOps


def timeit(fn, iters):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--tokens", default="37,1024,2048,4041,4096")
    ap.add_argument("--plain", action="store_true", help="also time the plain GEMM shapes")
    ap.add_argument("--resid", action="store_true", help="A/B the o / down residual GEMM variants")
    ap.add_argument("--rope", action="store_true", help="also A/B the qkv GEMM with the RoPE/KV epilogue")
    ap.add_argument("--head", action="store_true", help="also A/B the LM head: hipBLASLt + argmax vs argmax epilogue")
    ap.add_argument("--groups", default="", help="e.g. 4,8,16: also time gemm_swiglu per block-order group size")
    ap.add_argument("--prio", action="store_true",
                    help="also time gemm_swiglu with s_setprio flips per MFMA cluster / a static priority on wave row 0 / none")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    d, ffn = 4096, 14336
    ops = HipOps()
    w_gu = (torch.randn(2 * ffn, d, device=dev) * 0.02).to(torch.bfloat16)
    w_perm = G.swiglu_permute(w_gu)

    # ---- numerics
    for T in (1, 37, 300, 4041):
        x = torch.randn(T, d, device=dev).to(torch.bfloat16)
        ref = G.swiglu_reference(x, w_gu).float()
        fused = G.gemm_swiglu(x, w_perm).float()
        unf = ops.silu_mul(F.linear(x, w_gu)).float()
        plain = G.gemm(x, w_gu).float()
        pref = (x.float() @ w_gu.float().t())
        scale = ref.abs().max().item()
        print(json.dumps({"check": "numerics", "T": T,
                          "fused_max_err": (fused - ref).abs().max().item(),
                          "unfused_max_err": (unf - ref).abs().max().item(),
                          "ref_absmax": scale,
                          "plain_max_err": (plain - pref).abs().max().item(),
                          "plain_ref_absmax": pref.abs().max().item()}), flush=True)

    # ---- swiglu timing
    for T in [int(t) for t in a.tokens.split(",")]:
        x = torch.randn(T, d, device=dev).to(torch.bfloat16)
        out = torch.empty(T, ffn, dtype=torch.bfloat16, device=dev)

        def unfused():
            ops.silu_mul(F.linear(x, w_gu), out=out)

        def fused():
            G.gemm_swiglu(x, w_perm, out=out)

        def blas_only():
            F.linear(x, w_gu)

        fns = {"hipblaslt+silu_mul": unfused, "fused": fused, "hipblaslt_gemm_only": blas_only}
        if a.prio:
            ref_out = G.gemm_swiglu(x, w_perm).clone()
            for name, code in (("fused_prio_flips", 48), ("fused_prio_row0", 64), ("fused_noprio", 80)):
                fns[name] = (lambda code=code: G._launch(x, w_perm, out, G.EPI_SWIGLU + code))
                fns[name]()
                print(json.dumps({"check": name, "T": T, "bit_equal": bool(torch.equal(out, ref_out))}), flush=True)
        for gm in [int(v) for v in a.groups.split(",") if v]:
            fns[f"fused_g{gm}"] = (lambda gm=gm: G._launch(x, w_perm, out, G.EPI_SWIGLU, group_m=gm))
        for f in fns.values():
            f()
        torch.cuda.synchronize()
        res = {k: [] for k in fns}
        for _ in range(a.rounds):
            for k, f in fns.items():
                res[k].append(timeit(f, a.iters))
        med = {k: statistics.median(v) for k, v in res.items()}
        flop = 2.0 * T * 2 * ffn * d
        print(json.dumps({"bench": "swiglu", "T": T, **{k + "_ms": round(v, 4) for k, v in med.items()},
                          "fused_tflops": round(flop / med["fused"] / 1e9, 1),
                          "blas_tflops": round(flop / med["hipblaslt_gemm_only"] / 1e9, 1),
                          "speedup_vs_unfused": round(med["hipblaslt+silu_mul"] / med["fused"], 3)}), flush=True)

    if a.rope:
        from llm_message_queue_amd.ops.llama_ops import rope_tables
        Hq, Hkv, max_ctx, S = 32, 8, 512, 1536
        wqkv = (torch.randn((Hq + 2 * Hkv) * 128, d, device=dev) * 0.02).to(torch.bfloat16)
        cos_t, sin_t = rope_tables(max_ctx, 500000.0, dev)
        kc1 = torch.zeros(S, Hkv, max_ctx, 128, dtype=torch.bfloat16, device=dev)
        vc1, kc2, vc2 = torch.zeros_like(kc1), torch.zeros_like(kc1), torch.zeros_like(kc1)
        for T in (37, 1024, 2600, 4041):
            x = torch.randn(T, d, device=dev).to(torch.bfloat16)
            cell = torch.randperm(S * 64, device=dev)[:T]               # unique (slot, pos)
            slot = (cell // 64).to(torch.int32)
            pos = (cell % 64 * 7 % max_ctx).to(torch.int32)
            q1 = ops.rope_kv(F.linear(x, wqkv), pos, slot, cos_t, sin_t, Hq, Hkv, kc1, vc1)
            q2 = G.qkv_rope(x, wqkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2)
            sl, ps = slot.long(), pos.long()
            print(json.dumps({"check": "qkv_rope", "T": T, "q_max_diff": (q1.float() - q2.float()).abs().max().item(),
                              "q_absmax": q1.float().abs().max().item(),
                              "k_max_diff": (kc1[sl, :, ps].float() - kc2[sl, :, ps].float()).abs().max().item(),
                              "v_max_diff": (vc1[sl, :, ps].float() - vc2[sl, :, ps].float()).abs().max().item()}),
                  flush=True)
            fns = {"hipblaslt+rope_kv": lambda: ops.rope_kv(F.linear(x, wqkv), pos, slot, cos_t, sin_t, Hq, Hkv, kc1, vc1),
                   "fused": lambda: G.qkv_rope(x, wqkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2),
                   "fused_g4": lambda: G.qkv_rope(x, wqkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2, group_m=4),
                   "fused_g16": lambda: G.qkv_rope(x, wqkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2, group_m=16),
                   "fused_nosplit": lambda: G.qkv_rope(x, wqkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2,
                                                       split=False)}
            if T <= 1024:   # split every tile: the cost of a K-half + the handoff vs a whole tile
                fns["fused_allsplit"] = lambda: G.qkv_rope(x, wqkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2,
                                                           split_full=0)
            res = {k: [] for k in fns}
            for _ in range(a.rounds):
                for k, f in fns.items():
                    res[k].append(timeit(f, a.iters))
            med = {k: statistics.median(v) for k, v in res.items()}
            print(json.dumps({"bench": "qkv_rope", "T": T, **{k + "_ms": round(v, 4) for k, v in med.items()},
                              "speedup": round(med["hipblaslt+rope_kv"] / med["fused"], 3)}), flush=True)

    if a.head:
        V = 128256
        wh = (torch.randn(V, d, device=dev) * 0.02).to(torch.bfloat16)
        for M in (256, 512, 900, 1200, 1536):
            x = torch.randn(M, d, device=dev).to(torch.bfloat16)
            fns = {"hipblaslt+argmax": lambda: torch.argmax(F.linear(x, wh), dim=-1),
                   "fused": lambda: G.lm_head_argmax(x, wh)}
            agree = (fns["hipblaslt+argmax"]().int() == fns["fused"]()).float().mean().item()
            res = {k: [] for k in fns}
            for _ in range(a.rounds):
                for k, f in fns.items():
                    res[k].append(timeit(f, a.iters))
            med = {k: statistics.median(v) for k, v in res.items()}
            print(json.dumps({"bench": "lm_head", "M": M, **{k + "_ms": round(v, 4) for k, v in med.items()},
                              "speedup": round(med["hipblaslt+argmax"] / med["fused"], 3),
                              "tflops_fused": round(2 * M * V * d / med["fused"] / 1e9, 1),
                              "token_agreement": round(agree, 4)}), flush=True)

    if a.resid:
        # o / down into the residual stream: hipBLASLt beta = 1 vs the
        # hand-written residual epilogue
        shapes = {"o": (d, d), "down": (d, ffn)}
        for name, (N, K) in shapes.items():
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            for T in (4041, 4096):
                x = torch.randn(T, K, device=dev).to(torch.bfloat16)
                y = torch.randn(T, N, device=dev).to(torch.bfloat16)
                fns = {"hipblaslt_resid": lambda: y.addmm_(x, w.t()),
                       "hip_resid": lambda: G.gemm_residual(x, w, y),
                       "hip_resid_lds": lambda: G._launch(x, w, y, G.EPI_RESID_LDS),
                       "hip_resid_pre": lambda: G._launch(x, w, y, G.EPI_RESID_PRE),
                       "hip_plain": lambda: G.gemm(x, w, out=y)}
                for f in fns.values():
                    f()
                res = {k: [] for k in fns}
                for _ in range(a.rounds):
                    for k, f in fns.items():
                        res[k].append(timeit(f, a.iters))
                med = {k: statistics.median(v) for k, v in res.items()}
                flop = 2.0 * T * N * K
                print(json.dumps({"bench": "resid", "gemm": name, "T": T,
                                  **{k + "_ms": round(v, 4) for k, v in med.items()},
                                  **{k + "_tflops": round(flop / v / 1e9, 1) for k, v in med.items()}}), flush=True)

    if a.plain:
        shapes = {"qkv": (6144, d), "o": (d, d), "gate_up": (2 * ffn, d), "down": (d, ffn)}
        for name, (N, K) in shapes.items():
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            for T in (4041, 4096):
                x = torch.randn(T, K, device=dev).to(torch.bfloat16)
                y = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
                fns = {"hipblaslt": lambda: torch.mm(x, w.t(), out=y), "hip": lambda: G.gemm(x, w, out=y),
                       "hipblaslt_resid": lambda: y.addmm_(x, w.t()),
                       "hip_resid": lambda: G.gemm_residual(x, w, y),
                       "hip_r1sched": lambda: G._launch(x, w, y, G.EPI_STORE + 16),
                       "hip_nostagger": lambda: G._launch(x, w, y, G.EPI_STORE + 32)}
                for f in fns.values():
                    f()
                res = {k: [] for k in fns}
                for _ in range(a.rounds):
                    for k, f in fns.items():
                        res[k].append(timeit(f, a.iters))
                med = {k: statistics.median(v) for k, v in res.items()}
                flop = 2.0 * T * N * K
                print(json.dumps({"bench": "plain", "gemm": name, "T": T,
                                  **{k + "_ms": round(v, 4) for k, v in med.items()},
                                  **{k + "_tflops": round(flop / v / 1e9, 1) for k, v in med.items()}}), flush=True)


if __name__ == "__main__":
    main()
