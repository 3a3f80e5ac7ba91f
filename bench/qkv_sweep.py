"""Where the qkv projection's time goes at the serving shape (N = 6144,
K = 4096): the fused RoPE/KV kernel with and without the split-K tail, the
same tiles with the plain store epilogue, hipBLASLt ``F.linear``, and the
gate/up SwiGLU kernel at the same T as the throughput reference.  One JSON
line per T: median kernel ms over ``--iters`` CUDA-event-timed calls and the
achieved TFLOP/s."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_message_queue_amd.ops import gemm as G

D, F, HQ, HKV, CTX, SLOTS = 4096, 14336, 32, 8, 512, 64


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
    ap.add_argument("--tokens", default="3840,4041,4096,4226,4352")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--lib-dir", default="", help="A/B: load the native modules from this directory instead of _lib")
    a = ap.parse_args()
    if a.lib_dir:
        from llm_message_queue_amd import _native
        _native._LIB = os.path.abspath(a.lib_dir)
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N = (HQ + 2 * HKV) * 128
    w = ((torch.rand(N, D, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16)
    wgu = ((torch.rand(2 * F, D, device=dev) * 2 - 1) * 0.02).to(torch.bfloat16)
    ang = torch.arange(CTX, device=dev).float()[:, None] * torch.arange(64, device=dev).float()[None] * 1e-3
    cos_t, sin_t = ang.cos().contiguous(), ang.sin().contiguous()
    kc = torch.zeros(SLOTS, HKV, CTX, 128, dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    cus = G._cu_count(dev)
    for T in [int(t) for t in a.tokens.split(",")]:
        x = ((torch.rand(T, D, device=dev) * 2 - 1)).to(torch.bfloat16)
        pos = (torch.arange(T, device=dev, dtype=torch.int32) % CTX).contiguous()
        slot = (torch.arange(T, device=dev, dtype=torch.int32) // CTX % SLOTS).contiguous()
        q = torch.empty(T, HQ * 128, dtype=torch.bfloat16, device=dev)
        out = torch.empty(T, N, dtype=torch.bfloat16, device=dev)
        h = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
        r = {"T": T, "tiles": -(-T // 256) * (N // 256), "cus": cus, "split_full": G.split_plan(T, N, D, cus)}
        r["qkv_rope_split_ms"] = timed(lambda: G.qkv_rope(x, w, pos, slot, cos_t, sin_t, HQ, HKV, kc, vc, q_out=q), a.iters)
        r["qkv_rope_nosplit_ms"] = timed(
            lambda: G.qkv_rope(x, w, pos, slot, cos_t, sin_t, HQ, HKV, kc, vc, q_out=q, split=False), a.iters)
        r["store_ms"] = timed(lambda: G.gemm(x, w, out=out), a.iters)
        r["hipblaslt_ms"] = timed(lambda: torch.nn.functional.linear(x, w), a.iters)
        r["gate_up_ms"] = timed(lambda: G.gemm_swiglu(x, wgu, out=h), a.iters)
        fl = 2.0 * T * D * N
        for k in ("qkv_rope_split_ms", "qkv_rope_nosplit_ms", "store_ms", "hipblaslt_ms"):
            r[k.replace("_ms", "_tflops")] = round(fl / r[k] / 1e9, 1)
        r["gate_up_tflops"] = round(2.0 * T * D * 2 * F / r["gate_up_ms"] / 1e9, 1)
        for k in list(r):
            if k.endswith("_ms"):
                r[k] = round(r[k], 4)
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
