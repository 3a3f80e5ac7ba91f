"""Minimal driver for rocprofv3 --pmc passes over the serving step's GEMM
roles at T tokens (default 4096): qkv (the fused RoPE/KV-write kernel and
hipBLASLt), o and down (hipBLASLt ``addmm_`` beta = 1, what the model runs,
and the hand-written residual epilogue), gate/up (the fused SwiGLU kernel).
Each role runs 10 calls; the kernels are told apart in the counter CSV by
name and grid size (scripts/pmc_summary.py --by-grid)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_message_queue_amd.ops import gemm as G

T = int(os.environ.get("GEMM_T", "4096"))
ROLES = os.environ.get("GEMM_ROLES", "qkv,o,down,gate_up").split(",")
dev = torch.device("cuda")
D, F, HQ, HKV, CTX, SLOTS = 4096, 14336, 32, 8, 512, 64


def rnd(*shape, s=1.0):
    return (torch.rand(*shape, device=dev) * 2 - 1).mul_(s).to(torch.bfloat16)


x = rnd(T, D)
for role in ROLES:
    if role == "qkv":
        w = rnd((HQ + 2 * HKV) * 128, D, s=0.02)
        pos = (torch.arange(T, device=dev, dtype=torch.int32) % CTX).contiguous()
        slot = (torch.arange(T, device=dev, dtype=torch.int32) // CTX % SLOTS).contiguous()
        ang = torch.arange(CTX, device=dev).float()[:, None] * torch.arange(64, device=dev).float()[None] * 1e-3
        cos_t, sin_t = ang.cos().contiguous(), ang.sin().contiguous()
        kc = torch.zeros(SLOTS, HKV, CTX, 128, dtype=torch.bfloat16, device=dev)
        vc = torch.zeros_like(kc)
        for _ in range(10):
            G.qkv_rope(x, w, pos, slot, cos_t, sin_t, HQ, HKV, kc, vc)
            torch.nn.functional.linear(x, w)
    elif role in ("o", "down"):
        K = D if role == "o" else F
        a = x if role == "o" else rnd(T, F)
        w = rnd(D, K, s=0.02)
        res = rnd(T, D)
        for _ in range(10):
            res.addmm_(a, w.t())                         # hipBLASLt beta = 1 (the model's default)
            G.gemm_residual(a, w, res)                   # hand-written residual epilogue
    elif role == "gate_up":
        w = rnd(2 * F, D, s=0.02)
        h = torch.empty(T, F, dtype=torch.bfloat16, device=dev)
        for _ in range(10):
            G.gemm_swiglu(x, w, out=h)
            torch.mm(x, w.t())
    torch.cuda.synchronize()
print("ok")
