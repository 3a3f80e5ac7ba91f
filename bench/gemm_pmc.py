"""Minimal driver for rocprofv3 --pmc passes over the hand-written GEMM:
gate_up shape (T x 28672 x 4096), plain-store and SwiGLU epilogues and hipBLASLt (torch.mm), 10 calls each."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_message_queue_amd.ops import gemm as G

T = int(os.environ.get("GEMM_T", "4096"))
x = torch.randn(T, 4096, device="cuda").to(torch.bfloat16)
w = (torch.randn(28672, 4096, device="cuda") * 0.02).to(torch.bfloat16)
y = torch.empty(T, 28672, dtype=torch.bfloat16, device="cuda")
h = torch.empty(T, 14336, dtype=torch.bfloat16, device="cuda")
for _ in range(10):
    G.gemm(x, w, out=y)
    G.gemm_swiglu(x, w, out=h)
    torch.mm(x, w.t(), out=y)                   # hipBLASLt, for comparison
torch.cuda.synchronize()
print("ok")
