import sys, os, json, statistics
sys.path.insert(0, os.getcwd())
import torch
from llm_message_queue_amd.ops import gemm as G
def timeit(fn, iters=10):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters): fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / iters
T, N = 4096, 28672
for K in (1024, 2048, 4096, 8192):
    x = torch.randn(T, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    wp = G.swiglu_permute(w)
    out = torch.empty(T, N // 2, dtype=torch.bfloat16, device="cuda")
    f = lambda: G.gemm_swiglu(x, wp, out=out)
    f(); torch.cuda.synchronize()
    ms = statistics.median([timeit(f) for _ in range(7)])
    print(json.dumps({"K": K, "ms": round(ms, 4), "tflops": round(2 * T * N * K / ms / 1e9, 1)}), flush=True)
