"""Decode-attention precision probe: the decode kernel's q.k scores use
v_dot2_f32_bf16; compare its error against the fp32 reference with that of
the MFMA prefill-tile path on the same rows (round-3 check after the dot2
accumulator was found lossy in a GEMM experiment)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from llm_message_queue_amd.ops.llama_ops import HipOps, RefOps, make_tiles

hip, ref = HipOps(), RefOps()
dev = "cuda"
torch.manual_seed(3)
Hq, Hkv, S, C = 32, 8, 64, 512
kc = (torch.randn(S, Hkv, C, 128, device=dev) * 1.0).to(torch.bfloat16)
vc = torch.randn(S, Hkv, C, 128, device=dev).to(torch.bfloat16)
for ctx in (8, 32, 128, 511):
    n = S
    segs = [(s, ctx, 1) for s in range(n)]
    tiles = make_tiles(list(range(n)), [1] * n, list(range(n)), [ctx] * n)
    q = (torch.randn(n, Hq * 128, device=dev) * 1.0).to(torch.bfloat16)
    t = torch.from_numpy(tiles).to(dev)
    o_ref = ref.attention_tiles(q, kc, vc, torch.from_numpy(tiles), Hq, Hkv, 128 ** -0.5).float()
    o_dec = hip.attention_tiles(q, kc, vc, t, Hq, Hkv, 128 ** -0.5, n_dec=n).float()
    o_mfma = hip.attention_tiles(q, kc, vc, t, Hq, Hkv, 128 ** -0.5, n_dec=0).float()
    e_dec = (o_dec - o_ref).abs()
    e_mfma = (o_mfma - o_ref).abs()
    print(json.dumps({"ctx": ctx + 1, "ref_absmax": round(o_ref.abs().max().item(), 4),
                      "decode_err_max": round(e_dec.max().item(), 5), "decode_err_mean": round(e_dec.mean().item(), 6),
                      "mfma_err_max": round(e_mfma.max().item(), 5), "mfma_err_mean": round(e_mfma.mean().item(), 6)}))
