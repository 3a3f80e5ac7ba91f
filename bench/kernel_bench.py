"""Run each hand-written HIP kernel in isolation at serving-representative
sizes (for rocprofv3 counter collection and per-kernel timing).

    python bench/kernel_bench.py [--reps 50]
    rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_LDS_BANK_CONFLICT ... --kernel-trace --stats \\
        -d out -o k --output-format csv -- python3 bench/kernel_bench.py

Prints per-kernel mean time (CUDA events) and an achieved-throughput figure.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--only", default="")
    ap.add_argument("--lib-dir", default="", help="A/B: load the native modules from this directory instead of _lib")
    ap.add_argument("--text-batches", default="4096", help="preprocess batch sizes (messages), comma-separated")
    ap.add_argument("--summ-convs", default="64", help="summarise: conversations per batch (8 evicted turns each)")
    a = ap.parse_args()
    import numpy as np
    import torch
    if a.lib_dir:
        from llm_message_queue_amd import _native
        _native._LIB = os.path.abspath(a.lib_dir)

    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.ops.llama_ops import HipOps, make_tiles, rope_tables
    from llm_message_queue_amd.ops.text import TextPipeline
    from llm_message_queue_amd.preprocess.oracle import default_patterns

    dev = torch.device("cuda", 0)
    out = []
    want = set(a.only.split(",")) if a.only else None

    def rec(name, ms, **kw):
        d = {"kernel": name, "ms": round(ms, 4), **kw}
        out.append(d)
        print(json.dumps(d), flush=True)

    # --- preprocess pipeline (text_analyze + scan + MFMA embed_pool + head), 4096 messages
    if not want or "text" in want:
        pipe = TextPipeline(device="cuda:0")
        pats = default_patterns()
        for nb in (int(x) for x in a.text_batches.split(",")):
            msgs = [m.content for m in Workload(seed=1).make(nb)]
            ms = timeit(lambda: pipe.run(msgs, pats, 0, classify=True, prompt_cap=32), max(5, a.reps // 5))
            rec(f"preprocess_pipeline_{nb}msgs", ms, us_per_msg=round(ms * 1e3 / nb, 3))

    ops = HipOps()
    Hq, Hkv, S, C = 32, 8, 1024, 512
    # --- attention over a serving-like step: 768 decode tokens + 256 prefill chunks of 12
    if not want or "attention" in want:
        kc = (torch.randn(S, Hkv, C, 128, device=dev) * 0.5).to(torch.bfloat16)
        vc = torch.randn(S, Hkv, C, 128, device=dev).to(torch.bfloat16)
        rng = np.random.default_rng(0)
        starts, lens, slots, pos0 = [], [], [], []
        row = 0
        for i in range(768):                            # decode tokens, context 12..40
            starts.append(row); lens.append(1); slots.append(i); pos0.append(int(rng.integers(12, 40)))
            row += 1
        for i in range(256):                            # fresh prefill chunks
            n = int(rng.integers(4, 33))
            starts.append(row); lens.append(n); slots.append(768 + i); pos0.append(0)
            row += n
        T = row
        tiles = torch.from_numpy(make_tiles(starts, lens, slots, pos0)).to(dev)
        q = torch.randn(T, Hq * 128, device=dev).to(torch.bfloat16)
        o = torch.empty_like(q)
        for sk in (32, 64):
            ms = timeit(lambda: ops.attention_tiles(q, kc, vc, tiles, Hq, Hkv, 128 ** -0.5, out=o, n_dec=768,
                                                    seg_keys=sk), a.reps)
            rec(f"attention_tiles_step_seg{sk}", ms, tokens=T, decode=768)
            ms = timeit(lambda: ops.attention_tiles(q, kc, vc, tiles, Hq, Hkv, 128 ** -0.5, out=o, n_dec=768,
                                                    seg_keys=sk, mixed=False), a.reps)
            rec(f"attention_tiles_step_seg{sk}_two_launches", ms, tokens=T, decode=768)
            seg = tiles[768:].contiguous()
            ms = timeit(lambda: ops.attention_tiles(q, kc, vc, seg, Hq, Hkv, 128 ** -0.5, out=o, n_dec=0,
                                                    seg_keys=sk), a.reps)
            rec(f"attention_seg_only_keys{sk}", ms, tiles=int(seg.shape[0]))
        # long dialog contexts: 256 chunks of 4..32 new tokens at positions 100..460
        starts2, lens2, slots2, pos2 = [], [], [], []
        row2 = 0
        for i in range(256):
            n = int(rng.integers(4, 33))
            starts2.append(row2); lens2.append(n); slots2.append(i); pos2.append(int(rng.integers(100, 460)))
            row2 += n
        tiles2 = torch.from_numpy(make_tiles(starts2, lens2, slots2, pos2)).to(dev)
        q2 = torch.randn(row2, Hq * 128, device=dev).to(torch.bfloat16)
        o2 = torch.empty_like(q2)
        for sk in (32, 64):
            ms = timeit(lambda: ops.attention_tiles(q2, kc, vc, tiles2, Hq, Hkv, 128 ** -0.5, out=o2, n_dec=0,
                                                    seg_keys=sk), a.reps)
            rec(f"attention_seg_long_ctx_keys{sk}", ms, tiles=int(tiles2.shape[0]), tokens=row2)
        dec = tiles[:768].contiguous()
        ms = timeit(lambda: ops.attention_tiles(q, kc, vc, dec, Hq, Hkv, 128 ** -0.5, out=o, n_dec=768), a.reps)
        rec("attention_dec_only", ms, tokens=768)
        pos = torch.tensor(sum([list(range(p, p + n)) for p, n in zip(pos0, lens)], []), dtype=torch.int32,
                           device=dev)
        slot = torch.tensor(sum([[s] * n for s, n in zip(slots, lens)], []), dtype=torch.int32, device=dev)
        ms = timeit(lambda: ops.attention(q, kc, vc, pos, slot, Hq, Hkv, 128 ** -0.5, out=o), a.reps)
        rec("attention_per_token_step", ms, tokens=T)

    # --- elementwise: rmsnorm (fused residual), silu_mul, rope_kv at T = 4096
    if not want or "elementwise" in want:
        T, D, F = 4096, 4096, 14336
        x = torch.randn(T, D, device=dev).to(torch.bfloat16)
        res = torch.randn(T, D, device=dev).to(torch.bfloat16)
        w = torch.ones(D, device=dev, dtype=torch.bfloat16)
        y = torch.empty_like(x)
        ms = timeit(lambda: ops.rmsnorm(x, w, 1e-5, residual=res, out=y), a.reps)
        rec("rmsnorm_residual_T4096", ms, GBps=round(4 * T * D * 2 / ms / 1e6, 1))
        gu = torch.randn(T, 2 * F, device=dev).to(torch.bfloat16)
        act = torch.empty(T, F, device=dev, dtype=torch.bfloat16)
        ms = timeit(lambda: ops.silu_mul(gu, out=act), a.reps)
        rec("silu_mul_T4096", ms, GBps=round(3 * T * F * 2 / ms / 1e6, 1))
        cos, sin = rope_tables(C, device=dev)
        qkv = torch.randn(T, (Hq + 2 * Hkv) * 128, device=dev).to(torch.bfloat16)
        kc2 = torch.zeros(S, Hkv, C, 128, device=dev, dtype=torch.bfloat16)
        vc2 = torch.zeros_like(kc2)
        p = torch.randint(0, C, (T,), dtype=torch.int32, device=dev)
        sl = torch.randint(0, S, (T,), dtype=torch.int32, device=dev)
        ms = timeit(lambda: ops.rope_kv(qkv, p, sl, cos, sin, Hq, Hkv, kc2, vc2), a.reps)
        rec("rope_kv_T4096", ms, GBps=round(T * (Hq + 2 * Hkv) * 128 * 2 * 2 / ms / 1e6, 1))
    # --- conversation summarise-on-evict (N5): the text pipeline's pooled
    # embeddings -> summarise_project (segmented mean + MFMA projection +
    # running-summary blend) and the salient-token top-k, per batch of
    # conversations evicting 8 turns each
    if not want or "summarise" in want:
        from llm_message_queue_amd.conversation.summarise import SummaryEngine
        from llm_message_queue_amd.utils.config import default_config
        eng = SummaryEngine(default_config().preprocessor, device="cuda", k=8, alpha=0.8, dim=256)
        turns = [m.content for m in Workload(seed=3).make(8 * 512)]
        for nc in (int(x) for x in a.summ_convs.split(",")):
            groups = [(None if c % 2 else np.full(256, 0.1, dtype=np.float32), turns[8 * c:8 * c + 8])
                      for c in range(nc)]
            ms = timeit(lambda: eng.summarise(groups), max(5, a.reps // 5))
            rec(f"summarise_{nc}convs", ms, us_per_conv=round(ms * 1e3 / nc, 2), turns=8 * nc)
    print(json.dumps({"summary": out}))


if __name__ == "__main__":
    main()
