"""One full serving-engine step at the bench's Llama-3-8B dimensions (d 4096,
GQA 32/8, FFN 14336, vocab 128256; 2 of the 32 layers) through the HIP path
(hand-written kernels + residual-in-GEMM), against the same engine on the
plain-PyTorch fp32 reference ops: a prefill step (chunked
prompts of several slots, one spilling into the next step) and the decode
step after it, compared on the step's final hidden states and the sampled
rows' logits."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _engine(impl):
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    cfg = LlamaConfig(layers=2)                       # 8B dims, 2 layers
    eng = BackendEngine(cfg, slots=16, max_ctx=128, token_budget=96, device="cuda:0", impl=impl, seed=11,
                        residual_in_gemm=(impl == "hip"), prune_last=False)   # every row's hidden state
    # (last-layer row pruning has its own test: tests/test_prune_last.py)
    cap = []
    orig = eng.model.hidden

    def hidden(*a, **k):
        h = orig(*a, **k)
        cap.append(h.float().clone())
        return h
    eng.model.hidden = hidden
    return eng, cap


def test_8b_dims_engine_step_hip_vs_ref():
    from llm_message_queue_amd.backend.engine import Request
    rng = np.random.default_rng(3)
    prompts = [rng.integers(0, 128256, n).astype(np.int32) for n in (5, 17, 33, 40, 9)]   # 104 > 96: a chunk spills
    hip, cap_h = _engine("hip")
    ref, cap_r = _engine("ref")
    for eng in (hip, ref):
        eng.admit([Request(i, p.copy(), 3) for i, p in enumerate(prompts)])
    for step in range(4):                            # prefill (+ spill), then decodes
        hip.launch()
        hip.finish(block=True)
        ref.launch()
        ref.finish(block=True)
        # decode rows read the previous step's greedy tokens: feed both
        # engines the same ones so every step compares like with like
        ref._prev_out = hip._prev_out.clone()
        a, b = cap_h[step], cap_r[step]
        assert a.shape == b.shape
        err = ((a - b).abs().max() / b.abs().max()).item()
        assert err < 5e-2, (step, err)
        la = torch.nn.functional.linear(a.to(torch.bfloat16), hip.model.lm_head).float()
        lb = torch.nn.functional.linear(b.to(torch.bfloat16), ref.model.lm_head).float()
        scale = lb.abs().max().item()
        assert (la - lb).abs().max().item() / scale < 5e-2, step
        top2 = lb.topk(2, dim=-1).values
        decided = (top2[:, 0] - top2[:, 1]) > 0.1 * scale
        assert bool((la.argmax(-1) == lb.argmax(-1))[decided].all()), step
    assert not hip.active and not ref.active          # 3 tokens each: every request done after step 4
