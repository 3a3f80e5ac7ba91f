"""Last-layer row pruning (models/llama_stub.py ``hidden(rows=...)``): the
last layer's o projection and MLP run only for the step's sampled rows.  The
sampled rows' final hidden states and greedy tokens must equal the unpruned
forward's, and every token's K/V must still be written."""
import pytest
import torch

from llm_message_queue_amd.models.llama_stub import LlamaConfig, LlamaStub


def _step(model, T, slots):
    g = torch.Generator().manual_seed(1)
    tokens = torch.randint(0, model.cfg.vocab, (T,), generator=g)
    slot = (torch.arange(T) // 8 % slots).to(torch.int32)
    pos = (torch.arange(T) % 8).to(torch.int32)
    return tokens, pos, slot


@pytest.mark.parametrize("sampled", [[7, 15, 23], [0, 5, 9, 31], list(range(32)), []])   # []: only unfinished prefill chunks
def test_pruned_rows_match_full_forward(sampled):
    cfg = LlamaConfig(vocab=512, dim=256, layers=2, heads=2, kv_heads=1, ffn=512)
    full = LlamaStub(cfg, slots=4, max_ctx=16, device="cpu", impl="ref", prune_last=False)
    pruned = LlamaStub(cfg, slots=4, max_ctx=16, device="cpu", impl="ref", prune_last=True)
    tokens, pos, slot = _step(full, 32, 4)
    idx = torch.tensor(sampled, dtype=torch.long)
    h_full = full.hidden(tokens, pos, slot).index_select(0, idx)
    h_pruned = pruned.hidden(tokens, pos, slot, rows=idx)
    assert h_pruned.shape == (len(sampled), cfg.dim)
    torch.testing.assert_close(h_pruned, h_full, rtol=2e-2, atol=2e-2)
    assert torch.equal(full.forward(tokens, pos, slot, idx), pruned.forward(tokens, pos, slot, idx))
    # K/V of every token of every layer written the same way
    for i in range(cfg.layers):
        assert torch.equal(full.kcache[i], pruned.kcache[i])
        assert torch.equal(full.vcache[i], pruned.vcache[i])


@pytest.mark.gpu
@pytest.mark.parametrize("T,n_samp", [(600, 90), (2100, 700), (4041, 900), (300, 0)])
def test_pruned_rows_match_full_forward_hip(T, n_samp):
    """The HIP model (fused qkv / SwiGLU GEMMs, hipBLASLt residual GEMMs):
    full-row layers at T tokens, the pruned last layer at the sampled-row
    count, which takes other GEMM paths (e.g. SwiGLU fused at 700 rows,
    hipBLASLt + silu_mul at 90)."""
    dev = torch.device("cuda", 0)
    cfg = LlamaConfig(vocab=4096, dim=4096, layers=2, heads=32, kv_heads=8, ffn=14336)
    full = LlamaStub(cfg, slots=64, max_ctx=128, device=dev, impl="hip", prune_last=False)
    pruned = LlamaStub(cfg, slots=64, max_ctx=128, device=dev, impl="hip", prune_last=True)
    g = torch.Generator(device=dev).manual_seed(3)
    tokens = torch.randint(0, cfg.vocab, (T,), generator=g, device=dev)
    r = torch.arange(T, device=dev, dtype=torch.int32)
    slot = (r // 64 % 64).contiguous()
    pos = (r % 64).contiguous()
    idx = torch.randperm(T, generator=g, device=dev)[:n_samp].sort().values
    if n_samp == 0:                                  # a step of unfinished prefill chunks
        assert pruned.forward(tokens, pos, slot, idx).numel() == 0
        full.hidden(tokens, pos, slot)
        for i in range(cfg.layers):
            assert torch.equal(full.kcache[i], pruned.kcache[i])
        return
    h_full = full.hidden(tokens, pos, slot).index_select(0, idx).float()
    h_pruned = pruned.hidden(tokens, pos, slot, rows=idx).float()
    err = (h_pruned - h_full).abs().max().item()
    assert err <= 0.05 * h_full.abs().max().item(), err
    t_full = full.forward(tokens, pos, slot, idx)
    t_pruned = pruned.forward(tokens, pos, slot, idx)
    # bf16 GEMMs of different row counts take different kernels and round
    # differently, so near-ties of the random-weight logits can flip (88 / 90
    # equal at T = 600 on the box); every pruned token must be a near-argmax
    # of the unpruned hidden state's fp32 logits
    assert (t_full == t_pruned).float().mean().item() >= 0.9
    logits = h_full @ pruned.lm_head.float().t()
    top = logits.max(dim=1).values
    picked = logits.gather(1, t_pruned.long()[:, None])[:, 0]
    spread = (top - logits.mean(dim=1)).mean().item()
    assert ((top - picked) <= 0.05 * spread).all(), (top - picked).max().item()
    for i in range(cfg.layers):
        assert torch.equal(full.kcache[i], pruned.kcache[i])
