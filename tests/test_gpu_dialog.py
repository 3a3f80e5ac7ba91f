"""Semantics-exact dialog context on the HIP engine:
one conversation's next turn computes the same logits whether its context is

* the resident KV (the turn admitted into the slot that parked the dialog),
* a KV moved from another engine by the ``kv_move`` pack / unpack kernels, or
* a full replay of the dialog's real token ids (prompt + generated ids read
  back with ``Request.out_tokens``) on an engine that never saw it.

The logits are the fp32 products of the hidden rows the LM head sees and the
head weight.  Resident vs migrated: the same KV bytes, so identical.
Replay: the history is prefilled in one chunk instead of turn by turn, so
the KV entries can differ by bf16 roundings; the logits agree to bf16
tolerance and the greedy ids match."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = torch.device("cuda", 0)


def _engine(seed=11):
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    cfg = LlamaConfig(vocab=4096, dim=2048, layers=4, heads=16, kv_heads=4, ffn=4096)
    return BackendEngine(cfg, slots=8, max_ctx=128, token_budget=64, device=DEV, impl="hip", seed=seed)


def _serve(eng, req, heads):
    """Run ``req`` alone; ``heads`` collects the hidden rows the LM head saw."""
    orig = eng.model.ops.greedy_head

    def spy(x, w, fused=True, min_rows=256):
        heads.append(x.float().clone())
        return orig(x, w, fused, min_rows)
    eng.model.ops.greedy_head = spy
    try:
        eng.admit([req])
        while eng.active:
            eng.launch()
            eng.finish(block=True)
        torch.cuda.synchronize()
    finally:
        eng.model.ops.greedy_head = orig
    return req


def test_resident_migrated_and_replayed_turns_agree():
    from llm_message_queue_amd.backend.engine import Request
    from llm_message_queue_amd.parallel.comm import SoloComm
    from llm_message_queue_amd.parallel.migration import KVMigrator
    conv = 31337
    p1 = (np.arange(21) * 37 % 4000).astype(np.int32)
    p2 = (np.arange(9) * 11 % 4000 + 50).astype(np.int32)
    gen = 5
    # resident: both turns on one engine
    a = _engine()
    h = []
    t1 = _serve(a, Request(1, p1.copy(), gen, conv=conv), h)
    h_res = []
    r_res = _serve(a, Request(2, p2.copy(), gen, conv=conv), h_res)
    assert r_res.reused == len(p1) + gen - 1
    # migrated: turn 1 on b, its KV moved into c by kv_move, turn 2 on c
    b, c = _engine(), _engine()
    _serve(b, Request(1, p1.copy(), gen, conv=conv), [])
    slot_b, n = b.export_kv(conv)
    buf = KVMigrator(b.model, SoloComm()).pack(slot_b, n)
    slot_c = c.import_kv(conv, n)
    KVMigrator(c.model, SoloComm()).unpack(buf, slot_c)
    torch.cuda.synchronize()
    h_mig = []
    r_mig = _serve(c, Request(2, p2.copy(), gen, conv=conv), h_mig)
    assert r_mig.reused == n
    # replayed: the dialog's real ids (prompt + generated but the last) on a fresh engine
    hist = np.concatenate([p1, t1.out_tokens[:-1]]).astype(np.int32)
    assert len(hist) == n and np.any(t1.out_tokens != 0)
    d = _engine()
    h_rep = []
    r_rep = _serve(d, Request(2, p2.copy(), gen, conv=conv, history=hist), h_rep)
    assert r_rep.reused == 0 and len(r_rep.prompt) == len(hist) + len(p2)
    W = a.model.lm_head.float()
    logits = [torch.cat(x) @ W.t() for x in (h_res, h_mig, h_rep)]
    assert torch.equal(logits[0], logits[1]), "migrated KV differs from the resident KV"
    tol = 0.03 * logits[0].abs().max().item()
    assert (logits[2] - logits[0]).abs().max().item() <= tol
    assert r_res.out_tokens.tolist() == r_mig.out_tokens.tolist() == r_rep.out_tokens.tolist()
