"""Semantics-exact dialog context (VERDICT r5 missing #2, weak #4 / #5).

* The origin router's dialog history holds the REAL token ids: each turn's
  prompt as the engine took it and its generated ids (read back per step,
  ``Request.out_tokens``; carried home in the K_DONE record when another GPU
  ran the turn) -- exactly the positions the home GPU's parked KV holds.
* A turn replayed on another rank receives that history (K_HIST rows one
  exchange after its descriptor) instead of placeholder zeros, so the replay
  computes the same next turn as the resident KV.
* When a conversation's window was evicted, the N5 salient tokens are
  prepended to a replay as its compressed context (N5's output is consumed).

Reference: the context is real content -- `internal/statemanager/manager.go:133-135`
(completed content concatenated into Context), `internal/conversation/state_manager.go:290-306`
(the real last-N messages).  CPU engines on the fp32 reference ops; FakeComm
ranks in threads.  The GPU variant (resident / kv_move-migrated / replayed
logits) is in tests/test_gpu_dialog.py."""
import threading

import numpy as np
import pytest

from llm_message_queue_amd.backend.engine import BackendEngine, Request
from llm_message_queue_amd.gateway.router import Gateway, conv_key
from llm_message_queue_amd.models.llama_stub import LlamaConfig
from llm_message_queue_amd.models.message import Message, MessageStatus
from llm_message_queue_amd.parallel.comm import FakeComm
from llm_message_queue_amd.utils.config import default_config

MICRO = LlamaConfig(vocab=512, dim=2048, layers=2, heads=16, kv_heads=4, ffn=256)


def _eng(seed=7, slots=4):
    return BackendEngine(MICRO, slots=slots, max_ctx=64, token_budget=64, device="cpu", impl="ref", seed=seed)


def _cfg(strategy="least_connections"):
    c = default_config()
    c.queue.enable_metrics = False
    c.loadbalancer.algorithm = strategy
    return c


def _tick_all(gws):
    if len(gws) == 1:
        gws[0].tick()
        return
    ths = [threading.Thread(target=g.tick) for g in gws]
    for t in ths:
        t.start()
    for t in ths:
        t.join()


def _record_outputs(eng, sink):
    """Wrap ``eng.finish`` so every completed request's ids land in ``sink``."""
    orig = eng.finish

    def finish(block=False):
        res = orig(block)
        for r in res.completed:
            sink.append((r.meta, None if r.out_tokens is None else r.out_tokens.tolist(), np.asarray(r.prompt)))
        return res
    eng.finish = finish


def _serve(eng, req):
    eng.admit([req])
    while eng.active:
        eng.launch()
        eng.finish(block=True)
    return req


def _turn(i, cid="dlg"):
    return Message(id=f"t{i}", conversation_id=cid, user_id="u",
                   content=["tell me a story about a lighthouse", "and then what happened",
                            "how does it end"][i % 3], priority=3)


def test_history_is_the_parked_kv():
    """After a turn, the router's history of the dialog equals the token
    positions the engine parked: prompt + generated ids but the last."""
    eng = _eng()
    gw = Gateway(_cfg(), engine=eng, use_gpu_preprocess=False, prompt_cap=12, gen_tokens=3)
    t0 = _turn(0)
    gw.submit([t0])
    for _ in range(20):
        gw.tick()
        if t0.status == MessageStatus.COMPLETED:
            break
    ck = conv_key("dlg")
    slot, n = eng.export_kv(ck)
    hist = gw.conv_hist["dlg"].astype(np.int64) % MICRO.vocab
    plen = int(eng.s_plen[slot])
    kv_tokens = np.concatenate([eng.s_prompt[slot, :plen], eng.h_tokens[slot, :n - plen]])
    assert n == len(hist) and np.array_equal(hist, kv_tokens)
    assert np.any(eng.h_tokens[slot, :2] != 0)                 # real ids, not placeholders


def test_replay_equals_resident_single_gpu():
    """Turn 2 with the dialog's KV resident vs replayed from the router's
    history (KV dropped): same greedy ids."""
    prompts = [np.arange(3, 14, dtype=np.int32), np.arange(40, 47, dtype=np.int32)]
    ck = 4242
    res = _eng()
    _serve(res, Request(1, prompts[0].copy(), 3, conv=ck))
    a = _serve(res, Request(2, prompts[1].copy(), 3, conv=ck))
    assert a.reused > 0
    rep = _eng()
    r1 = _serve(rep, Request(1, prompts[0].copy(), 3, conv=ck))
    hist = np.concatenate([prompts[0], r1.out_tokens[:-1]])
    rep.drop_parked(ck)                                        # evicted: the next turn must replay
    b = _serve(rep, Request(2, prompts[1].copy(), 3, conv=ck, history=hist))
    assert b.reused == 0 and len(b.prompt) == len(hist) + len(prompts[1])
    assert a.out_tokens.tolist() == b.out_tokens.tolist()


def test_remote_replay_carries_the_real_history():
    """Home GPU down: turn 2 replays on the other rank.  Its prompt there is
    the real dialog (K_HIST rows), not zeros, and its ids equal the
    single-GPU resident run of the same dialog."""
    W = 2
    comms = FakeComm.make(W, timeout_s=20)
    gws = [Gateway(_cfg("local_first"), engine=_eng(seed=7), comm=comms[r], use_gpu_preprocess=False,
                   prompt_cap=12, gen_tokens=3) for r in range(W)]
    outs = [[], []]
    for g, o in zip(gws, outs):
        _record_outputs(g.engine, o)
    t1 = _turn(1, "d2")
    gws[1].submit([t1])
    for _ in range(40):
        _tick_all(gws)
        if t1.status == MessageStatus.COMPLETED:
            break
    assert gws[1].conv_home["d2"] == 1
    hist = gws[1].conv_hist["d2"].copy()
    gws[1].set_healthy(False, "test")                          # its KV is gone with it
    t2 = _turn(2, "d2")
    gws[1].submit([t2])
    for _ in range(40):
        _tick_all(gws)
        if t2.status == MessageStatus.COMPLETED:
            break
    assert t2.status == MessageStatus.COMPLETED and gws[1].conv_home["d2"] == 0
    meta, ids2, prompt2 = next(x for x in outs[0] if isinstance(x[0], tuple) and x[0][1] == t2.handle)
    p2 = np.asarray(t2.prompt_ids, dtype=np.uint32)[:12].astype(np.int64).astype(np.int32)
    want = np.concatenate([hist.astype(np.int64) % MICRO.vocab, p2.astype(np.int64) % MICRO.vocab])
    assert np.array_equal(prompt2, want), "the replay did not prefill the dialog's real tokens"
    assert np.count_nonzero(prompt2[:len(hist)]) > len(hist) // 2
    # the same dialog on one GPU with its KV resident
    ref = _eng(seed=7)
    p1 = np.asarray(t1.prompt_ids, dtype=np.uint32)[:12].astype(np.int64).astype(np.int32)
    _serve(ref, Request(1, p1, 3, conv=77))
    r2 = _serve(ref, Request(2, p2.copy(), 3, conv=77))
    assert r2.reused > 0 and r2.out_tokens.tolist() == ids2
    # ... and the origin's history now holds turn 2's real ids from the K_DONE record
    h2 = gws[1].conv_hist["d2"]
    assert np.array_equal(h2[len(hist) + len(p2):] % MICRO.vocab, np.asarray(ids2[:-1]))


@pytest.mark.parametrize("residency", [True, False])
def test_k_done_records_carry_generated_ids_home(residency):
    """A dialog turn run on another rank: its generated ids travel back in
    the completion record and extend the origin's history -- also with KV
    residency off (the descriptor's conversation key is then -1; the
    DIALOG_TURN flag still marks it a dialog turn)."""
    W = 2
    comms = FakeComm.make(W, timeout_s=20)
    gws = [Gateway(_cfg("round_robin"), engine=_eng(seed=7), comm=comms[r], use_gpu_preprocess=False,
                   prompt_cap=12, gen_tokens=3) for r in range(W)]
    for g in gws:
        g.kv_residency = residency
    outs = [[], []]
    for g, o in zip(gws, outs):
        _record_outputs(g.engine, o)
    turns = [_turn(i, f"c{i}") for i in range(4)]
    gws[0].submit(turns)
    for _ in range(60):
        _tick_all(gws)
        if all(t.status == MessageStatus.COMPLETED for t in turns):
            break
    ran_remote = [t for t in turns if gws[0].conv_home[t.conversation_id] == 1]
    assert ran_remote, "round robin placed nothing on rank 1"
    for t in ran_remote:
        ids = next(x[1] for x in outs[1] if isinstance(x[0], tuple) and x[0][1] == t.handle)
        h = gws[0].conv_hist[t.conversation_id]
        assert h[-2:].tolist() == ids[:-1]
    assert gws[0].counters["dialog_ids_placeholder"] == 0
    assert gws[0].counters["dialog_ids_real"] == len(turns)


def test_evicted_window_prefix_is_prepended_to_a_replay():
    """N5's salient tokens of an evicted window reach the model: a replay
    prefills them ahead of the dialog history (a resident turn does not)."""
    from llm_message_queue_amd.conversation.state_manager import StateManager
    sm = StateManager()
    conv = sm.create_conversation("u")
    with sm._lock:
        sm._convs[conv.id].summary_tokens = [101, 202, 303]
    eng = _eng()
    gw = Gateway(_cfg(), engine=eng, use_gpu_preprocess=False, prompt_cap=12, gen_tokens=2, state_manager=sm)
    m = _turn(0, conv.id)
    gw.submit([m])
    gw.ingest()
    gw.conv_hist[conv.id] = np.arange(10, 20, dtype=np.int32)   # a dialog this GPU does not hold
    seen = []
    orig = eng.admit
    eng.admit = lambda reqs: (seen.extend(reqs), orig(reqs))[1]
    gw.dispatch()
    assert len(seen) == 1
    r = seen[0]
    assert r.reused == 0
    assert r.prompt[:3].tolist() == [101, 202, 303]
    assert r.prompt[3:13].tolist() == list(range(10, 20))
