"""Descriptor rows of the job-wide exchange (``gateway/gateway_exchange.py``):
what a router packs for another GPU (``_fill_descs``) is what that GPU
unpacks into an engine request (``_foreign_requests``), and a completion
record completes the origin's message (``_remote_done_rows``)."""
import numpy as np

from llm_message_queue_amd.gateway.descriptors import (DESC_HDR, DIALOG_TURN, K_DISPATCH, K_DONE, KV_MIGRATE, _get64,
                                                       _put64, conv_key)
from tests.test_tier_caps import _gateway


def test_put64_get64_roundtrip():
    vals = np.array([0, 1, -1, 2 ** 62 + 12345, -(2 ** 40) - 7, 2 ** 63 - 1], dtype=np.int64)
    buf = np.zeros((len(vals), 4), dtype=np.int32)
    _put64(buf, 1, vals)
    assert (_get64(buf, 1) == vals).all()
    assert (buf[:, 0] == 0).all() and (buf[:, 3] == 0).all()


def _msgs():
    from llm_message_queue_amd.models.message import Message
    out = []
    for i, (conv, plen, tier) in enumerate((("c-a", 3, 0), ("", 0, 2), ("c-b", 12, 3))):
        m = Message(id=f"m{i}", content="x", conversation_id=conv, priority=3 - tier, timeout=(i + 1) * 1_500_000_000)
        m.tier = tier
        m.arrival_ns = 10_000_000_000 + i
        m.enqueued_at = m.arrival_ns + 1_000 * (i + 1)
        m.popped_ns = m.enqueued_at + 250_000 * (i + 1)
        m.prompt_ids = np.arange(7, 7 + plen, dtype=np.uint32) if plen else None
        out.append(m)
    return out


def test_descriptor_roundtrip():
    gw = _gateway(True, [0, 0, 0, 0])
    gw.conv_hist["c-b"] = np.zeros(5, dtype=np.int32)
    msgs = _msgs()
    cap = 8
    buf = np.zeros((len(msgs), DESC_HDR + cap), dtype=np.int32)
    gw._fill_descs(buf, msgs, 3, cap, {id(msgs[2]): 1})
    assert (buf[:, 0] == K_DISPATCH).all()
    # home GPU 1 -> flags (1 + 1) | KV_MIGRATE; conversation turns flagged DIALOG_TURN
    assert buf[2, 11] == (2 | KV_MIGRATE | DIALOG_TURN) and buf[0, 11] == DIALOG_TURN and buf[1, 11] == 0
    reqs = gw._foreign_requests(buf, cap)
    for m, r in zip(msgs, reqs):
        origin, h, tier, arr, enq, dec = r.meta
        assert (origin, h, tier, arr, enq) == (3, m.handle, m.tier, m.arrival_ns, m.enqueued_at)
        assert r.tier == m.tier and r.gen_tokens == gw.gen_tokens
        # the decision time travels as whole microseconds after enqueue
        assert dec == m.enqueued_at + (m.popped_ns - m.enqueued_at) // 1000 * 1000
        plen = 0 if m.prompt_ids is None else min(cap, len(m.prompt_ids))
        want = list(m.prompt_ids[:plen]) if plen else [0]
        assert r.prompt.tolist() == want                                   # prompts are truncated to the cap
        assert r.conv == (conv_key(m.conversation_id) if m.conversation_id else -1)
        assert r.timeout_ns == m.timeout // 1_000_000 * 1_000_000
        assert r.dialog == bool(m.conversation_id)
    assert reqs[2].history is not None and len(reqs[2].history) == 5     # replay length of a non-resident dialog
    assert reqs[0].history is None


def test_remote_done_completes_origin_message():
    gw = _gateway(True, [0, 0, 0, 0])
    m = _msgs()[0]
    gw.remote_out[m.handle] = m
    gw.inflight_by_tier[m.tier] += 1
    done = []
    gw.on_complete = done.append
    rows = np.zeros((2, DESC_HDR), dtype=np.int32)
    rows[:, 0] = K_DONE
    _put64(rows, 1, [m.handle, 987654321])      # the second handle is unknown: ignored
    rows[:, 3] = 1
    _put64(rows, 5, [1_000, 1_000])
    _put64(rows, 7, [4_000, 4_000])
    gw._remote_done_rows(rows)
    assert done == [m] and m.handle not in gw.remote_out
    assert gw.inflight_by_tier[m.tier] == 0 and gw.counters["completed"] == 1
