"""In-flight processing timeout and cancellation (VERDICT r4 missing #1).

Reference: every message is processed under
``context.WithTimeout(msg.Timeout)`` and a failure goes through
``handleFailure`` -- retry with backoff while RetryCount < MaxRetries, else
the dead-letter queue (`internal/priorityqueue/worker.go:162-188, 202-239`).
Here a request's attempt gets ``Message.timeout`` from its admission into a
GPU batch slot; past it the engine aborts the request (slot freed for the
next admission) and the gateway retries or dead-letters it.  ``DELETE
/api/v1/messages/{id}`` aborts a running request on whichever GPU runs it."""
import threading
import time

import numpy as np
import pytest

from llm_message_queue_amd.backend.engine import BackendEngine, Request
from llm_message_queue_amd.gateway.router import Gateway
from llm_message_queue_amd.gateway.workload import Workload
from llm_message_queue_amd.models.llama_stub import LlamaConfig
from llm_message_queue_amd.models.message import MessageStatus
from llm_message_queue_amd.parallel.comm import FakeComm
from llm_message_queue_amd.queue.dead_letter import DeadLetterQueue
from llm_message_queue_amd.queue.delayed import DelayedQueue
from llm_message_queue_amd.queue.worker import FixedBackoff
from llm_message_queue_amd.utils.config import default_config


def _cfg():
    c = default_config()
    c.queue.enable_metrics = False
    return c


def _gw(max_retries, gen_tokens=40, slots=8, comm=None, backoff_ms=20):
    eng = BackendEngine(LlamaConfig.tiny(), slots=slots, max_ctx=64, token_budget=128, device="cpu", impl="ref")
    dlq = DeadLetterQueue()
    gw = Gateway(_cfg(), engine=eng, comm=comm, use_gpu_preprocess=False, prompt_cap=8, gen_tokens=gen_tokens,
                 dead_letter=dlq)
    gw.attach_retry_queue(DelayedQueue(), FixedBackoff(backoff_ms * 1_000_000, max_retries))
    return gw, eng, dlq


def test_engine_expire_and_cancel_free_slots_for_the_next_admission():
    eng = BackendEngine(LlamaConfig.tiny(), slots=4, max_ctx=64, token_budget=64, device="cpu", impl="ref")
    reqs = [Request(i, np.arange(5, dtype=np.int32), gen_tokens=30, timeout_ns=(1_000 if i < 2 else 0))
            for i in range(3)]
    eng.admit(reqs)
    eng.launch()
    eng.finish(block=True)
    slot_of = {r.req_id: r.slot for r in reqs}
    assert all(r.deadline_ns == r.admitted_ns + r.timeout_ns for r in reqs[:2]) and reqs[2].deadline_ns == 0
    got = eng.expire(time.monotonic_ns() + 10_000)
    assert sorted(r.req_id for r in got) == [0, 1] and eng.expired_total == 2
    assert eng.inflight() == 1 and eng.expire(time.monotonic_ns() + 10**12) == []   # no deadline: never
    assert [r.req_id for r in eng.cancel([2, 99])] == [2] and eng.cancelled_total == 1
    assert eng.inflight() == 0 and not eng.active
    # the freed slots are taken first by the next admission (LIFO free list)
    nxt = eng.admit([Request(10, np.arange(4, dtype=np.int32), gen_tokens=2)])[0]
    assert nxt.slot == slot_of[2]
    while eng.active:
        eng.launch()
    assert [r.req_id for r in eng.finish(block=True).completed] == [10]


def test_inflight_timeout_aborts_retries_then_dead_letters():
    """A request still decoding past its deadline is aborted mid-decode, its
    slot is reused by the next admission, it is retried after the backoff
    (fresh queue deadline, not shed) and dead-lettered when its retry times
    out too -- with RetryCount == MaxRetries, as the reference."""
    gw, eng, dlq = _gw(max_retries=1)
    msgs = Workload(seed=4).make(3)
    for m in msgs:
        m.timeout = 150_000_000                      # 150 ms of processing per attempt
    gw.submit(msgs)
    gw.tick()
    assert eng.inflight() == 3 and all(m.status == MessageStatus.PROCESSING for m in msgs)
    slots = {r.slot for r in eng.active.values()}
    time.sleep(0.2)
    gw.tick()                                        # deadline passed mid-decode
    assert gw.counters["inflight_timeout"] == 3 and eng.expired_total == 3
    assert gw.counters["retried"] == 3 and gw.retrying() == 3 and eng.inflight() == 0
    assert all(m.retry_count == 1 and m.status == MessageStatus.PENDING for m in msgs)
    assert int(gw.inflight_by_tier.sum()) == 0
    fresh = Workload(seed=5).make(1)[0]              # the next admission reuses a freed slot
    gw.submit([fresh])
    gw.tick()
    assert next(r.slot for r in eng.active.values() if r.meta is fresh) in slots
    time.sleep(0.03)                                 # backoff over: the retries re-enter and are admitted
    # (queue-deadline shedding is covered by tests/test_gateway_retry.py; here
    # a slow host -- a 40-token CPU forward per tick -- must not shed a retry
    # that waited out a tick behind the fresh request's steps)
    gw.shed_expired = False
    for _ in range(40):                              # (the timer thread may run late on a loaded host)
        gw.tick()
        if all(m.status == MessageStatus.PROCESSING for m in msgs):
            break
        time.sleep(0.002)
    gw.shed_expired = True
    assert all(m.status == MessageStatus.PROCESSING for m in msgs), (
        [(m.status, m.retry_count) for m in msgs], dict(gw.counters))
    assert gw.counters["expired"] == 0
    time.sleep(0.2)
    gw.tick()                                        # the retry times out too: retries spent
    assert gw.counters["retry_exhausted"] == 3 and dlq.size() == 3
    items = dlq.get_all()
    assert all(it.retry_count == 1 and "processing timeout" in it.fail_reason for it in items)
    assert all(m.status == MessageStatus.FAILED for m in msgs)
    for _ in range(200):                             # the fresh request (30 s timeout) completes
        gw.tick()
        if fresh.status == MessageStatus.COMPLETED:
            break
    assert fresh.status == MessageStatus.COMPLETED and int(gw.inflight_by_tier.sum()) == 0


def test_inflight_timeout_off_runs_to_completion():
    gw, eng, _dlq = _gw(max_retries=1, gen_tokens=6)
    gw.inflight_timeout = False
    msgs = Workload(seed=4).make(2)
    for m in msgs:
        m.timeout = 100_000_000
    gw.submit(msgs)
    gw.tick()
    assert eng.inflight() == 2
    time.sleep(0.15)
    for _ in range(50):
        gw.tick()
    assert gw.counters["inflight_timeout"] == 0 and all(m.status == MessageStatus.COMPLETED for m in msgs)


def test_cancel_running_request_single_rank():
    gw, eng, _dlq = _gw(max_retries=3)
    msgs = Workload(seed=6).make(3)
    gw.submit(msgs)
    gw.tick()
    assert eng.inflight() == 3
    f = gw.request_cancel(msgs[1])
    gw.tick()
    assert f.result(timeout=1) == "cancelled"
    assert msgs[1].status == MessageStatus.CANCELLED and gw.counters["cancelled"] == 1
    assert eng.cancelled_total == 1 and eng.inflight() == 2
    f2 = gw.request_cancel(Workload(seed=7).make(1)[0])   # not in flight here
    gw.tick()
    assert f2.result(timeout=1) == ""
    for _ in range(200):
        gw.tick()
        if gw.counters["completed"] == 2:
            break
    assert gw.counters["completed"] == 2 and int(gw.inflight_by_tier.sum()) == 0
    st = gw.qm.get_all_queue_stats()
    assert sum(s.processing_count for s in st.values()) == 0


def _tick_all(gws, n=1, sleep=0.0):
    for _ in range(n):
        ths = [threading.Thread(target=g.tick) for g in gws]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if sleep:
            time.sleep(sleep)


def test_multirank_cancel_reaches_the_gpu_running_the_request():
    """Rank 0's requests overflow onto rank 1's GPU; cancelling one that runs
    there sends K_CANCEL with the next exchange, rank 1 aborts it (slot
    freed) and reports K_CANCELLED back; the rest complete and every
    in-flight count returns to zero."""
    comms = FakeComm.make(2, timeout_s=20)
    g0, e0, _d0 = _gw(max_retries=3, slots=2, comm=comms[0])
    g1, e1, _d1 = _gw(max_retries=3, slots=8, comm=comms[1])
    msgs = Workload(seed=8).make(6)
    g0.submit(msgs)
    _tick_all([g0, g1], 2)
    remote = [m for m in g0.remote_out.values()]
    assert remote, "the plan placed nothing on rank 1"
    victim = remote[0]
    f = g0.request_cancel(victim)
    for _ in range(6):
        _tick_all([g0, g1])
        if g0.counters["cancelled"]:
            break
    assert f.result(timeout=1) == "forwarded"
    assert g0.counters["cancelled"] == 1 and victim.status == MessageStatus.CANCELLED
    assert e1.cancelled_total == 1 and victim.handle not in g0.remote_out
    for _ in range(300):
        _tick_all([g0, g1])
        if g0.counters["completed"] == 5:
            break
    assert g0.counters["completed"] == 5
    assert int(g0.inflight_by_tier.sum()) == 0 and int(g1.inflight_by_tier.sum()) == 0
    assert not g1.foreign and e0.inflight() == 0 and e1.inflight() == 0


def test_multirank_timeout_on_the_remote_gpu_goes_back_to_the_origin():
    """A request running on another rank's GPU past its deadline: that rank
    aborts it and reports K_TIMEOUT; the origin router takes the failure
    path (here no retries left -> its dead-letter queue)."""
    comms = FakeComm.make(2, timeout_s=20)
    g0, e0, d0 = _gw(max_retries=0, slots=2, comm=comms[0])
    g1, e1, _d1 = _gw(max_retries=0, slots=8, comm=comms[1])
    msgs = Workload(seed=9).make(6)
    for m in msgs:
        m.timeout = 15_000_000
    g0.submit(msgs)
    _tick_all([g0, g1], 2)
    n_remote = len(g0.remote_out)
    assert n_remote > 0
    _tick_all([g0, g1], 1, sleep=0.04)
    for _ in range(8):
        _tick_all([g0, g1])
        if d0.size() == 6:
            break
    assert d0.size() == 6 and g0.counters["inflight_timeout"] == 6
    assert e1.expired_total == n_remote and e0.expired_total == 6 - n_remote
    assert not g0.remote_out and not g1.foreign
    assert int(g0.inflight_by_tier.sum()) == 0 and int(g1.inflight_by_tier.sum()) == 0


def test_delete_cancels_a_running_request_through_the_api():
    """``DELETE /api/v1/messages/{id}`` on a request running in a GPU slot
    aborts it there (the round-4 API only dropped it from the index while
    the slot kept running it)."""
    from fastapi.testclient import TestClient
    from llm_message_queue_amd.api.server import create_app
    from llm_message_queue_amd.gateway.app import GatewayApp
    cfg = _cfg()
    cfg.backend.gen_tokens = 50
    eng = BackendEngine(LlamaConfig.tiny(), slots=4, max_ctx=128, token_budget=64, device="cpu", impl="ref")
    eng.inject(slow_ms=20)                          # ~1 s per request: still running at the DELETE
    app = GatewayApp(cfg, use_gpu=False, engine=eng, start=False)
    from llm_message_queue_amd.balancer.load_balancer import Endpoint
    app.lb.add_endpoint(Endpoint(id="gpu0", type="llm", gpu_index=0, max_connections=4))   # (as cli serve)
    app.start()
    try:
        c = TestClient(create_app(app))
        r = c.post("/api/v1/messages", json={"content": "long running job", "user_id": "u"})
        assert r.status_code == 202
        mid = r.json()["message_id"]
        t0 = time.time()
        while time.time() - t0 < 10 and c.get(f"/api/v1/messages/{mid}").json().get("status") != "processing":
            time.sleep(0.02)
        r = c.delete(f"/api/v1/messages/{mid}")
        assert r.status_code == 200 and r.json()["cancelled"] is True and r.json()["dequeued"] is False
        assert eng.cancelled_total == 1 and app.gateway.counters["cancelled"] == 1
        assert c.get(f"/api/v1/messages/{mid}").status_code == 404
    finally:
        eng.inject(slow_ms=0)
        app.stop()


@pytest.mark.gpu
def test_gpu_cancelled_slot_reuse_matches_a_fresh_slot():
    """On the HIP engine: a request cancelled mid-prefill frees its slot; the
    next request admitted into that slot generates exactly the tokens it
    generates in a fresh engine (nothing of the aborted request leaks)."""
    import torch

    def run(cancel_first):
        eng = BackendEngine(LlamaConfig.tiny(), slots=4, max_ctx=128, token_budget=32, device="cuda:0",
                            impl="hip", seed=3)
        if cancel_first:
            a = eng.admit([Request(1, (np.arange(100) * 7 % 500).astype(np.int32), gen_tokens=8)])[0]
            eng.launch()                                # a 32-token chunk of its 100-token prompt
            eng.finish(block=True)
            assert [r.req_id for r in eng.cancel([1])] == [1]
            slot = a.slot
        b = eng.admit([Request(2, (np.arange(20) * 3 % 500).astype(np.int32), gen_tokens=6)])[0]
        if cancel_first:
            assert b.slot == slot
        toks = []
        while eng.active:
            eng.launch()
            eng.finish(block=True)
            toks.append(eng._prev_out.cpu().tolist())
        torch.cuda.synchronize()
        return b.slot, toks

    s1, t1 = run(True)
    s2, t2 = run(False)
    assert t1 == t2 and len(t1) == 6


def test_a_retry_gets_a_fresh_queue_deadline():
    """A retried request is judged against its REQUEUE time, not its first
    arrival (its first deadline has passed by definition)."""
    from llm_message_queue_amd.gateway.gateway_failure import FailureMixin
    now = time.monotonic_ns()
    m = Workload(seed=12).make(1)[0]
    m.timeout = 100_000_000
    m.arrival_ns = now - 500_000_000
    m.enqueued_at = now - 10_000_000
    assert FailureMixin._expired(m, now)                 # first attempt: 500 ms since arrival
    m.retry_count = 1
    assert not FailureMixin._expired(m, now)             # retry: 10 ms since its requeue
    m.enqueued_at = now - 200_000_000
    assert FailureMixin._expired(m, now)
