"""Backend-failure retries on the GPU gateway path (reference
`internal/priorityqueue/worker.go:202-239`, `delayed_queue.go`,
`dead_letter_queue.go:62-119`): requests an evacuated backend hands back wait
out a backoff in the DelayedQueue before re-entering their tier, and land in
the dead-letter queue once their retries are spent."""
import time

from llm_message_queue_amd.backend.engine import BackendEngine
from llm_message_queue_amd.gateway.router import Gateway
from llm_message_queue_amd.gateway.workload import Workload
from llm_message_queue_amd.models.llama_stub import LlamaConfig
from llm_message_queue_amd.queue.dead_letter import DeadLetterQueue
from llm_message_queue_amd.queue.delayed import DelayedQueue
from llm_message_queue_amd.queue.worker import FixedBackoff
from llm_message_queue_amd.utils.config import default_config


def _gw(max_retries):
    cfg = default_config()
    cfg.queue.enable_metrics = False
    eng = BackendEngine(LlamaConfig.tiny(), slots=8, max_ctx=64, token_budget=128, device="cpu", impl="ref")
    dlq = DeadLetterQueue()
    gw = Gateway(cfg, engine=eng, use_gpu_preprocess=False, prompt_cap=8, gen_tokens=4, dead_letter=dlq)
    dq = DelayedQueue()                        # no drain thread: the tick polls it
    gw.attach_retry_queue(dq, FixedBackoff(20_000_000, max_retries))
    return gw, eng, dlq, dq


def test_evacuated_requests_retry_after_backoff_then_complete():
    gw, eng, dlq, dq = _gw(max_retries=2)
    msgs = Workload(seed=3).make(4)
    gw.submit(msgs)
    gw.tick()                                   # ingest + admit
    assert eng.inflight() == 4
    n = gw.set_healthy(False, "injected fault")
    assert n == 4 and gw.counters["retried"] == 4 and gw.retrying() == 4
    assert gw.pending() == 0                    # waiting out the backoff, not queued yet
    gw.set_healthy(True)
    gw.tick()
    assert gw.pending() + eng.inflight() == 0   # still in the delayed queue
    time.sleep(0.03)
    t0 = time.time()
    while gw.counters["completed"] < 4 and time.time() - t0 < 20:
        gw.tick()
    assert gw.counters["completed"] == 4 and gw.retrying() == 0
    assert all(m.retry_count == 1 for m in msgs) and dlq.size() == 0


def test_retries_exhausted_go_to_the_dead_letter_queue():
    gw, eng, dlq, dq = _gw(max_retries=1)
    msgs = Workload(seed=4).make(3)
    gw.submit(msgs)
    gw.tick()
    gw.set_healthy(False, "fault 1")
    gw.set_healthy(True)
    time.sleep(0.03)
    gw.tick()                                   # back in the queue and re-admitted
    assert eng.inflight() == 3
    gw.set_healthy(False, "fault 2")            # second failure: retries (1) spent
    assert gw.counters["retry_exhausted"] == 3 and dlq.size() == 3
    items = dlq.get_all()
    # dead-lettered with RetryCount == MaxRetries, as the reference's
    # handleFailure (worker.go:210) -- not incremented on that path
    assert all("retries exhausted" in it.fail_reason and it.retry_count == 1 for it in items)
    assert gw.retrying() == 0 and gw.pending() == 0


def _pair():
    import threading
    from llm_message_queue_amd.parallel.comm import FakeComm
    comms = FakeComm.make(2)
    gws = []
    for r in range(2):
        cfg = default_config()
        cfg.queue.enable_metrics = False
        eng = BackendEngine(LlamaConfig.tiny(), slots=8, max_ctx=64, token_budget=128, device="cpu", impl="ref")
        gw = Gateway(cfg, engine=eng, comm=comms[r], use_gpu_preprocess=False, prompt_cap=8, gen_tokens=4,
                     dead_letter=DeadLetterQueue())
        gw.attach_retry_queue(DelayedQueue(), FixedBackoff(20_000_000, 3))
        gws.append(gw)

    def tick():
        ths = [threading.Thread(target=g.tick) for g in gws]
        [t.start() for t in ths]
        [t.join() for t in ths]
    return gws, tick


def _remote_inflight(gws, tick, n):
    msgs = Workload(seed=9).make(n)
    for m in msgs:
        m.metadata["home_gpu"] = 1                  # every turn is placed on GPU 1
    gws[0].submit(msgs)
    for _ in range(6):
        tick()
        if gws[1].engine.inflight() == n:
            break
    assert gws[1].engine.inflight() == n and len(gws[0].remote_out) == n
    return msgs


def test_remote_operator_drain_requeues_without_spending_a_retry():
    """a request handed back by a backend that never failed it
    (an operator's drain) re-enters its tier at once -- no backoff, no retry."""
    gws, tick = _pair()
    msgs = _remote_inflight(gws, tick, 4)
    assert gws[1].set_healthy(False, "operator drain", failure=False) == 4
    tick()                                          # the K_FAIL records travel back to the origin
    assert gws[0].counters["handed_back"] == 4 and gws[0].counters["retried"] == 0
    assert all(m.retry_count == 0 for m in msgs) and gws[0].retrying() == 0
    t0 = time.time()
    while gws[0].counters["completed"] < 4 and time.time() - t0 < 20:
        tick()
    assert gws[0].counters["completed"] == 4 and all(m.retry_count == 0 for m in msgs)


def test_remote_backend_failure_takes_the_retry_path():
    gws, tick = _pair()
    msgs = _remote_inflight(gws, tick, 4)
    assert gws[1].set_healthy(False, "injected fault") == 4
    tick()
    assert gws[0].counters["handed_back"] == 4 and gws[0].counters["retried"] == 4
    assert all(m.retry_count == 1 for m in msgs)
    time.sleep(0.03)
    t0 = time.time()
    while gws[0].counters["completed"] < 4 and time.time() - t0 < 20:
        tick()
    assert gws[0].counters["completed"] == 4
