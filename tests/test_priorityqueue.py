"""Parity ports of reference tests/priorityqueue_test.go (MultiLevelQueue,
QueueManager, Worker, DelayedQueue, DeadLetterQueue) + native-core extras."""
import queue as pyqueue
import threading
import time

import pytest

from llm_message_queue_amd.models.message import Message, new_message
from llm_message_queue_amd.queue import (DeadLetterQueue, DelayedQueue, ExponentialBackoff, FixedBackoff,
                                         IndexOutOfRange, MultiLevelQueue, QueueEmpty, QueueFull,
                                         QueueManager, QueueManagerConfig, QueueNotFound, Worker, WorkerConfig)

LEVELS = ["realtime", "high", "normal", "low"]


def mlq4():
    q = MultiLevelQueue(100)
    for n in LEVELS:
        q.add_queue(n)
    return q


# ---------------------------------------------------------------- MultiLevelQueue (:25-238)
def test_push_and_pop():
    q = mlq4()
    msgs = {n: new_message("c", "u", f"msg {n}", i + 1) for i, n in enumerate(LEVELS)}
    for i, n in enumerate(LEVELS):
        q.push(n, msgs[n], i + 1)
    for n in LEVELS:
        assert q.size(n) == 1
    for n in LEVELS:
        assert q.pop(n).id == msgs[n].id
    for n in LEVELS:
        with pytest.raises(QueueEmpty):
            q.pop(n)


def test_peek_does_not_remove():
    q = mlq4()
    m = new_message("c", "u", "x", 1)
    q.push("realtime", m, 1)
    assert q.peek("realtime").id == m.id
    assert q.size("realtime") == 1


def test_queue_stats():
    q = mlq4()
    for _ in range(5):
        q.push("realtime", new_message("c", "u", "r", 1), 1)
    for _ in range(3):
        q.push("high", new_message("c", "u", "h", 2), 2)
    assert q.get_stats("realtime").pending_count == 5
    assert q.get_stats("high").pending_count == 3


def test_complete_fail_messages():
    q = mlq4()
    for _ in range(5):
        q.push("normal", new_message("c", "u", "n", 3), 3)
    for _ in range(5):
        q.pop("normal")
    for _ in range(3):
        q.complete_message("normal")
    for _ in range(2):
        q.fail_message("normal")
    st = q.get_stats("normal")
    assert (st.completed_count, st.failed_count, st.processing_count, st.pending_count) == (3, 2, 0, 0)


def test_order_priority_then_fifo():
    q = MultiLevelQueue(0)
    q.add_queue("mixed")
    ids = []
    for i, p in enumerate([3, 1, 3, 2, 1, 4, 2]):
        m = new_message("c", "u", str(i), p)
        ids.append((p, i, m.id))
        q.push("mixed", m, p)
    got = [q.pop("mixed").id for _ in range(7)]
    assert got == [mid for _, _, mid in sorted(ids)]


def test_capacity_and_missing_queue():
    q = MultiLevelQueue(2)
    q.add_queue("a")
    q.push("a", new_message("c", "u", "1", 3))
    q.push("a", new_message("c", "u", "2", 3))
    with pytest.raises(QueueFull):
        q.push("a", new_message("c", "u", "3", 3))
    with pytest.raises(QueueNotFound):
        q.push("nope", new_message("c", "u", "3", 3))
    with pytest.raises(QueueEmpty):
        q.pop("nope")


def test_stats_are_copies():
    q = mlq4()
    s = q.get_stats("low")
    q.push("low", new_message("c", "u", "x", 4))
    assert s.pending_count == 0 and q.get_stats("low").pending_count == 1


def test_pop_tiers_strict_priority_aging_and_budgets():
    q = mlq4()
    for i in range(3):
        q.push("low", new_message("c", "u", f"l{i}", 4))
    for i in range(3):
        q.push("realtime", new_message("c", "u", f"r{i}", 1))
    msgs, tiers, _ = q.pop_tiers(LEVELS, 4, [0, 0, 0, 0], [-1, -1, -1, -1])
    assert [m.content for m in msgs] == ["r0", "r1", "r2", "l0"]
    assert list(tiers) == [0, 0, 0, 3]
    # aging: an overdue low head jumps ahead of fresh realtime work
    q.push("realtime", new_message("c", "u", "r9", 1))
    time.sleep(0.02)
    msgs, _, _ = q.pop_tiers(LEVELS, 1, [0, 0, 0, 5_000_000], [-1, -1, -1, -1])
    assert msgs[0].content == "l1"
    # budgets cap a tier
    msgs, _, _ = q.pop_tiers(LEVELS, 5, [0, 0, 0, 0], [0, -1, -1, 1])
    assert [m.content for m in msgs] == ["l2"]


def test_pop_tiers_adaptive_lifo():
    """While a tier's head is older than its LIFO threshold, the newest
    request is served (overload); FIFO otherwise."""
    q = mlq4()
    for i in range(4):
        q.push("normal", new_message("c", "u", f"n{i}", 3))
    time.sleep(0.01)
    # head younger than 1 s: FIFO
    msgs, _, _ = q.pop_tiers(LEVELS, 1, [0] * 4, [-1] * 4, [0, 0, 1_000_000_000, 0])
    assert msgs[0].content == "n0"
    # head older than 1 ms: newest first; other tiers unaffected
    q.push("high", new_message("c", "u", "h0", 2))
    q.push("high", new_message("c", "u", "h1", 2))
    msgs, tiers, _ = q.pop_tiers(LEVELS, 4, [0] * 4, [-1] * 4, [0, 0, 1_000_000, 0])
    assert [m.content for m in msgs] == ["h0", "h1", "n3", "n2"] and list(tiers) == [1, 1, 2, 2]
    st = q.get_stats("normal")
    assert st.pending_count == 1 and st.processing_count == 3
    with pytest.raises(Exception):
        q.pop_tiers(LEVELS, 1, [0] * 4, [-1] * 4, [0, 0])          # per-tier lengths must match


def test_pop_tiers_skip_leaves_requests_in_place():
    """``skip``: requests homed on another GPU are passed over (aging, strict
    priority and LIFO look at the first / last request not skipped) and stay
    queued in their original order for the tick's plan."""
    import numpy as np
    q = mlq4()
    r = [new_message("c", "u", f"r{i}", 1) for i in range(4)]
    n = [new_message("c", "u", f"n{i}", 3) for i in range(3)]
    for m in r:
        q.push("realtime", m)
    for m in n:
        q.push("normal", m)
    skip = np.array([r[0].handle, r[2].handle, n[2].handle], dtype=np.int64)
    msgs, tiers, _ = q.pop_tiers(LEVELS, 10, [0] * 4, [-1] * 4, None, skip)
    assert [m.content for m in msgs] == ["r1", "r3", "n0", "n1"] and list(tiers) == [0, 0, 2, 2]
    assert [m.content for m in q.messages("realtime")] == ["r0", "r2"]
    st = q.get_stats("realtime")
    assert st.pending_count == 2 and st.processing_count == 2
    # LIFO picks the newest request that is not skipped
    for i in range(3, 6):
        q.push("normal", new_message("c", "u", f"n{i}", 3))
    time.sleep(0.005)
    last = q.messages("normal")[-1]
    msgs, _, _ = q.pop_tiers(LEVELS, 1, [0] * 4, [0, -1, -1, -1], [0, 0, 1_000_000, 0],
                             np.array([last.handle], dtype=np.int64))
    assert msgs[0].content == "n4"
    # a fully skipped tier yields nothing; without skip the plan takes them in order
    msgs, _, _ = q.pop_tiers(LEVELS, 5, [0] * 4, [-1, 0, 0, 0], None, skip)
    assert msgs == []
    msgs, _, _ = q.pop_tiers(LEVELS, 5, [0] * 4, [-1, 0, 0, 0])
    assert [m.content for m in msgs] == ["r0", "r2"]


def test_concurrent_push_pop_no_loss():
    q = MultiLevelQueue(0)
    for n in LEVELS:
        q.add_queue(n)
    N = 4000
    got = []
    lock = threading.Lock()

    def prod(k):
        for i in range(N // 4):
            q.push(LEVELS[i % 4], new_message("c", "u", f"{k}-{i}", (i % 4) + 1))

    def cons():
        while True:
            msgs, _, _ = q.pop_tiers(LEVELS, 64, [0] * 4, [-1] * 4)
            with lock:
                got.extend(m.content for m in msgs)
                if len(got) >= N:
                    return
            if not msgs:
                time.sleep(0.0005)

    ts = [threading.Thread(target=prod, args=(k,)) for k in range(4)] + [threading.Thread(target=cons)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=30)
    assert len(got) == N and len(set(got)) == N


# ---------------------------------------------------------------- QueueManager (:271-362)
def qm():
    m = QueueManager(QueueManagerConfig(enable_metrics=False, monitor_interval=50_000_000,
                                        cleanup_interval=50_000_000), name="t")
    m.create_queue("test-queue", 100)
    return m


def test_manager_push_pop():
    m = qm()
    msg = new_message("c", "u", "hello", 3)
    m.push_message("test-queue", msg)
    assert m.pop_message("test-queue").id == msg.id


def test_manager_batch_ops():
    m = qm()
    assert m.batch_push_messages("test-queue", [new_message("c", "u", str(i), 3) for i in range(5)]) == 5
    assert m.size("test-queue") == 5
    assert len(m.batch_pop_messages("test-queue", 3)) == 3


def test_manager_complete_fail():
    m = qm()
    for i in range(5):
        m.push_message("test-queue", new_message("c", "u", str(i), 3))
    popped = [m.pop_message("test-queue") for _ in range(5)]
    for x in popped[:3]:
        m.complete_message("test-queue", x.id, 1000)
    for x in popped[3:]:
        m.fail_message("test-queue", x.id, RuntimeError("e"))
    st = m.get_queue_stats("test-queue")
    assert (st.completed_count, st.failed_count, st.processing_count) == (3, 2, 0)


def test_manager_priority_rules_and_monitor():
    from llm_message_queue_amd.queue import default_priority_rules
    m = QueueManager(QueueManagerConfig(enable_metrics=True, priority_adjust_rules=default_priority_rules(),
                                        monitor_interval=20_000_000, cleanup_interval=20_000_000,
                                        scaling_thresholds={"q": 1}), name="rules")
    m.create_queue("q")
    vip = new_message("c", "u", "x", 4)
    vip.metadata["vip_user"] = True
    long = new_message("c", "u", "y" * 10001, 1)
    m.push_message("q", vip)
    m.push_message("q", long)
    assert vip.priority == 2 and long.priority == 4
    m.start()
    time.sleep(0.1)
    m.stop()
    assert m.threshold_events and m.threshold_events[-1]["queue"] == "q"


def test_two_managers_with_metrics_do_not_collide():
    a = QueueManager(QueueManagerConfig(enable_metrics=True), name="a")
    b = QueueManager(QueueManagerConfig(enable_metrics=True), name="b")
    a.create_queue("x")
    b.create_queue("x")
    a.push_message("x", new_message("c", "u", "1", 3))
    b.push_message("x", new_message("c", "u", "1", 3))


# ---------------------------------------------------------------- Worker (:365-469)
def test_worker_processes_messages():
    m = qm()
    done = pyqueue.Queue()

    def fn(ctx, msg):
        done.put(msg.id)
        return None

    w = Worker(WorkerConfig(id="w1", queue_name="test-queue", max_batch_size=10, process_interval=10_000_000,
                            max_concurrent=5, backoff_strategy=ExponentialBackoff(10_000_000, 100_000_000, 2, 3)),
               m, fn)
    w.start()
    ids = []
    for i in range(5):
        msg = new_message("c", "u", str(i), 3)
        ids.append(msg.id)
        m.push_message("test-queue", msg)
    got = {done.get(timeout=2) for _ in range(5)}
    w.stop()
    assert got == set(ids)
    met = w.get_metrics()
    assert met.processed_count == 5 and met.success_count == 5


def test_worker_retry_via_delayed_then_dead_letter():
    m = qm()
    dq = DelayedQueue()
    dq.start()
    dlq = DeadLetterQueue(10)
    attempts = []

    def fn(ctx, msg):
        attempts.append(time.monotonic())
        return RuntimeError("boom")

    w = Worker(WorkerConfig(id="w", queue_name="test-queue", max_batch_size=4, process_interval=5_000_000,
                            max_concurrent=2, backoff_strategy=FixedBackoff(30_000_000, 2)),
               m, fn, delayed_queue=dq, dead_letter_queue=dlq)
    w.start()
    m.push_message("test-queue", new_message("c", "u", "fail", 3))
    t0 = time.monotonic()
    while dlq.size() == 0 and time.monotonic() - t0 < 3:
        time.sleep(0.01)
    w.stop()
    dq.close()
    assert dlq.size() == 1 and len(attempts) == 3
    assert attempts[1] - attempts[0] >= 0.025 and attempts[2] - attempts[1] >= 0.025   # backoff honoured
    met = w.get_metrics()
    assert met.retry_count == 2 and met.failure_count == 3 and met.dead_lettered == 1
    st = m.get_queue_stats("test-queue")
    assert st.failed_count == 1 and st.processing_count == 0


def test_backoff():
    b = ExponentialBackoff(100, 1000, 2.0, 3)
    assert [b.next_backoff(i) for i in (0, 1, 2, 3, 4, 5)] == [100, 100, 200, 400, 800, 1000]
    assert FixedBackoff(7, 2).next_backoff(5) == 7


# ---------------------------------------------------------------- DelayedQueue (:496-566)
def test_delayed_scheduling_order_and_time():
    out = pyqueue.Queue()
    dq = DelayedQueue(lambda m: out.put((m.id, time.monotonic())))
    dq.start()
    t0 = time.monotonic()
    a, b = new_message("c", "u", "a", 3), new_message("c", "u", "b", 3)
    dq.schedule_after(b, 500_000_000)
    dq.schedule_after(a, 200_000_000)
    first = out.get(timeout=2)
    second = out.get(timeout=2)
    dq.close()
    assert first[0] == a.id and first[1] - t0 >= 0.199
    assert second[0] == b.id and second[1] - t0 >= 0.499


def test_delayed_peek():
    dq = DelayedQueue()
    m = new_message("c", "u", "x", 3)
    ready = time.time_ns() + 1_000_000_000
    dq.schedule(m, ready)
    got, at, ok = dq.peek()
    assert ok and got.id == m.id and abs(at - ready) < 10_000_000
    assert dq.size() == 1
    dq.clear()
    assert dq.size() == 0
    dq.close()


# ---------------------------------------------------------------- DeadLetterQueue (:585-697)
def test_dlq_push_and_get():
    d = DeadLetterQueue(10)
    m = new_message("c", "u", "x", 3)
    m.retry_count = 3
    d.push(m, "boom", "src")
    it = d.get(0)
    assert (it.fail_reason, it.source_queue, it.retry_count) == ("boom", "src", 3)
    with pytest.raises(IndexOutOfRange):
        d.get(5)


def test_dlq_requeue():
    d = DeadLetterQueue(10)
    m = qm()
    m.create_queue("requeue-test")
    msg = new_message("c", "u", "x", 3)
    msg.retry_count = 3
    d.push(msg, "boom", "requeue-test")
    d.requeue(0, m)
    assert d.size() == 0
    assert m.pop_message("requeue-test").retry_count == 0


def test_dlq_batch_requeue_handlers_and_notify():
    d = DeadLetterQueue(10)
    m = qm()
    m.create_queue("rq")
    seen, ch = [], pyqueue.Queue(1)
    d.add_handler(lambda it: seen.append(it.message.id))
    d.add_notification_channel(ch)
    for i in range(5):
        d.push(new_message("c", "u", str(i), 3), "r", "rq")
    assert d.batch_requeue([0, 2, 4], m) == 3
    assert d.size() == 2
    assert len(m.batch_pop_messages("rq", 10)) == 3
    time.sleep(0.05)
    assert len(seen) == 5 and ch.qsize() == 1 and d.dropped_notifications == 4
    with pytest.raises(QueueFull):
        small = DeadLetterQueue(1)
        small.push(new_message("c", "u", "a", 3), "r", "q")
        small.push(new_message("c", "u", "b", 3), "r", "q")


def test_dlq_bulk_handlers_run_on_one_worker_thread():
    """Overload shedding moves thousands of messages at once: every handler
    call still runs (asynchronously, in order) but on one worker thread, not a
    thread per item."""
    import threading
    d = DeadLetterQueue(0)
    seen = []
    d.add_handler(lambda it: seen.append(it.message.id))
    before = threading.active_count()
    msgs = [new_message("c", "u", str(i), 3) for i in range(5000)]
    assert d.push_many(msgs, "timeout", "low") == 5000
    assert threading.active_count() <= before + 1
    t0 = time.time()
    while len(seen) < 5000 and time.time() - t0 < 10:
        time.sleep(0.01)
    assert seen == [m.id for m in msgs]


def test_pop_tiers_matches_a_python_model():
    """Property test of the native dispatcher pop against a plain-Python
    model: strict priority over tiers, priority buckets then FIFO inside a
    tier, per-tier budgets, and ``skip`` (handles passed over in place)."""
    import numpy as np
    from hypothesis import given, settings, strategies as st
    from llm_message_queue_amd import _native

    item = st.tuples(st.integers(0, 2), st.integers(1, 3))          # (tier, priority)

    @settings(max_examples=150, deadline=None)
    @given(st.lists(item, max_size=40), st.data())
    def run(items, data):
        q = _native.mlq().MultiLevelQueue(0)
        names = ["t0", "t1", "t2"]
        for n in names:
            q.add_queue(n)
        model = {t: [] for t in range(3)}
        for h, (t, p) in enumerate(items):
            q.push(names[t], h, p)
            model[t].append((p, h))
        for _round in range(3):
            skip = set(data.draw(st.lists(st.integers(0, max(0, len(items) - 1)), max_size=10)))
            budget = data.draw(st.lists(st.integers(-1, 5), min_size=3, max_size=3))
            count = data.draw(st.integers(0, 12))
            hs, ti, _e = q.pop_tiers(names, count, [0, 0, 0], budget, [],
                                     np.array(sorted(skip), dtype=np.int64))
            want, b = [], list(budget)
            while len(want) < count:
                pick = None
                for t in range(3):
                    if b[t] == 0:
                        continue
                    cand = sorted((p, k, h) for k, (p, h) in enumerate(model[t]) if h not in skip)
                    if cand:
                        pick = (t, cand[0])
                        break
                if pick is None:
                    break
                t, (_p, k, h) = pick
                model[t].pop(k)
                want.append((h, t))
                if b[t] > 0:
                    b[t] -= 1
            assert list(zip(hs.tolist(), ti.tolist())) == want
            for t in range(3):
                assert q.size(names[t]) == len(model[t])

    run()
