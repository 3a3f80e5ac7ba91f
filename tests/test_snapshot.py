"""Queue checkpoint/resume: queued, in-flight, delayed-retry and dead-letter
messages survive a restart (the reference loses all of them; its queue
snapshots are doc-only, docs/configuration.md:290-309)."""
import time

import numpy as np

from llm_message_queue_amd.models.message import MessageStatus, new_message
from llm_message_queue_amd.queue.factory import QueueFactory, QueueType
from llm_message_queue_amd.queue.snapshot import read_snapshot, write_snapshot
from llm_message_queue_amd.utils.config import default_config


def factory():
    cfg = default_config().queue
    cfg.enable_metrics = False
    f = QueueFactory(cfg)
    m = f.create_queue_manager("standard", QueueType.STANDARD)
    for lv in ("realtime", "high", "normal", "low"):
        if not m.has_queue(lv):
            m.create_queue(lv)
    return f, m


def test_snapshot_roundtrip(tmp_path):
    f, m = factory()
    queued = [new_message("c", "u", f"msg {i}", 3) for i in range(5)]
    for q in queued:
        q.queue_name = "normal"
        q.prompt_ids = np.arange(4, dtype=np.uint32) + 7
        m.push_message("normal", q)
    rt = new_message("c", "u", "now", 1)
    m.push_message("realtime", rt)
    infl = new_message("c", "u", "was running", 2)
    infl.queue_name, infl.status = "high", MessageStatus.PROCESSING
    dead = new_message("c", "u", "failed thrice", 4)
    dead.retry_count = 3
    f.dead_letter_queue.push(dead, "boom", "low")
    later = new_message("c", "u", "retry me", 3)
    later.queue_name = "normal"
    ready = time.time_ns() + 200_000_000
    f.delayed_queue.schedule(later, ready)
    path = str(tmp_path / "snap.jsonl")
    counts = write_snapshot(f, path, inflight=[infl])
    assert counts == {"queued": 6, "inflight": 1, "delayed": 1, "dead_letter": 1}
    f.close()

    g, n = factory()
    got = read_snapshot(g, path)
    assert got == {"queued": 6, "inflight": 1, "delayed": 1, "dead_letter": 1, "rejected": 0}
    out = n.batch_pop_messages("normal", 10)
    assert [x.id for x in out] == [q.id for q in queued]                     # FIFO order preserved
    assert np.array_equal(out[0].prompt_ids, queued[0].prompt_ids)
    assert n.pop_message("realtime").id == rt.id
    h = n.pop_message("high")
    assert h.id == infl.id and h.status == MessageStatus.PENDING             # in-flight re-queued
    it = g.dead_letter_queue.get(0)
    assert (it.message.id, it.fail_reason, it.source_queue, it.retry_count) == (dead.id, "boom", "low", 3)
    msg, r, ok = g.delayed_queue.peek()
    assert ok and msg.id == later.id and r == ready
    t0 = time.time()                                                          # the retry still fires on time
    while n.size("normal") == 0 and time.time() - t0 < 3:
        time.sleep(0.01)
    assert n.pop_message("normal").id == later.id and time.time_ns() >= ready - 2_000_000
    g.close()
    assert read_snapshot(g, str(tmp_path / "missing.jsonl")) is None


def test_gateway_app_resumes_after_restart(tmp_path):
    from llm_message_queue_amd.gateway.app import GatewayApp
    cfg = default_config()
    cfg.queue.worker.process_interval = 5_000_000
    cfg.preprocessor.batch_window_us = 200
    cfg.queue.snapshot_path = str(tmp_path / "q.jsonl")
    a = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1), start=False)    # no dispatcher running
    msgs = [new_message("", "u", "urgent thing" if i % 2 else f"plain {i}", 0) for i in range(12)]
    for x in msgs:
        assert a.submit(x) is None
    a.stop()                                                                      # snapshot at shutdown
    b = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1))
    try:
        t0 = time.time()
        while time.time() - t0 < 10:
            if all((b.messages.get(x.id) or x).status == "completed" for x in msgs):
                break
            time.sleep(0.02)
        got = [b.messages.get(x.id) for x in msgs]
        assert all(g is not None and g.status == "completed" for g in got)
        assert [g.priority for g in got] == [x.priority for x in msgs]          # preprocessing kept
    finally:
        b.stop()


def test_multi_rank_snapshot_files(tmp_path):
    """Every rank of a multi-GPU job snapshots its own queues to
    ``<path>.rank<r>``; at start rank r replays its file plus those of ranks
    k = r mod world of a previous job of another size (and rank 0 a
    single-rank file), so nothing is replayed twice or lost."""
    from types import SimpleNamespace
    from llm_message_queue_amd.gateway.app import GatewayApp
    base = str(tmp_path / "q.snap")

    def app(rank, world):
        return SimpleNamespace(cfg=SimpleNamespace(queue=SimpleNamespace(snapshot_path=base)),
                               gateway=SimpleNamespace(rank=rank, world=world))

    assert GatewayApp.snapshot_file(app(0, 1)) == base
    assert GatewayApp.snapshot_file(app(3, 8)) == base + ".rank3"
    for f in [base] + [f"{base}.rank{k}" for k in range(8)] + [base + ".rank1.resumed", base + ".rankx"]:
        open(f, "w").close()
    got = {r: GatewayApp._snapshots_to_resume(app(r, 4)) for r in range(4)}
    assert got[0] == [base, base + ".rank0", base + ".rank4"]
    assert got[1] == [base + ".rank1", base + ".rank5"]
    assert sorted(sum(got.values(), [])) == sorted([base] + [f"{base}.rank{k}" for k in range(8)])
