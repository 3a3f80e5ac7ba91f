"""Serve-loop stall watchdog (``server.stall_dump_after``)."""


def _watchdog_app(dump_s, fatal_s, pending=3):
    import threading
    from types import SimpleNamespace
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.server.stall_dump_after = int(dump_s * 1e9)
    cfg.server.stall_fatal_after = int(fatal_s * 1e9)
    logged = []
    door = []

    class App(SimpleNamespace):
        _set_stalled = GatewayApp._set_stalled
        health = GatewayApp.health

    gw = SimpleNamespace(counters={"ticks": 7}, pending=lambda: pending, inbox_size=lambda: 0,
                         preprocessing=lambda: 0, engine=None, rank=0)
    app = App(gateway=gw, cfg=cfg, _stop=threading.Event(), stalled="", fatal=None,
              front_door=SimpleNamespace(set_health=lambda ok, reason="": door.append((ok, reason))),
              log=SimpleNamespace(error=lambda msg, **kw: logged.append((msg, kw))))
    th = threading.Thread(target=GatewayApp._stall_watchdog, args=(app,), daemon=True)
    return app, th, logged, door


def test_stall_watchdog_dumps_stacks_once(capfd):
    """``server.stall_dump_after``: no tick while requests wait -> one error
    log and every thread's stack on stderr (what a hung rank was doing), and
    /health (the app's and the C++ front door's) reports the stall."""
    import time
    app, th, logged, door = _watchdog_app(0.2, 0)
    th.start()
    time.sleep(0.8)
    assert app.health()[0] is False and "stalled" in app.health()[1]
    assert door and door[-1][0] is False
    app.gateway.counters["ticks"] += 1                 # ticks resume: healthy again
    time.sleep(0.12)                                   # (< stall_dump_after: not stalled anew yet)
    assert app.health() == (True, "") and door[-1] == (True, "")
    app._stop.set()
    th.join(2)
    assert len(logged) >= 1 and logged[0][1]["waiting"] == 3
    assert app.fatal is None                           # stall_fatal_after 0: never fatal
    assert "_stall_watchdog" in capfd.readouterr().err   # the dump names the watchdog's own frame


def test_stall_watchdog_fatal_after_threshold():
    """``server.stall_fatal_after``: a stall that lasts is fatal -- the app
    records it (cli serve exits non-zero for a restart) and stops."""
    import time
    app, th, logged, _door = _watchdog_app(0.1, 0.5)
    t0 = time.monotonic()
    th.start()
    th.join(5)
    assert not th.is_alive() and 0.4 < time.monotonic() - t0 < 3
    assert isinstance(app.fatal, RuntimeError) and "stall_fatal_after" in str(app.fatal)
    assert app._stop.is_set() and app.health()[0] is False
    assert [m for m, _ in logged][-1].startswith("serve loop stall is fatal")


def test_stall_watchdog_ignores_an_idle_loop():
    """No request waiting: an idle loop that sleeps is no stall."""
    import time
    app, th, logged, _door = _watchdog_app(0.1, 0.3, pending=0)
    th.start()
    time.sleep(0.8)
    app._stop.set()
    th.join(2)
    assert app.fatal is None and not logged and app.health() == (True, "")


def test_engine_step_timeout_raises_backend_hung():
    """A queued forward whose completion event never fires: the engine's
    non-blocking poll and its blocking reap both raise BackendHung once the
    step is older than ``step_timeout_s`` instead of waiting forever."""
    import time as _t
    import pytest
    from llm_message_queue_amd.backend.engine import BackendEngine, BackendHung, _Inflight
    from llm_message_queue_amd.models.llama_stub import LlamaConfig

    class NeverDone:
        def query(self):
            return False

        def synchronize(self):
            raise AssertionError("must not block unbounded")

    eng = BackendEngine(LlamaConfig.tiny(), slots=4, max_ctx=64, token_budget=64, device="cpu", impl="ref",
                        step_timeout_s=0.05)
    eng._q.append(_Inflight(1, NeverDone(), 8, 8, 0, [], [], _t.perf_counter(), None, _t.monotonic_ns()))
    assert eng.poll_one() is False                 # young step: just not done yet
    _t.sleep(0.08)
    with pytest.raises(BackendHung):
        eng.poll_one()
    with pytest.raises(BackendHung):
        eng.finish(block=True)


def test_serve_loop_exits_on_backend_hung():
    from llm_message_queue_amd.backend.engine import BackendEngine, BackendHung
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.enable_metrics = False
    eng = BackendEngine(LlamaConfig.tiny(), slots=4, max_ctx=64, token_budget=64, device="cpu", impl="ref")
    app = GatewayApp(cfg, use_gpu=False, engine=eng, start=False)

    def boom(*a, **k):
        raise BackendHung("forward step 7 incomplete 60.0 s after launch")
    app.gateway.tick = boom
    app.start()
    app._loop_thread.join(5)
    assert isinstance(app.fatal, BackendHung) and app._stop.is_set()
    app.stop()


def test_serve_loop_defect_is_fatal_not_a_zombie():
    """An unexpected exception in the tick used to end the dispatcher thread
    silently while the API kept accepting requests; now it is logged and
    fatal (the process exits non-zero and is restarted)."""
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.enable_metrics = False
    eng = BackendEngine(LlamaConfig.tiny(), slots=4, max_ctx=64, token_budget=64, device="cpu", impl="ref")
    app = GatewayApp(cfg, use_gpu=False, engine=eng, start=False)

    def boom(*a, **k):
        raise KeyError("a bug")
    app.gateway.tick = boom
    app.start()
    app._loop_thread.join(5)
    assert isinstance(app.fatal, KeyError) and app._stop.is_set()
    app.stop()


def test_no_periodic_full_gc_by_default(monkeypatch):
    """A full collection stops the process for the whole serving heap (the
    CPU-sim soak's p99 went 43 -> 383 ms with one every 20 s), so the serve
    loop only freezes survivors by default; a full pass runs only when
    ``server.gc_full_interval`` asks for it."""
    import gc
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.utils.config import default_config
    calls = {"collect": 0, "freeze": 0}
    monkeypatch.setattr(gc, "collect", lambda *a: calls.__setitem__("collect", calls["collect"] + 1) or 0)
    monkeypatch.setattr(gc, "freeze", lambda: calls.__setitem__("freeze", calls["freeze"] + 1))
    monkeypatch.setattr(gc, "unfreeze", lambda: None)
    for full, want in ((None, 0), (1_000_000_000, 1)):
        cfg = default_config()
        cfg.queue.enable_metrics = False
        if full is not None:
            cfg.server.gc_full_interval = full
        eng = BackendEngine(LlamaConfig.tiny(), slots=4, max_ctx=64, token_budget=64, device="cpu", impl="ref")
        app = GatewayApp(cfg, use_gpu=False, engine=eng, start=False)
        calls.update(collect=0, freeze=0)
        app._gc_freeze_at = app._gc_full_at = 0.0
        app._gc_maintenance(3600.0)
        assert calls["collect"] == want and calls["freeze"] == 1, (full, calls)
        app.stop()


def test_message_index_unfiltered_page_matches_scan():
    """GET /messages without filters reads only the page (a scan of the
    200k-message index costs ~100 ms of interpreter time the serve loop
    shares); the page and count match the filtered scan's semantics."""
    from llm_message_queue_amd.gateway.app import MessageStore
    from llm_message_queue_amd.models.message import Message
    st = MessageStore(max_items=50)
    for i in range(80):
        st.put(Message(id=f"m{i}", content="x", priority=3, user_id="u"))
    n, page = st.query(limit=7, offset=3)
    n2, page2 = st.query(limit=7, offset=3, user_id="u")
    assert n == n2 == 50 and [m.id for m in page] == [m.id for m in page2] == [f"m{i}" for i in range(33, 40)]
    assert st.query(limit=5, offset=48)[1][-1].id == "m79" and st.query(limit=5, offset=60)[1] == []


def test_message_index_filtered_queries_match_a_scan():
    """The per-user / per-conversation sub-indexes give the same pages and
    counts as a full scan through puts, re-puts, removals and evictions."""
    import random
    from llm_message_queue_amd.gateway.app import MessageStore
    from llm_message_queue_amd.models.message import Message
    rng = random.Random(5)
    st = MessageStore(max_items=60)
    for step in range(3000):
        op = rng.random()
        mid = f"m{rng.randrange(120)}"
        if op < 0.6:
            st.put(Message(id=mid, content="x", priority=3, user_id=f"u{rng.randrange(5)}",
                           conversation_id=rng.choice(["", "c1", "c2", "c3"])))
        elif op < 0.75:
            st.remove(mid)
        else:
            u = rng.choice(["", "u0", "u1", "u3"])
            c = rng.choice(["", "c1", "c2"])
            s = rng.choice(["", "pending", "completed"])
            off, lim = rng.randrange(0, 20), rng.randrange(0, 15)
            allm = st.values()
            want = [m for m in allm if (not u or m.user_id == u) and (not c or m.conversation_id == c)
                    and (not s or m.status == s)]
            n, page = st.query(user_id=u, conversation_id=c, status=s, limit=lim, offset=off)
            assert n == len(want) and [m.id for m in page] == [m.id for m in want[off:off + lim]], step
    assert len(st.values()) <= 60


def test_message_index_reput_after_key_change_does_not_leak():
    """the same Message object re-put after its user_id changed
    leaves nothing under the old key (the index remembers where it filed it)."""
    from llm_message_queue_amd.gateway.app import MessageStore
    from llm_message_queue_amd.models.message import Message
    st = MessageStore(max_items=10)
    m = Message(id="m1", content="x", priority=3, user_id="alice", conversation_id="c1")
    st.put(m)
    m.user_id, m.conversation_id = "bob", ""
    st.put(m)
    assert "alice" not in st._by["user_id"] and "c1" not in st._by["conversation_id"]
    assert st.query(user_id="bob")[0] == 1 and st.query(user_id="alice")[0] == 0
    st.remove("m1")
    assert not st._by["user_id"] and not st._keys
    for i in range(30):                                   # eviction unindexes too
        st.put(Message(id=f"e{i}", content="x", priority=3, user_id=f"u{i}"))
    assert len(st._keys) == 10 and len(st._by["user_id"]) == 10
