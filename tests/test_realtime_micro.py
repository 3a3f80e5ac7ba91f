"""Realtime micro-forwards (``backend.realtime_mode = micro``, VERDICT r5
missing #1): realtime requests take slots of a separate pool that only small
forwards over those slots touch, on their own stream, so their 4 forwards do
not wait for the 41 ms serving steps.

* the engine generates the same greedy tokens for a request whichever pool
  serves it (CPU: the fp32 reference ops, exact; GPU: the HIP kernels on two
  concurrent streams, same ids);
* the pools never share a slot, aborts return a slot to its own pool, and the
  gateway completes realtime requests from the micro pool;
* generated ids are read back per step (``Request.out_tokens``).
Reference claim the mode exists for: realtime processing < 100 ms
(`/root/reference/docs/architecture.md:233`)."""
import numpy as np
import pytest
import torch


def _engine(mode, device="cpu", impl="ref", **kw):
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    return BackendEngine(LlamaConfig.tiny(), slots=kw.pop("slots", 8), max_ctx=64, token_budget=kw.pop("budget", 32),
                         device=device, impl=impl, seed=3, realtime_mode=mode, micro_slots=kw.pop("micro_slots", 4),
                         **kw)


def _requests(n=12, seed=0, gen=4):
    from llm_message_queue_amd.backend.engine import Request
    rng = np.random.default_rng(seed)
    return [Request(req_id=i, prompt=rng.integers(0, 1000, size=5 + i % 7).astype(np.int32), gen_tokens=gen,
                    tier=i % 3) for i in range(n)]


def _serve(eng, reqs):
    got = {}
    pend = list(reqs)
    for _ in range(200):
        if not pend and not eng.active and not eng.queued_steps():
            break
        adm = eng.admit(pend)
        ids = {id(r) for r in adm}
        pend = [r for r in pend if id(r) not in ids]
        eng.launch()
        eng.pump_micro()
        for r in eng.finish(block=True).completed:
            got[r.req_id] = (r.out_tokens.tolist(), r.micro)
    return got


def test_micro_pool_same_tokens_cpu():
    a = _serve(_engine("off"), _requests())
    eng = _engine("micro")
    b = _serve(eng, _requests())
    assert sorted(a) == sorted(b) == list(range(12))
    assert all(len(v[0]) == 4 for v in a.values())
    assert {k: v[0] for k, v in a.items()} == {k: v[0] for k, v in b.items()}
    assert sum(v[1] for v in b.values()) == 4                # tier 0: ids 0, 3, 6, 9
    assert all(v[1] == (k % 3 == 0) for k, v in b.items())
    assert eng.micro_steps >= 4 and len(eng.free_micro) == eng.micro_slots and len(eng.free) == eng.slots


def test_micro_pools_never_share_a_slot_and_aborts_return_home():
    eng = _engine("micro")
    reqs = _requests(12, gen=8)                              # longer than the micro run-ahead (4)
    adm = eng.admit(reqs)
    micro = [r for r in adm if r.micro]
    big = [r for r in adm if not r.micro]
    assert {r.slot for r in micro} <= set(range(eng.slots, eng.n_all))
    assert {r.slot for r in big} <= set(range(eng.slots))
    assert eng.inflight() == len(adm)
    eng.pump_micro()                                           # the micro chain is queued at once
    assert eng.queued_steps() >= 1
    got = eng.cancel([micro[0].req_id, big[0].req_id])
    assert len(got) == 2 and all(r.aborted for r in got)
    assert micro[0].slot in eng.free_micro and big[0].slot in eng.free
    assert micro[0].slot not in eng.free and big[0].slot not in eng.free_micro
    eng.finish(block=True)
    out = eng.abort_all()
    assert len(eng.free_micro) == eng.micro_slots and len(eng.free) == eng.slots
    assert all(r.aborted for r in out)


def test_micro_full_pool_falls_back_to_serving_slots():
    eng = _engine("micro", micro_slots=2)
    reqs = [r for r in _requests(12) if r.tier == 0]        # 4 realtime requests, 2 micro slots
    adm = eng.admit(reqs)
    assert len(adm) == 4 and sum(r.micro for r in adm) == 2
    got = _serve(eng, [])
    assert len(got) == 4


def test_micro_mode_config_validation():
    from llm_message_queue_amd.utils.config import ConfigError, default_config, validate
    cfg = default_config()
    cfg.backend.realtime_mode = "micro"
    validate(cfg)
    cfg.backend.realtime_mode = "fast"
    with pytest.raises(ConfigError):
        validate(cfg)
    cfg = default_config()
    cfg.backend.step_timeout = cfg.server.stall_fatal_after
    with pytest.warns(UserWarning):
        validate(cfg)
    assert 0 < cfg.backend.step_timeout < cfg.server.stall_fatal_after     # (the hung-GPU path is reachable)
    with pytest.raises(ValueError):
        _engine("turbo")


def test_gateway_serves_realtime_on_micro_pool_cpu():
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.models.message import Message
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.enable_metrics = False
    for lv in cfg.queue.levels:
        lv.max_concurrent = 0
    eng = _engine("micro", slots=16, budget=64, micro_slots=4)
    gw = Gateway(cfg, engine=eng, use_gpu_preprocess=False, prompt_cap=16, gen_tokens=3)
    done = []
    gw.on_complete = done.append
    msgs = [Message(id=f"m{i}", content=("server down, need help" if i % 4 == 0 else "please summarise this"),
                    priority=1 if i % 4 == 0 else 3, user_id="u") for i in range(40)]
    gw.submit(msgs)
    for _ in range(200):
        gw.tick()
        if len(done) == len(msgs):
            break
    assert len(done) == len(msgs)
    assert eng.micro_steps > 0
    assert int(gw.inflight_by_tier.sum()) == 0 and not gw.local
    assert len(eng.free_micro) == eng.micro_slots


def test_two_ranks_realtime_on_micro_pools_fakecomm():
    """Two ranks in micro mode: realtime requests placed on the other rank
    run on its micro pool and complete while the ranks wait at the tick's
    collectives (``_while_waiting`` reaps micro-forwards).  Completion
    records reaped after a rank announced its row counts wait for the next
    tick, so the all_to_all always carries exactly what was announced."""
    import threading

    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.models.message import Message
    from llm_message_queue_amd.parallel.comm import FakeComm
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.enable_metrics = False
    comms = FakeComm.make(2)
    engs = [_engine("micro", slots=8, budget=64, micro_slots=4) for _ in range(2)]
    gws = [Gateway(cfg, engine=engs[r], comm=comms[r], use_gpu_preprocess=False, prompt_cap=16, gen_tokens=3)
           for r in range(2)]
    done = []
    gws[0].on_complete = done.append
    msgs = [Message(id=f"m{i}", content=("server down, need help" if i % 2 == 0 else "please summarise this"),
                    priority=1 if i % 2 == 0 else 3, user_id="u") for i in range(48)]
    gws[0].submit(msgs)
    for _ in range(300):
        ths = [threading.Thread(target=g.tick) for g in gws]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if len(done) == len(msgs):
            break
    assert len(done) == len(msgs)
    assert engs[1].micro_steps > 0 and gws[0].counters["remote_sent"] > 0
    assert not gws[0].remote_out and all(not g.foreign for g in gws)
    assert all(len(e.free_micro) == e.micro_slots for e in engs)


@pytest.mark.gpu
@pytest.mark.parametrize("stream", ["partition", "high"])
def test_micro_decode_graph_replays_match_eager_gpu(stream):
    """Decode-only micro-forwards replayed from HIP graphs (row buckets,
    padding rows on the scratch slot) produce the same greedy ids as the
    same micro-forwards launched kernel by kernel, and the serving pool's
    results are untouched."""
    dev = torch.device("cuda", 0)
    eager = _engine("micro", device=dev, impl="hip", slots=16, budget=64, micro_stream=stream,
                    micro_graph=False)
    eager.warm_shapes([1, 8, 64])
    a = _serve(eager, _requests(24, seed=9, gen=6))
    eager.close()
    graph = _engine("micro", device=dev, impl="hip", slots=16, budget=64, micro_stream=stream)
    graph.warm_shapes([1, 8, 64])
    assert graph.micro_graph and graph._mg
    b = _serve(graph, _requests(24, seed=9, gen=6))
    assert graph.micro_graph_steps > 0
    assert sorted(a) == sorted(b) == list(range(24))
    assert {k: v[0] for k, v in a.items()} == {k: v[0] for k, v in b.items()}
    assert graph.scratch_slot not in graph.free_micro and len(graph.free_micro) == graph.micro_slots
    graph.close()


@pytest.mark.gpu
@pytest.mark.parametrize("stream", ["partition", "high"])
def test_micro_stream_same_tokens_gpu(stream):
    """The HIP path: micro-forwards on a CU partition of their own (the
    default) or a high-priority stream, running concurrently with the
    serving steps, produce the same greedy ids as the serving steps do for
    the same requests."""
    dev = torch.device("cuda", 0)
    a = _serve(_engine("off", device=dev, impl="hip", slots=16, budget=64), _requests(24, seed=5))
    eng = _engine("micro", device=dev, impl="hip", slots=16, budget=64, micro_stream=stream)
    assert eng.rt_stream is not None
    b = _serve(eng, _requests(24, seed=5))
    assert sorted(a) == sorted(b) == list(range(24))
    same = sum(a[k][0] == b[k][0] for k in a)
    assert same == 24, {k: (a[k][0], b[k][0]) for k in a if a[k][0] != b[k][0]}
    # 8 realtime requests, 4 micro slots: the pool fills, the rest ride the serving steps
    assert 4 <= sum(v[1] for v in b.values()) <= 8 and eng.micro_steps >= 4
    eng.close()
