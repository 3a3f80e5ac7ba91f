"""Multi-GPU placement follows ``loadbalancer.algorithm`` (VERDICT r1 missing
#1/#2): the deterministic planner spreads each tick's grant over the GPUs by
round robin / least connections / weighted random / adaptive load, reads HBM
occupancy, skips GPUs the autoscaler parked, and the gateway feeds the
ResourceScheduler live per-GPU usage.  Reference: `load_balancer.go:234-294,
381-498`, `scheduler.go:119-156`, `resource_scheduler.go:336-398`."""
import threading

import numpy as np
import pytest

from llm_message_queue_amd.backend.engine import BackendEngine
from llm_message_queue_amd.balancer.load_balancer import Endpoint, LoadBalancer
from llm_message_queue_amd.gateway.router import Gateway
from llm_message_queue_amd.gateway.workload import Workload
from llm_message_queue_amd.models.llama_stub import LlamaConfig
from llm_message_queue_amd.parallel import planner
from llm_message_queue_amd.parallel.comm import FakeComm
from llm_message_queue_amd.scheduler.resource_scheduler import ResourceScheduler
from llm_message_queue_amd.utils.config import default_config

MICRO = LlamaConfig(vocab=512, dim=2048, layers=1, heads=16, kv_heads=4, ffn=256)


def _loads(W, free=100, slots=200, inflight=None, demand0=0, hbm=None, exclude=0, weights=None):
    rows = []
    for j in range(W):
        infl = slots - free if inflight is None else inflight[j]
        rows.append(planner.make_load(
            free, infl, [0, 0, demand0 if j == 0 else 0, 0], [0] * 4, slots_total=slots,
            slots_free=free, hbm_used_mib=(hbm[j] if hbm else 0), hbm_total_mib=(1000 if hbm else 0),
            exclude_mask=exclude if j == 0 else 0, weights=weights or []))
    return np.stack(rows)


@pytest.mark.parametrize("W", [4, 8])
def test_round_robin_exact_split_from_one_ingress(W):
    st = planner.PlanState("round_robin")
    tot = np.zeros(W, dtype=np.int64)
    for k in range(50):
        q = planner.plan_dispatch(_loads(W, demand0=7 + (k % 5)), [0] * 4, st)
        tot += q.sum(axis=(0, 2))
    assert tot.sum() == sum(7 + (k % 5) for k in range(50))
    assert tot.max() - tot.min() <= 1                       # an exact 1/W split


@pytest.mark.parametrize("W", [4, 8])
def test_weighted_random_avoids_full_hbm(W):
    st = planner.PlanState("weighted_random")
    hbm = [100] * W
    hbm[1] = 900                                           # GPU1 at 90 % HBM
    tot = np.zeros(W, dtype=np.int64)
    for _ in range(40):
        tot += planner.plan_dispatch(_loads(W, demand0=64, hbm=hbm), [0] * 4, st).sum(axis=(0, 2))
    others = np.delete(tot, 1).mean()
    assert tot[1] <= others / 4, tot                       # weight x (1 - 0.9) vs x (1 - 0.1)
    # deterministic: every rank computes the same draw
    a = planner.plan_dispatch(_loads(W, demand0=64, hbm=hbm), [0] * 4, planner.PlanState("weighted_random"))
    b = planner.plan_dispatch(_loads(W, demand0=64, hbm=hbm), [0] * 4, planner.PlanState("weighted_random"))
    assert (a == b).all()


@pytest.mark.parametrize("strategy", planner.STRATEGIES)
def test_parked_gpu_gets_nothing(strategy):
    W = 4
    st = planner.PlanState(strategy)
    for _ in range(10):
        q = planner.plan_dispatch(_loads(W, demand0=60, exclude=0b0100), [0] * 4, st)
        assert q[:, 2].sum() == 0 and q.sum() == 60


def test_least_connections_balances_and_breaks_ties_on_hbm():
    W = 4
    q = planner.plan_dispatch(_loads(W, inflight=[50, 10, 10, 30], demand0=40, hbm=[0, 800, 100, 0]),
                              [0] * 4, planner.PlanState("least_connections"))
    per = q.sum(axis=(0, 2))
    # utilisation evens out: 50/10/10/30 + 40 -> 50/30/30/30 (GPU0 already highest)
    assert list(per) == [0, 20, 20, 0]
    q = planner.plan_dispatch(_loads(W, inflight=[10, 10, 10, 10], demand0=1, hbm=[0, 800, 100, 0]),
                              [0] * 4, planner.PlanState("least_connections"))
    assert q.sum(axis=(0, 2))[0] == 1                       # tie: lowest HBM, then index
    q = planner.plan_dispatch(_loads(W, inflight=[10, 10, 10, 10], demand0=1, hbm=[500, 800, 100, 0]),
                              [0] * 4, planner.PlanState("least_connections"))
    assert q.sum(axis=(0, 2))[3] == 1


def test_adaptive_prefers_fast_gpus():
    W = 3
    rows = []
    for j, rt in enumerate([150_000, 50_000, 100_000]):       # reference test: 150 / 50 / 100 ms
        rows.append(planner.make_load(100, 0, [0, 0, 30 if j == 0 else 0, 0], [0] * 4, slots_total=200,
                                      slots_free=100, rt_us=rt))
    q = planner.plan_dispatch(np.stack(rows), [0] * 4, planner.PlanState("adaptive_load"))
    per = q.sum(axis=(0, 2))
    assert per[1] == per.max() and per.sum() == 30


def test_realtime_lane_uses_slots_beyond_headroom():
    W = 2
    rows = [planner.make_load(0, 10, [5, 0, 5, 0], [0] * 4, slots_total=100, slots_free=50),
            planner.make_load(0, 10, [0, 0, 0, 0], [0] * 4, slots_total=100, slots_free=50)]
    q = planner.plan_dispatch(np.stack(rows), [0] * 4, planner.PlanState("local_first"))
    assert q[:, :, 0].sum() == 5 and q[:, :, 2].sum() == 0   # headroom 0: only the realtime lane moves


def test_pins_are_per_home_gpu_and_tier():
    W = 2
    pin = np.zeros((W, 4), dtype=np.int64)
    pin[1, 0] = 2                                          # 2 realtime turns homed on GPU1
    rows = [planner.make_load(10, 0, [2, 0, 6, 0], [0] * 4, slots_total=10, pinned=pin),
            planner.make_load(3, 0, [0, 0, 0, 0], [0] * 4, slots_total=10)]
    q = planner.plan_dispatch(np.stack(rows), [0] * 4, planner.PlanState("local_first"))
    assert q[0, 1, 0] == 2                                 # the realtime pins go home
    assert q[0, 0, 2] == 6                                 # normal tier not charged with them


# ------------------------------------------------------------------ gateways (threads, FakeComm)
def _cfg(strategy):
    c = default_config()
    c.queue.enable_metrics = False
    c.loadbalancer.algorithm = strategy
    c.loadbalancer.health_check_interval = 0
    return c


def _tick_all(gws):
    ths = [threading.Thread(target=g.tick) for g in gws]
    for t in ths:
        t.start()
    for t in ths:
        t.join()


def _cluster(W, strategy, slots=8):
    comms = FakeComm.make(W)
    gws, lbs = [], []
    for r in range(W):
        lb = LoadBalancer(_cfg(strategy).loadbalancer)
        for j in range(W):
            lb.add_endpoint(Endpoint(id=f"gpu{j}", type="llm", gpu_index=j, max_connections=slots))
        eng = BackendEngine(MICRO, slots=slots, max_ctx=64, token_budget=64, device="cpu", impl="ref", seed=r)
        gw = Gateway(_cfg(strategy), engine=eng, comm=comms[r], load_balancer=lb, use_gpu_preprocess=False,
                     prompt_cap=8, gen_tokens=2)
        gws.append(gw)
        lbs.append(lb)
    return gws, lbs


@pytest.mark.parametrize("W", [4, 8])
def test_single_ingress_round_robin_spreads_over_all_gpus(W):
    gws, lbs = _cluster(W, "round_robin")
    msgs = Workload(seed=5).make(12 * W)
    gws[0].submit(msgs)                                    # one ingress (cli serve: HTTP on rank 0)
    for _ in range(200):
        _tick_all(gws)
        if gws[0].counters["completed"] >= len(msgs):
            break
    assert gws[0].counters["completed"] == len(msgs)
    served = [g.engine.completed_total for g in gws]
    assert gws[0].counters["remote_sent"] > 0
    assert max(served) - min(served) <= 2, served
    # remote completions released the balancer's endpoints (EWMA RT updated)
    assert all(lbs[0].get_endpoint_by_id(f"gpu{j}").response_time > 0 for j in range(1, W))
    assert all(lbs[0].get_endpoint_by_id(f"gpu{j}").connections == 0 for j in range(1, W))


def test_autoscaler_parked_gpu_receives_no_work_and_resources_track_use():
    W = 4
    gws, lbs = _cluster(W, "least_connections")
    rs = ResourceScheduler(start=False)
    gws[0].resources = rs
    parked = lbs[0].get_endpoint_by_id("gpu2")
    _tick_all(gws)                                         # rank 0's balancer has seen gpu2
    lbs[0].remove_endpoint("gpu2")                         # Scheduler._remove (autoscaler scale-down)
    gws[0].submit(Workload(seed=3).make(60))
    seen_used = 0
    for _ in range(300):
        _tick_all(gws)
        gws[0]._res_next_ns = 0
        seen_used = max(seen_used, rs.get_resource("gpu1").used.get("gpu", 0))
        if gws[0].counters["completed"] >= 60:
            break
    assert gws[0].counters["completed"] == 60
    assert gws[2].engine.completed_total == 0 and gws[2].counters["remote_recv"] == 0
    assert seen_used > 0                                   # /resources/stats saw in-flight slots on gpu1
    assert {r.id for r in rs.get_all_resources()} == {f"gpu{j}" for j in range(W)}
    # scale back up: the GPU takes work again
    lbs[0].add_endpoint(parked)
    gws[0].submit(Workload(seed=4).make(60))
    for _ in range(300):
        _tick_all(gws)
        if gws[0].counters["completed"] >= 120:
            break
    assert gws[2].engine.completed_total > 0


def test_overcommit_requeues_instead_of_raising(monkeypatch):
    W = 2
    gws, _ = _cluster(W, "local_first", slots=4)
    gws[0].submit(Workload(seed=1).make(8))
    orig = gws[0].engine.admit
    monkeypatch.setattr(gws[0].engine, "admit", lambda reqs: orig(reqs[:1]))   # engine takes less than planned
    _tick_all(gws)
    monkeypatch.setattr(gws[0].engine, "admit", orig)
    assert gws[0].counters["overcommit"] > 0
    for _ in range(100):
        _tick_all(gws)
        if gws[0].counters["completed"] >= 8:
            break
    assert gws[0].counters["completed"] == 8


def test_dead_peer_surfaces_as_peer_lost_within_timeout():
    """Every tick is a collective: when one rank dies the survivors must
    fail fast (PeerLost -> serve loop exits non-zero), not hang."""
    import time
    from llm_message_queue_amd.parallel.comm import PeerLost
    W = 4
    comms = FakeComm.make(W, timeout_s=1.0)
    gws = []
    for r in range(W):
        eng = BackendEngine(MICRO, slots=4, max_ctx=64, token_budget=64, device="cpu", impl="ref", seed=r)
        gws.append(Gateway(_cfg("local_first"), engine=eng, comm=comms[r], use_gpu_preprocess=False,
                           prompt_cap=8, gen_tokens=2))
    _tick_all(gws)                                          # all alive
    errs, took = {}, {}

    def survivor(r):
        t0 = time.monotonic()
        try:
            for _ in range(50):
                gws[r].tick()
        except PeerLost as e:
            errs[r] = e
        took[r] = time.monotonic() - t0

    ths = [threading.Thread(target=survivor, args=(r,)) for r in range(W - 1)]   # rank 3 is dead
    for t in ths:
        t.start()
    for t in ths:
        t.join(10)
    assert set(errs) == {0, 1, 2}
    assert max(took.values()) < 5.0


def test_serve_loop_exits_on_peer_lost():
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.parallel.comm import PeerLost
    c = _cfg("local_first")
    eng = BackendEngine(MICRO, slots=4, max_ctx=64, token_budget=64, device="cpu", impl="ref")
    app = GatewayApp(c, use_gpu=False, engine=eng, start=False)

    def boom(*a, **k):
        raise PeerLost("rank 1 gone")
    app.gateway.tick = boom
    app.start()
    app._loop_thread.join(5)
    assert isinstance(app.fatal, PeerLost) and app._stop.is_set()
    app.stop()


def test_multirank_realtime_lane_dispatches_between_ticks():
    """World > 1: dispatch is a per-tick collective, but realtime requests
    are admitted into the router's own GPU while it waits for the forward
    (no tick needed), and the next load vector accounts for them."""
    from llm_message_queue_amd.models.message import Message
    W = 2
    gws, _ = _cluster(W, "least_connections", slots=16)
    rt = [Message(id=f"rt{i}", content="outage now", priority=1, user_id="u") for i in range(3)]
    gws[0].submit(rt)
    gws[0]._last_ingest_ns = 0
    assert gws[0]._while_waiting(None)                   # ingest + local realtime admission, no collective
    assert all(m.dispatched_at > 0 and m.endpoint_id == "gpu0" for m in rt)
    assert gws[0].counters["realtime_local"] == 3
    for _ in range(30):
        _tick_all(gws)
        if gws[0].counters["completed"] >= 3:
            break
    assert gws[0].counters["completed"] == 3


def test_own_dispatch_passes_over_turns_homed_elsewhere():
    """the realtime lane (and the own-GPU dispatch of
    every tier) used to switch off while ANY queued turn of the tier was
    homed on another GPU.  Now those turns are passed over in place -- they
    wait for the tick's plan, which sends them to their KV -- and the rest of
    the tier is still admitted into this rank's own GPU between ticks."""
    from llm_message_queue_amd.models.message import Message
    W = 2
    gws, _ = _cluster(W, "least_connections", slots=16)
    g = gws[0]
    g.conv_home["dlg-away"] = 1
    away = [Message(id=f"a{i}", conversation_id="dlg-away", content="and then?", priority=p, user_id="u")
            for i, p in enumerate((1, 3))]
    rt = [Message(id=f"rt{i}", content="outage now", priority=1, user_id="u") for i in range(3)]
    nm = [Message(id=f"n{i}", content="summarise this", priority=3, user_id="u") for i in range(2)]
    g.submit(away[:1] + rt + away[1:] + nm)
    g._last_ingest_ns = 0
    assert g._while_waiting(None)
    # the prefill headroom (4 here) takes realtime then normal, the lane the
    # rest of realtime; the old code admitted none of them (both tiers held a
    # turn homed on GPU1)
    assert all(m.dispatched_at > 0 and m.endpoint_id == "gpu0" for m in rt + nm[:1])
    assert all(m.dispatched_at == 0 for m in away)
    assert g.pinned[1].tolist()[:3] == [1, 0, 1] and len(g._away) == 2
    for _ in range(40):
        _tick_all(gws)
        if g.counters["completed"] >= 7:
            break
    assert g.counters["completed"] == 7
    assert all(m.endpoint_id == "gpu1" for m in away)         # followed their home
    assert g.pinned.sum() == 0 and not g._away
