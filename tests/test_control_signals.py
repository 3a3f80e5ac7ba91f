"""Control-plane signals that act (VERDICT r2 missing #4):

* live HBM occupancy: a GPU's published footprint is weights + RESIDENT KV
  (active contexts + parked dialogs), so a GPU whose parked dialogs fill its
  KV pool draws less new work under the weighted-random placement (reference
  endpoints carry load state, `internal/loadbalancer/load_balancer.go:35-49`);
* the ResourceScheduler heartbeats KV tokens for every GPU and its autoscale
  decisions park / unpark GPU endpoints (`resource_scheduler.go:525-571`
  only logs);
* pins are released under the key they were counted with;
* a KV migration whose destination went unhealthy between the order tick and
  the execute tick leaves no unmatched send behind.
CPU engines on the reference ops; FakeComm ranks in threads."""
import threading

import numpy as np

from llm_message_queue_amd.backend.engine import BackendEngine
from llm_message_queue_amd.balancer.load_balancer import Endpoint, LoadBalancer
from llm_message_queue_amd.gateway.router import Gateway, conv_key
from llm_message_queue_amd.gateway.workload import Workload
from llm_message_queue_amd.models.llama_stub import LlamaConfig
from llm_message_queue_amd.models.message import Message
from llm_message_queue_amd.parallel import planner
from llm_message_queue_amd.parallel.comm import FakeComm
from llm_message_queue_amd.scheduler.resource_scheduler import (ResourceRequest, ResourceScheduler,
                                                                 ResourceSchedulerConfig, RequestQueued)
from llm_message_queue_amd.utils.config import default_config

MICRO = LlamaConfig(vocab=512, dim=2048, layers=1, heads=16, kv_heads=4, ffn=256)


def _cfg(strategy="least_connections"):
    c = default_config()
    c.queue.enable_metrics = False
    c.loadbalancer.algorithm = strategy
    c.loadbalancer.health_check_interval = 0
    return c


def _lb(W, slots):
    lb = LoadBalancer(_cfg().loadbalancer)
    for j in range(W):
        lb.add_endpoint(Endpoint(id=f"gpu{j}", type="llm", gpu_index=j, max_connections=slots))
    return lb


def _tick_all(gws):
    ths = [threading.Thread(target=g.tick) for g in gws]
    for t in ths:
        t.start()
    for t in ths:
        t.join()


def test_engine_reports_resident_kv():
    e = BackendEngine(MICRO, slots=8, max_ctx=64, token_budget=64, device="cpu", impl="ref", seed=1)
    assert e.resident_kv_tokens() == 0 and e.kv_token_capacity() == 8 * 64
    e.import_kv(11, 40)
    e.import_kv(12, 24)
    assert e.resident_kv_tokens() == 64
    assert e.kv_bytes_per_token() == MICRO.layers * 2 * MICRO.kv_heads * MICRO.head_dim * 2


def test_parked_kv_steers_weighted_random_placement():
    """World 8: GPU 3's parked dialogs fill ~90 % of its KV pool.  Its
    published footprint rises with them, and weighted_random gives it at most
    a quarter of a fair share of one router's traffic."""
    W, slots, ctx = 8, 64, 512
    comms = FakeComm.make(W)
    gws = [Gateway(_cfg("weighted_random"), engine=BackendEngine(MICRO, slots=slots, max_ctx=ctx, token_budget=256,
                                                                  device="cpu", impl="ref", seed=r),
                   comm=comms[r], use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2) for r in range(W)]
    full = gws[3].engine
    for c in range(58):
        full.import_kv(1000 + c, ctx)                     # 58 x 512 of 64 x 512 positions parked
    loads = np.stack([g._my_load() for g in gws])
    assert loads[3, planner.L_KV_TOKENS] == 58 * ctx and loads[3, planner.L_KV_CAP] == slots * ctx
    frac = loads[:, planner.L_HBM_USED] / loads[:, planner.L_HBM_TOTAL]
    assert frac[3] > 0.85 and (np.delete(frac, 3) < 0.5).all(), frac
    st = planner.PlanState("weighted_random")
    tot = np.zeros(W, dtype=np.int64)
    for _ in range(40):
        ld = loads.copy()
        ld[0, planner.L_DEPTH + 2] = 64                   # router 0: 64 normal-tier requests per tick
        tot += planner.plan_dispatch(ld, [0] * 4, st).sum(axis=(0, 2))
    fair = tot.sum() / W
    assert tot[3] <= fair / 4, tot


def test_resource_scheduler_heartbeats_kv_tokens_for_every_gpu():
    W = 2
    comms = FakeComm.make(W)
    gws = [Gateway(_cfg(), engine=BackendEngine(MICRO, slots=8, max_ctx=1024, token_budget=64, device="cpu",
                                               impl="ref", seed=r), comm=comms[r], use_gpu_preprocess=False,
                   prompt_cap=8, gen_tokens=2, load_balancer=_lb(W, 8)) for r in range(W)]
    rs = ResourceScheduler(start=False)
    gws[0].attach_resource_scheduler(rs, act=False)
    gws[1].engine.import_kv(77, 1000)
    _tick_all(gws)
    r1 = rs.get_resource("gpu1")
    assert r1.capacity["tokens"] == 8 * 1024 and r1.used["tokens"] == 1000
    assert rs.get_resource("gpu0").used["tokens"] == 0
    assert r1.used["memory"] > rs.get_resource("gpu0").used["memory"]


def _serve(gws, origin, n, ticks=80):
    gws[origin].submit(Workload(seed=5).make(n))
    want = gws[origin].counters["completed"] + n
    for _ in range(ticks):
        _tick_all(gws)
        if gws[origin].counters["completed"] >= want:
            return True
    return False


def test_resource_scheduler_scale_down_parks_a_gpu_and_scale_up_returns_it():
    W, slots = 8, 16
    comms = FakeComm.make(W, timeout_s=30)
    # KV pool large against the weights (as on the GPU: 96 GiB vs 16 GB), so
    # an idle job's resource load is low
    gws = [Gateway(_cfg("round_robin"), engine=BackendEngine(MICRO, slots=slots, max_ctx=2048, token_budget=64,
                                                              device="cpu", impl="ref", seed=r),
                   comm=comms[r], use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2,
                   load_balancer=_lb(W, slots)) for r in range(W)]
    rs = ResourceScheduler(ResourceSchedulerConfig(enable_auto_scaling=True, scale_cooldown=0, min_resources=1,
                                                   max_resources=W), start=False)
    gws[0].attach_resource_scheduler(rs, act=True)
    _tick_all(gws)                                         # every GPU heartbeated into rank 0's scheduler
    assert len(rs.get_all_resources()) == W
    assert rs.check_auto_scaling() == "scale_down"         # idle job
    assert rs.parked == ["gpu7"]                           # least loaded; ties -> highest id
    before = gws[7].engine.completed_total
    assert _serve(gws, 0, 48)
    assert gws[7].engine.completed_total == before         # parked: the planner sent it nothing
    assert all(g.engine.completed_total > 0 for g in gws[:7])
    # a request the pool cannot satisfy waits in the pending queue -> scale up
    try:
        rs.request_resource(ResourceRequest("big", "llm", {"gpu": 10 ** 6}))
    except RequestQueued:
        pass
    assert rs.check_auto_scaling() == "scale_up" and rs.parked == []
    assert _serve(gws, 0, 48)
    assert gws[7].engine.completed_total > before          # back in placement


def test_pin_released_under_the_key_it_was_counted():
    """a queued turn's pin is counted under its home at
    enqueue time; if the conversation is re-homed while it waits, the pop
    must release that same key (the old code decremented the new home and
    left the old one inflated for good)."""
    comms = FakeComm.make(2)
    gw = Gateway(_cfg(), engine=None, comm=comms[0], use_gpu_preprocess=False)
    m = Message(id="x", conversation_id="dlg", content="hi", priority=3)
    gw.conv_home["dlg"] = 1
    m.queue_name = "normal"
    gw._pin(m, +1)
    assert gw.pinned[1].sum() == 1
    gw.conv_home["dlg"] = 0                               # re-homed (migration) while queued
    gw._pin(m, -1)
    assert gw.pinned.sum() == 0
    gw._pin(m, -1)                                        # idempotent
    assert gw.pinned.sum() == 0


def test_migration_to_a_destination_that_went_unhealthy_leaves_no_mail():
    """the order is decided in tick t, executed in t+1.
    If the destination turns unhealthy in between (its held turn is handed
    back), the home must not send: the header exchange only matches a
    transfer that both sides still want.  The turn is re-placed and served;
    no unmatched message stays in any mailbox."""
    W = 3
    comms = FakeComm.make(W, timeout_s=30)
    lbs = [_lb(W, 4) for _ in range(W)]
    gws = [Gateway(_cfg("least_connections"), engine=BackendEngine(MICRO, slots=4, max_ctx=64, token_budget=64,
                                                                    device="cpu", impl="ref", seed=7),
                   comm=comms[r], load_balancer=lbs[r], use_gpu_preprocess=False, prompt_cap=12, gen_tokens=2)
           for r in range(W)]
    turn = lambda i: Message(id=f"t{i}", conversation_id="dlg-x", user_id="u", content="tell me more", priority=3)
    gws[0].submit([turn(1)])
    for _ in range(40):
        _tick_all(gws)
        if gws[0].counters["completed"] >= 1:
            break
    home = gws[0].conv_home["dlg-x"]
    assert gws[home].engine.export_kv(conv_key("dlg-x"))[1] > 0
    lbs[0].remove_endpoint(f"gpu{home}")                  # park the home: the next turn must move
    gws[0].submit([turn(2)])
    flipped = None
    for _ in range(60):
        _tick_all(gws)
        if flipped is None:
            for r, g in enumerate(gws):
                if g._await_kv:                           # order decided, not yet executed
                    g.set_healthy(False, "test: destination lost")
                    flipped = r
        if gws[0].counters["completed"] >= 2:
            break
    assert flipped is not None and flipped != home
    assert gws[0].counters["completed"] == 2
    assert all(not v for v in comms[0].hub.mail.values()), comms[0].hub.mail
    # the KV is still parked at the home or moved once to the third GPU, never lost to the dead one
    assert gws[flipped].engine.kv_imported == 0


def test_every_removal_of_a_queued_turn_releases_its_pin():
    """a queued conversation turn is counted once under
    its (home GPU, tier) pin.  Admin delete, a peer's remove / dequeue and
    retention cleanup take it out of the queue without a dispatch; each must
    release the pin, or the planner (and the extra-step guard, which skips a
    tier with turns homed elsewhere) reads a phantom turn for good."""
    from llm_message_queue_amd.gateway.app import GatewayApp
    comms = FakeComm.make(2)
    cfg = _cfg()
    cfg.queue.worker.process_interval = 5_000_000
    app = GatewayApp(cfg, use_gpu=False, comm=comms[0], start=False)
    gw = app.gateway
    assert gw.world == 2

    def queued(mid):
        m = Message(id=mid, conversation_id="dlg-" + mid, content="hi", priority=3, metadata={"home_gpu": 1})
        m.queue_name = "normal"
        assert gw._enqueue([m])[0][1] is None
        app.messages.put(m)
        return m

    queued("a")
    assert gw.pinned[1].sum() == 1
    assert app.peer_op("remove", ["a"]) == {"dequeued": True, "cancelled": False}   # peer 'remove'
    assert gw.pinned.sum() == 0
    queued("b")
    assert app.peer_op("dequeue", ["standard", "b"]) is True            # peer 'dequeue'
    assert gw.pinned.sum() == 0
    queued("c")
    from fastapi.testclient import TestClient
    from llm_message_queue_amd.api.server import create_app
    with TestClient(create_app(app)) as c:                               # local DELETE route
        r = c.delete("/api/v1/messages/c")
        assert r.status_code == 200 and r.json()["dequeued"] is True
    assert gw.pinned.sum() == 0
    m = queued("d")                                                      # retention cleanup
    m.enqueued_at = 1
    app.standard.config.max_retention_period = 1
    assert app.standard.cleanup_stale_messages() == 1
    assert gw.pinned.sum() == 0
    app.stop()


def test_pin_bookkeeping_is_thread_safe():
    """Admin deletes and peer dequeues release pins from other threads
    (``qm.on_remove``) while the serve loop reads the homed-away set for
    its own-GPU pops: no torn update, no 'set changed size' in the loop."""
    import threading
    comms = FakeComm.make(2)
    gw = Gateway(_cfg(), engine=None, comm=comms[0], use_gpu_preprocess=False)
    gw.conv_home["far"] = 1
    msgs = [Message(id=f"x{i}", conversation_id="far", content="hi", priority=3) for i in range(400)]
    for m in msgs:
        m.queue_name = "normal"
    stop = threading.Event()
    errs = []

    def churn(part):
        try:
            for _ in range(20):
                for m in part:
                    gw._pin(m, +1)
                for m in part:
                    gw._pin(m, -1)
        except Exception as e:          # noqa: BLE001
            errs.append(e)

    def reader():
        try:
            while not stop.is_set():
                gw._skip_away()
        except Exception as e:          # noqa: BLE001
            errs.append(e)

    r = threading.Thread(target=reader)
    r.start()
    ths = [threading.Thread(target=churn, args=(msgs[i::4],)) for i in range(4)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    stop.set()
    r.join()
    assert not errs
    assert gw.pinned.sum() == 0 and not gw._away
