"""Multi-rank ticks with GPUs of different speed (SimEngine: the engine's host
side for real, the forward as a simulated device clock; FakeComm ranks in
threads).

Every tick is one collective, so under pure lock-step a faster GPU idles for
the speed difference every tick and the job serves N x its SLOWEST GPU.  With
``gpu.extra_steps`` a rank whose run-ahead queue has room while a peer is
still behind launches one extra forward from its own queue
(``Gateway._extra_local_step``), so the job approaches the SUM of its GPUs'
capacities (bench.py ``--sim-gpu`` measures it at 8 ranks)."""
import threading
import time

import numpy as np

from llm_message_queue_amd.backend.engine import Request
from llm_message_queue_amd.backend.sim_engine import SimEngine
from llm_message_queue_amd.gateway.router import Gateway
from llm_message_queue_amd.gateway.workload import Workload
from llm_message_queue_amd.parallel.comm import FakeComm
from llm_message_queue_amd.utils.config import default_config


def test_sim_engine_clock():
    """Steps run back to back on the simulated device at step_ms(T) / speed
    (tile-quantised), completion events fire at their end time, the run-ahead
    queue bounds the host like a real GPU's."""
    e = SimEngine(speed=2.0, tile_ms=4.0, base_ms=2.0, slots=64, token_budget=512)
    assert e.step_ms(1) == 3.0 and e.step_ms(256) == 3.0 and e.step_ms(257) == 5.0
    e.time_steps = True
    e.admit([Request(req_id=i, prompt=np.arange(20, dtype=np.int32), gen_tokens=3) for i in range(40)])
    assert e.ready_tokens() == 512                     # 800 prompt tokens pending, capped at the budget
    t0 = time.monotonic()
    e.launch()
    e.launch()
    assert e.queued_steps() == 2                       # asynchronous: nothing finished yet
    e.launch()                                         # queue full: waits for the oldest step
    e.finish(block=True)
    wall = (time.monotonic() - t0) * 1e3
    # T = 512 (prefill), 313 (25 decodes + the last 288 prompt tokens), 40
    # decodes: 2, 2 and 1 tiles -> 5 + 5 + 3 ms at speed 2
    assert e.gpu_steps == 3 and abs(e.gpu_step_ms - 13.0) < 1e-6
    assert wall >= 12.5                                # the three steps ran back to back
    assert e.completed_total == 25 and e.step_id == 3   # completions count at launch (the last token's step)


def _cfg(extra: bool):
    c = default_config()
    c.queue.enable_metrics = False
    c.loadbalancer.algorithm = "least_connections"
    c.loadbalancer.health_check_interval = 0
    c.gpu.extra_steps = extra
    for lv in c.queue.levels:
        lv.max_concurrent = 4096
    return c


def _run(extra: bool, ticks: int = 40):
    W = 2
    # virtual time: the simulated GPUs and the "is my
    # peer behind?" question run on per-rank VirtualClocks, so the outcome
    # depends on the simulated speeds only, not on how the OS schedules the
    # two threads (the wall-clock version failed on a loaded host)
    comms = FakeComm.make(W, timeout_s=60, virtual=True)
    speeds = [1.0, 0.6]
    gws = [Gateway(_cfg(extra), engine=SimEngine(speed=speeds[r], tile_ms=2.0, base_ms=1.0, slots=256,
                                                 token_budget=1024, clock=comms[r].clock),
                   comm=comms[r], use_gpu_preprocess=False, prompt_cap=16, gen_tokens=2) for r in range(W)]
    wls = [Workload(seed=r) for r in range(W)]

    def loop(r):
        g = gws[r]
        for _ in range(ticks):
            need = 512 - g.pending() - g.engine.inflight()
            if need > 0:
                g.submit(wls[r].make(need))      # saturated: every rank keeps a local backlog
            g.tick()

    ths = [threading.Thread(target=loop, args=(r,)) for r in range(W)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return gws


def test_faster_gpu_takes_extra_steps_and_job_serves_more():
    on = _run(True)
    off = _run(False)
    # pure lock-step: one forward per tick on every rank
    assert all(g.engine.step_id <= g.counters["ticks"] for g in off)   # (the first tick has nothing yet)
    assert all(g.counters["extra_steps"] == 0 for g in off)
    # the fast rank (speed 1.0 vs 0.6) fills its idle time with extra forwards;
    # the slow one is ahead of its peer only in transients
    fast, slow = on
    assert fast.counters["extra_steps"] >= 10, fast.counters
    assert fast.engine.step_id > fast.counters["ticks"]
    # in simulated time the slow GPU is never ahead of the fast one
    assert slow.counters["extra_steps"] == 0, (slow.counters, fast.counters)
    # more tokens through the job in the same number of ticks
    assert sum(g.engine.total_tokens for g in on) > 1.15 * sum(g.engine.total_tokens for g in off)


def test_virtual_time_runs_are_reproducible():
    """The same virtual-time run twice: identical counters, steps, tokens --
    nothing depends on thread scheduling."""
    a, b = _run(True, ticks=25), _run(True, ticks=25)
    for ga, gb in zip(a, b):
        assert ga.counters["extra_steps"] == gb.counters["extra_steps"]
        assert ga.engine.step_id == gb.engine.step_id and ga.engine.total_tokens == gb.engine.total_tokens


def test_extra_steps_skip_a_parked_gpu():
    """A GPU the autoscaler parked takes no new local work in extra steps."""
    c = _cfg(True)
    comms = FakeComm.make(2, timeout_s=30)
    g = Gateway(c, engine=SimEngine(slots=64, token_budget=256), comm=comms[0], use_gpu_preprocess=False,
                prompt_cap=16, gen_tokens=2)
    g._exclude_mask = lambda: 1                            # rank 0's own GPU excluded
    g.submit(Workload(seed=1).make(64))
    g.ingest()
    assert g.pending() > 0
    assert comms[0].peers_behind()                         # rank 1 has not reached the exchange
    assert g._extra_local_step() is False
    assert g.counters["extra_admitted"] == 0 and g.engine.step_id == 0
    g._exclude_mask = lambda: 0                            # back in placement: the extra step runs
    assert g._extra_local_step() is True
    assert g.counters["extra_admitted"] > 0 and g.engine.step_id == 1


def test_extra_step_backend_error_evacuates_instead_of_raising():
    """A HIP error in the extra forward takes the GPU out of placement (its
    admitted requests go back to the queue) like an error in the tick's own
    launch -- the tick does not raise."""
    comms = FakeComm.make(2, timeout_s=30)
    g = Gateway(_cfg(True), engine=SimEngine(slots=64, token_budget=256), comm=comms[0], use_gpu_preprocess=False,
                prompt_cap=16, gen_tokens=2)
    g.submit(Workload(seed=2).make(64))
    g.ingest()
    queued = g.pending()
    g.engine.inject(fail_launch=1)
    assert g._extra_local_step() is False
    assert not g.healthy and "injected" in g.health_reason
    assert g.counters["extra_admitted"] > 0 and g.counters["evacuated"] == g.counters["extra_admitted"]
    assert g.pending() == queued                          # every admitted request is queued again


def test_extra_steps_with_dialogs_and_rehoming_lose_nothing():
    """Extra local steps alongside conversation residency and KV migration:
    two simulated GPUs of different speed serve dialogs; midway the slow GPU
    is parked on rank 0's balancer, so its dialogs' next turns re-home (KV
    migration).  Every submitted message completes exactly once."""
    from llm_message_queue_amd.balancer.load_balancer import Endpoint, LoadBalancer
    W = 2
    comms = FakeComm.make(W, timeout_s=60)
    lbs = []
    gws = []
    for r in range(W):
        cfg = _cfg(True)
        lb = LoadBalancer(cfg.loadbalancer)
        for j in range(W):
            lb.add_endpoint(Endpoint(id=f"gpu{j}", type="llm", gpu_index=j, max_connections=128))
        lbs.append(lb)
        gws.append(Gateway(cfg, engine=SimEngine(speed=[1.0, 0.6][r], tile_ms=2.0, base_ms=1.0, slots=128,
                                                 max_ctx=256, token_budget=512),
                           comm=comms[r], load_balancer=lb, use_gpu_preprocess=False, prompt_cap=16, gen_tokens=2))
    wls = [Workload(seed=40 + r, conversations=12) for r in range(W)]
    submitted = [0, 0]

    def loop(r, ticks, feed):
        g = gws[r]
        for t in range(ticks):
            if feed and t < 50 and g.pending() < 200:
                batch = wls[r].make(24)
                g.submit(batch)
                submitted[r] += len(batch)
            if r == 0 and feed and t == 25:
                lbs[0].remove_endpoint("gpu1")            # park the slow GPU: its dialogs re-home
            g.tick()

    ths = [threading.Thread(target=loop, args=(r, 90, True)) for r in range(W)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    done = lambda: sum(g.counters["completed"] for g in gws)
    for _ in range(40):
        if done() >= sum(submitted):
            break
        ths = [threading.Thread(target=loop, args=(r, 10, False)) for r in range(W)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
    assert done() == sum(submitted), (done(), submitted, [g.counters for g in gws])
    assert gws[0].counters["extra_steps"] > 0
    moved = sum(g.counters["kv_migrated"] + g.counters["kv_migrate_replays"] for g in gws)
    assert moved > 0, [g.counters for g in gws]
