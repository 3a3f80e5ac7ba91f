"""Gateway data path on CPU (reference-op engine), the deterministic RCCL
planner, and multi-rank dispatch: threads with FakeComm (world 2/4/8) and
real torch.distributed gloo processes (world 2)."""
import os
import socket
import threading

import numpy as np
import pytest
import torch

from llm_message_queue_amd.backend.engine import BackendEngine
from llm_message_queue_amd.gateway.router import Gateway, LatencyRecorder, hist_percentile
from llm_message_queue_amd.gateway.workload import PoissonArrivals, Workload
from llm_message_queue_amd.models.llama_stub import LlamaConfig
from llm_message_queue_amd.parallel import planner
from llm_message_queue_amd.parallel.comm import FakeComm, SoloComm
from llm_message_queue_amd.utils.config import default_config

MICRO = LlamaConfig(vocab=512, dim=2048, layers=1, heads=16, kv_heads=4, ffn=256)


def cfg():
    c = default_config()
    c.queue.enable_metrics = False
    return c


def engine(slots=8, seed=0, token_budget=64):
    return BackendEngine(MICRO, slots=slots, max_ctx=64, token_budget=token_budget, device="cpu", impl="ref",
                         seed=seed)


def run_until_done(gws, n_expected, max_ticks=400):
    for _ in range(max_ticks):
        if len(gws) == 1:
            gws[0].tick()
        else:
            ths = [threading.Thread(target=g.tick) for g in gws]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        if sum(g.counters["completed"] for g in gws) >= n_expected:
            return True
    return False


# ---------------------------------------------------------------- single rank
def test_gateway_cpu_end_to_end_and_priority_order():
    gw = Gateway(cfg(), engine=engine(slots=4), use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2)
    msgs = Workload(seed=2).make(40)
    gw.submit(msgs)
    gw.ingest()
    # one dispatch: the 4 free slots go to the most urgent tier present
    n = gw.dispatch()
    assert n == 4
    dispatched = [m for m in msgs if m.dispatched_at]
    assert sorted(m.priority for m in dispatched) == sorted(m.priority for m in msgs)[:4]
    assert run_until_done([gw], 40)
    assert gw.counters["dispatched"] == 40 and gw.pending() == 0
    st = gw.qm.get_all_queue_stats()
    assert sum(s.completed_count for s in st.values()) == 40
    assert sum(s.processing_count for s in st.values()) == 0
    summ = gw.rec.summary()
    assert summ["count"] == 40 and summ["p99_ms"] >= summ["p50_ms"] > 0


def test_engine_async_launch_never_drops_completions():
    from llm_message_queue_amd.backend.engine import Request
    eng = engine(slots=8)
    eng.admit([Request(i, np.arange(3, dtype=np.int32), gen_tokens=2) for i in range(8)])
    # 4 launches with no finish in between: launch() itself reaps the full queue
    for _ in range(4):
        eng.launch()
    res = eng.finish(block=True)
    assert len(res.completed) == 8 and eng.completed_total == 8
    assert sorted(r.req_id for r in res.completed) == list(range(8))
    assert eng.free_slots() == 8 and not eng.finish(block=True).completed


def test_latency_histogram_percentiles():
    rec = LatencyRecorder(4)
    v = np.array([1_000_000] * 98 + [400_000_000, 900_000_000])
    rec.record(np.zeros(100, dtype=np.int64), v, v)
    s = rec.summary()
    assert 0.9 < s["p50_ms"] < 1.1 and 390 < s["p99_ms"] < 410


def test_poisson_arrivals_rate():
    a = PoissonArrivals(1000.0, seed=1)
    a.reset(0.0)
    assert abs(len(a.due(10.0)) - 10000) < 400


# ---------------------------------------------------------------- planner
def load(free, depth, age=(0, 0, 0, 0), healthy=True, slots=10, **kw):
    return planner.make_load(free, slots - free, depth, age, healthy=healthy, slots_total=slots, **kw)


def test_plan_local_first_then_least_loaded():
    # GPU0 has 2 free of 10, GPU1 8, GPU2 5: router 0 keeps 2 locally, the
    # other 8 water-fill slot utilisation (GPU1 0.2 -> 0.5 first, then both)
    loads = np.stack([load(2, [0, 0, 10, 0]), load(8, [0, 0, 0, 0]), load(5, [0, 0, 0, 0])])
    q = planner.plan_dispatch(loads, [0] * 4, planner.PlanState("local_first"))
    assert q[0, 0, 2] == 2 and q[0, 1, 2] == 6 and q[0, 2, 2] == 2
    assert q.sum() == 10
    # least_connections: water-fill every GPU's utilisation (0.8 / 0.2 /
    # 0.5): GPU1 to 0.5, GPU1+GPU2 to 0.8, the last unit to the lowest index
    q = planner.plan_dispatch(loads, [0] * 4, planner.PlanState("least_connections"))
    assert q.sum() == 10 and list(q[0, :, 2]) == [1, 6, 3]


def test_plan_strict_priority_and_proportional_split():
    loads = np.stack([load(3, [4, 0, 10, 0]), load(3, [2, 0, 10, 0])])
    q = planner.plan_dispatch(loads, [0] * 4)
    assert q[:, :, 0].sum() == 6 and q[:, :, 2].sum() == 0           # realtime takes every slot
    assert q[0, :, 0].sum() == 4 and q[1, :, 0].sum() == 2
    loads = np.stack([load(2, [0, 0, 30, 0]), load(2, [0, 0, 10, 0])])
    q = planner.plan_dispatch(loads, [0] * 4)
    assert q[0, :, 2].sum() == 3 and q[1, :, 2].sum() == 1           # 4 slots split 3:1


def test_plan_aging_and_unhealthy():
    loads = np.stack([load(2, [5, 0, 0, 3], age=(0, 0, 0, 9_000_000)), load(4, [0, 0, 0, 0], healthy=False)])
    q = planner.plan_dispatch(loads, [0, 0, 0, 5_000_000])
    assert q[0, 0, 3] == 2 and q[:, 1].sum() == 0                     # overdue low first; no unhealthy target


# ---------------------------------------------------------------- multi-rank (threads)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_fakecomm_multirank_dispatch(world):
    comms = FakeComm.make(world)
    gws = [Gateway(cfg(), engine=engine(slots=4, seed=r), comm=comms[r], use_gpu_preprocess=False, prompt_cap=8,
                   gen_tokens=2) for r in range(world)]
    # all demand on rank 0: the planner must spread it over every GPU
    gws[0].submit(Workload(seed=7).make(12 * world))
    assert run_until_done(gws, 12 * world)
    assert all(g.pending() == 0 for g in gws)
    assert gws[0].counters["completed"] == 12 * world
    assert gws[0].counters["remote_sent"] > 0
    assert sum(g.counters["remote_recv"] for g in gws[1:]) == gws[0].counters["remote_sent"]
    assert all(g.engine.completed_total > 0 for g in gws)
    assert not gws[0].remote_out and all(not g.foreign for g in gws)


def test_grant_shortfall_from_concurrent_removal_keeps_the_exchange():
    """A queued request removed between the published load and the pop (a
    DELETE on the API thread, a peer 'remove', an admin dequeue) -- or popped
    and found cancelled -- leaves the router short of the plan's grant.  The
    receiving GPU expects exactly the grant's row count: the sender pads the
    shortfall with empty rows instead of breaking the all_to_all (found by
    the round-6 HTTP soak with DELETE churn: 'expected 4 rows from 0, got 3')."""
    world = 2
    comms = FakeComm.make(world)
    gws = [Gateway(cfg(), engine=engine(slots=8, seed=r), comm=comms[r], use_gpu_preprocess=False, prompt_cap=8,
                   gen_tokens=2) for r in range(world)]
    # few requests, room for all: the plan grants the whole published depth,
    # part of it to GPU 1
    msgs = Workload(seed=7).make(6)
    for m in msgs:
        m.priority = 3
    gws[0].submit(msgs)
    gws[0].ingest()
    gw0 = gws[0]
    removed, short = [], []
    orig_pop = gw0.qm.pop_tiers

    def racing_pop(tiers, n, *args, **kw):
        # the API thread dequeues one queued message right before the pop
        if not removed and n > 0:
            for m in msgs:
                if m.queue_name and gw0.qm.remove_message(m.queue_name, m):
                    removed.append(m)
                    break
        out = orig_pop(tiers, n, *args, **kw)
        short.append(n - len(out[0]))
        return out
    gw0.qm.pop_tiers = racing_pop
    assert run_until_done(gws, 5, max_ticks=100)
    assert len(removed) == 1 and max(short) == 1                      # the grant was not filled
    assert gw0.counters["completed"] == 5 and all(g.pending() == 0 for g in gws)
    assert gw0.counters["remote_sent"] > 0
    assert not gw0.remote_out and all(not g.foreign for g in gws)
    assert removed[0].dispatched_at == 0


# ---------------------------------------------------------------- multi-process gloo
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _gloo_worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from llm_message_queue_amd.parallel.comm import TorchComm
    comm = TorchComm()
    gw = Gateway(cfg(), engine=engine(slots=4, seed=rank), comm=comm, use_gpu_preprocess=False, prompt_cap=8,
                 gen_tokens=2)
    if rank == 0:
        gw.submit(Workload(seed=11).make(24))
    done = False
    for _ in range(300):
        gw.tick()
        tot = comm.all_gather_i64(np.array([gw.counters["completed"]]))
        if tot.sum() >= 24:
            done = True
            break
    g = comm.all_gather_i64(np.array([gw.counters["completed"], gw.counters["remote_recv"],
                                      gw.engine.completed_total]))
    b = comm.broadcast_i64(np.array([rank * 10 + 5]), root=1)
    if rank == 0:
        out.put((done, g.tolist(), int(b[0])))
    dist.destroy_process_group()


def test_gloo_world2_dispatch():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    import queue as _q
    res = None
    for _ in range(240):
        try:
            res = q.get(timeout=1)
            break
        except _q.Empty:
            if any(p.exitcode not in (None, 0) for p in ps):
                break
    for p in ps:
        p.join(timeout=60)
        if p.is_alive():
            p.kill()
    assert res is not None, [p.exitcode for p in ps]
    done, g, b = res
    assert done and g[0][0] == 24 and g[1][1] > 0 and g[1][2] > 0 and b == 15


# ---------------------------------------------------------------- affinity + KV migration
def test_affinity_routes_to_home_gpu():
    comms = FakeComm.make(2)
    gws = [Gateway(cfg(), engine=engine(slots=8, seed=r, token_budget=256), comm=comms[r], use_gpu_preprocess=False,
                   prompt_cap=8, gen_tokens=1) for r in range(2)]
    msgs = Workload(seed=5).make(6)
    for m in msgs:
        m.priority = 3
        m.metadata["home_gpu"] = 1
    gws[0].submit(msgs)
    assert run_until_done(gws, 6)
    assert gws[1].counters["remote_recv"] == 6          # all went to their home GPU despite local capacity


def test_kv_migration_fakecomm():
    from llm_message_queue_amd.models.llama_stub import LlamaStub
    from llm_message_queue_amd.parallel.migration import KVMigrator
    comms = FakeComm.make(2)
    a = LlamaStub(MICRO, slots=2, max_ctx=16, device="cpu", impl="ref", seed=1)
    b = LlamaStub(MICRO, slots=2, max_ctx=16, device="cpu", impl="ref", seed=2)
    for L in range(MICRO.layers):
        a.kcache[L][1, :, :5].normal_()
        a.vcache[L][1, :, :5].normal_()
    ma, mb = KVMigrator(a, comms[0]), KVMigrator(b, comms[1])
    t = threading.Thread(target=lambda: ma.send(1, 1, 5))
    t.start()
    nb = mb.recv(0, 0, 5)
    t.join()
    assert nb == MICRO.layers * 2 * MICRO.kv_heads * 5 * 128 * 2
    for L in range(MICRO.layers):
        assert torch.equal(b.kcache[L][0, :, :5], a.kcache[L][1, :, :5])
        assert torch.equal(b.vcache[L][0, :, :5], a.vcache[L][1, :, :5])


def test_telemetry_fault_injection_marks_unhealthy():
    from llm_message_queue_amd.backend.slot_page import SlotPage
    from llm_message_queue_amd.backend.telemetry import TelemetryService
    page = SlotPage("pytest-telem", 0)
    try:
        page.set_health(True)
        bad = []
        ts = TelemetryService(pages={0: page}, synthetic=1, on_unhealthy=lambda g, r: bad.append((g, r)))
        ts.inject(0, "valid", 1)
        ts.inject(0, "hbm_used_mb", 1000)
        ts.inject(0, "hbm_total_mb", 288000)
        ts.publish()
        assert page.read()["hbm_used_mib"] == 1000 and not bad
        ts.inject(0, "ecc_uncorrectable", 3)
        ts.publish()
        assert bad and bad[0][0] == 0 and "ECC" in bad[0][1] and page.read()["healthy"] == 0
    finally:
        page.close(unlink=True)


# ---------------------------------------------------------------- failure detection / evacuation
@pytest.mark.parametrize("world", [2, 4])
def test_backend_fault_evacuates_and_reroutes(world):
    comms = FakeComm.make(world)
    gws = [Gateway(cfg(), engine=engine(slots=4, seed=r), comm=comms[r], use_gpu_preprocess=False, prompt_cap=8,
                   gen_tokens=3) for r in range(world)]
    n = 16 * world
    msgs = Workload(seed=3).make(n)
    for i, m in enumerate(msgs):                      # half the conversations live on the GPU that will fail
        if i % 2:
            m.metadata["home_gpu"] = 1
    gws[0].submit(msgs)
    for _ in range(3):                                # get work in flight everywhere
        ths = [threading.Thread(target=g.tick) for g in gws]
        [t.start() for t in ths]
        [t.join() for t in ths]
    assert gws[1].engine.inflight() > 0
    gws[1].engine.inject(fail_launch=1)               # next forward on GPU 1 raises (HIP OOM)
    assert run_until_done(gws, n)
    assert not gws[1].healthy and "out of memory" in gws[1].health_reason
    assert gws[1].counters["evacuated"] > 0 and gws[0].counters["handed_back"] > 0
    assert gws[0].counters["completed"] == n and all(g.pending() == 0 for g in gws)
    assert not gws[0].remote_out and all(not g.foreign for g in gws)
    # after the fault GPU 1 got no new work
    before = gws[1].engine.completed_total
    gws[0].submit(Workload(seed=4).make(8))
    assert run_until_done(gws, n + 8)
    assert gws[1].engine.completed_total == before
    # operator brings it back: it is used again
    gws[1].set_healthy(True)
    gws[0].submit(Workload(seed=5).make(8 * world))
    assert run_until_done(gws, n + 8 + 8 * world)
    assert gws[1].engine.completed_total > before


def test_single_rank_fault_requeues_and_recovers():
    gw = Gateway(cfg(), engine=engine(slots=4), use_gpu_preprocess=False, prompt_cap=8, gen_tokens=3)
    gw.submit(Workload(seed=8).make(10))
    gw.tick(); gw.tick()
    gw.engine.inject(fail_launch=1)
    gw.tick()
    assert not gw.healthy and gw.counters["evacuated"] > 0 and gw.engine.inflight() == 0
    for _ in range(5):
        gw.tick()
    assert gw.counters["completed"] < 10 and gw.pending() > 0      # no healthy backend: requests wait
    gw.set_healthy(True)
    assert run_until_done([gw], 10)
    st = gw.qm.get_all_queue_stats()
    assert sum(s.processing_count for s in st.values()) == 0


def test_admit_capacity_bounds_prefill_backlog():
    """The dispatcher may only admit what the next step can start prefilling:
    requests beyond that wait in the priority queue, not inside the engine."""
    from llm_message_queue_amd.backend.engine import Request
    eng = engine(slots=16, token_budget=64)
    assert eng.admit_capacity() == 4                    # 64 tokens / mean prompt 16
    eng.admit([Request(i, np.arange(30, dtype=np.int32), gen_tokens=2) for i in range(3)])
    assert eng.admit_capacity() == 0                    # 3 decode-to-be + 90 pending prefill >= 64
    eng.step()
    eng.step()
    assert 0 < eng.admit_capacity() <= eng.free_slots()
    gw = Gateway(cfg(), engine=engine(slots=16, token_budget=64), use_gpu_preprocess=False, prompt_cap=30,
                 gen_tokens=2)
    gw.submit(Workload(seed=1).make(40))
    gw.ingest()
    n = gw.dispatch()
    assert 0 < n < 16 and gw.pending() == 40 - n       # slots were free, prefill headroom was not


def test_engine_attention_tiles_match_per_token_path():
    """The engine's segment tiles (decode rows + prefill chunks cut at 16)
    give the same tokens as per-token attention (reference ops on CPU)."""
    from llm_message_queue_amd.backend.engine import Request
    outs = []
    for use_tiles in (False, True):
        eng = BackendEngine(MICRO, slots=6, max_ctx=64, token_budget=24, device="cpu", impl="ref", seed=9)
        eng.use_tiles = use_tiles
        rng = np.random.default_rng(0)
        reqs = [Request(i, rng.integers(0, 500, size=int(rng.integers(1, 40))).astype(np.int32), gen_tokens=3)
                for i in range(10)]
        done = []
        pending = list(reqs)
        for _ in range(200):
            pending = pending[len(eng.admit(pending)):]
            done += eng.step().completed
            if len(done) == 10:
                break
        assert len(done) == 10
        outs.append({r.req_id: (r.generated, r.prefilled) for r in done})
        outs.append(eng.model.kcache[0].clone())
    assert outs[0] == outs[2] and torch.equal(outs[1], outs[3])


def test_request_tracer_chrome_trace(tmp_path):
    import json
    from llm_message_queue_amd.utils.tracing import RequestTracer
    gw = Gateway(cfg(), engine=engine(slots=4), use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2)
    tr = RequestTracer(sample_every=1)
    gw.tracer = gw.engine.tracer = tr
    gw.submit(Workload(seed=2).make(10))
    assert run_until_done([gw], 10)
    n = tr.dump(str(tmp_path / "t.json"))
    ev = json.load(open(tmp_path / "t.json"))["traceEvents"]
    assert n == len(ev)
    served = [e for e in ev if e.get("name") == "served"]
    steps = [e for e in ev if e.get("name", "").startswith("step ")]
    assert len(served) == 10 and steps and all(e["dur"] >= 0 for e in served + steps)
    assert {e["tid"] for e in served} <= {1, 2, 3, 4}


# ---------------------------------------------------------------- conversation KV residency
def test_conversation_kv_resident_between_turns_matches_full_prefill():
    """Turn 2 of a dialog admitted into the slot that kept turn 1's KV must
    produce exactly the KV a fresh prefill of the whole dialog produces
    (gen_tokens=1: the cached context is exactly the turn-1 prompt)."""
    from llm_message_queue_amd.backend.engine import Request
    p1 = np.arange(5, 17, dtype=np.int32)
    p2 = np.arange(100, 109, dtype=np.int32)
    a = engine(slots=4, token_budget=64)
    a.admit([Request(1, p1, gen_tokens=1, conv=77)])
    a.drain()
    assert a.resident_context(77) == len(p1) and a.free_slots() == 4      # parked slot counts as free
    (r2,) = a.admit([Request(2, p2, gen_tokens=1, conv=77)])
    assert r2.reused == len(p1)
    a.drain()
    assert a.kv_reused_tokens == len(p1) and r2.prefilled == len(p2)
    b = engine(slots=4, token_budget=64)
    (rb,) = b.admit([Request(3, np.concatenate([p1, p2]), gen_tokens=1)])
    b.drain()
    n = len(p1) + len(p2)
    for L in range(MICRO.layers):
        assert torch.allclose(a.model.kcache[L][r2.slot, :, :n].float(), b.model.kcache[L][rb.slot, :, :n].float(),
                              atol=2e-2)
        assert torch.allclose(a.model.vcache[L][r2.slot, :, :n].float(), b.model.vcache[L][rb.slot, :, :n].float(),
                              atol=2e-2)


def test_conversation_slots_evicted_lru_when_full():
    from llm_message_queue_amd.backend.engine import Request
    e = engine(slots=2, token_budget=64)
    for c in (1, 2):
        e.admit([Request(c, np.arange(4, dtype=np.int32), gen_tokens=2, conv=c)])
    e.drain()
    assert e.resident_context(1) == 5 and e.resident_context(2) == 5
    e.admit([Request(3, np.arange(4, dtype=np.int32), gen_tokens=2, conv=3)])   # evicts conv 1 (LRU)
    e.drain()
    assert e.resident_context(1) == 0 and e.resident_context(2) == 5 and e.kv_evictions == 1
    # a context that would overflow max_ctx restarts from scratch
    (r,) = e.admit([Request(4, np.arange(60, dtype=np.int32), gen_tokens=2, conv=2)])
    assert r.reused == 0


@pytest.mark.parametrize("residency", [True, False])
def test_gateway_dialog_turns_reuse_or_replay(residency):
    """Turn 2 of a conversation: with KV residency only its new tokens are
    prefilled (the dialog KV is reused); without it the dialog is replayed."""
    gw = Gateway(cfg(), engine=engine(slots=8, token_budget=256), use_gpu_preprocess=False, prompt_cap=8,
                 gen_tokens=3)
    gw.kv_residency = residency
    t1 = Workload(seed=9).make(4)
    for i, m in enumerate(t1):
        m.conversation_id = f"dlg-{i}"
    gw.submit(t1)
    assert run_until_done([gw], 4)
    tok1 = gw.engine.total_tokens
    t2 = Workload(seed=10).make(4)
    for i, m in enumerate(t2):
        m.conversation_id = f"dlg-{i}"
    gw.submit(t2)
    assert run_until_done([gw], 8)
    tok2 = gw.engine.total_tokens - tok1
    new_prefill = sum(len(m.prompt_ids) for m in t2) + 4 * (3 - 1)      # prompts + decode steps
    if residency:
        assert gw.engine.kv_reused_tokens > 0 and tok2 == new_prefill
        assert all(gw.conv_home[f"dlg-{i}"] == 0 for i in range(4))
    else:
        assert gw.engine.kv_reused_tokens == 0 and tok2 > new_prefill    # dialog replayed


def test_coordinated_stop_across_ranks():
    """One rank stopping makes every rank leave after the same tick (ticks are
    collectives; a rank-local exit would strand the others)."""
    comms = FakeComm.make(3)
    gws = [Gateway(cfg(), engine=engine(slots=4, seed=r), comm=comms[r], use_gpu_preprocess=False, prompt_cap=8,
                   gen_tokens=2) for r in range(3)]
    ticks = [0, 0, 0]

    def loop(r):
        while not gws[r].peers_stopping:
            if r == 1 and ticks[r] == 5:
                gws[r].request_stop()
            gws[r].tick()
            ticks[r] += 1

    ths = [threading.Thread(target=loop, args=(r,)) for r in range(3)]
    [t.start() for t in ths]
    [t.join(timeout=30) for t in ths]
    assert not any(t.is_alive() for t in ths)
    assert ticks[0] == ticks[1] == ticks[2] == 6


# ---------------------------------------------------------------- overload shedding
def test_expired_requests_go_to_dead_letter_not_gpu():
    """A request still queued past its deadline (arrival + timeout) is shed
    to the DLQ with status ``timeout``; live ones are served (BASELINE
    config 5: dead-letter under sustained overload)."""
    from llm_message_queue_amd.queue.dead_letter import DeadLetterQueue
    import time
    dlq = DeadLetterQueue()
    gw = Gateway(cfg(), engine=engine(slots=4), use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2,
                 dead_letter=dlq)
    msgs = Workload(seed=5).make(30)
    now = time.monotonic_ns()
    for i, m in enumerate(msgs):
        if i % 3 == 0:                       # 10 requests arrived 2 s ago with a 1 s deadline
            m.arrival_ns = now - 2_000_000_000
            m.timeout = 1_000_000_000
    stale = [m for i, m in enumerate(msgs) if i % 3 == 0]
    # the stale ones queued first (tier heads), then the live ones
    gw.submit(stale)
    gw.ingest()
    gw.submit([m for i, m in enumerate(msgs) if i % 3])
    gw.ingest()
    gw.dispatch()
    assert gw.counters["expired"] == 10 and dlq.size() == 10
    assert all(m.status == "timeout" and not m.dispatched_at for m in stale)
    assert {it.message.id for it in dlq.get_all()} == {m.id for m in stale}
    assert all(it.fail_reason == "deadline exceeded before dispatch" for it in dlq.get_all())
    assert run_until_done([gw], 20)
    assert gw.counters["completed"] == 20 and gw.pending() == 0
    # shedding off: everything is served
    c = cfg()
    c.queue.shed_expired = False
    gw2 = Gateway(c, engine=engine(slots=4), use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2)
    ms = Workload(seed=6).make(6)
    for m in ms:
        m.arrival_ns, m.timeout = now - 2_000_000_000, 1_000_000_000
    gw2.submit(ms)
    assert run_until_done([gw2], 6) and gw2.counters["expired"] == 0


def test_expired_requests_behind_a_live_head_are_shed_at_pop():
    from llm_message_queue_amd.queue.dead_letter import DeadLetterQueue
    import time
    dlq = DeadLetterQueue()
    gw = Gateway(cfg(), engine=engine(slots=8, token_budget=256), use_gpu_preprocess=False, prompt_cap=8,
                 gen_tokens=2, dead_letter=dlq)
    msgs = Workload(seed=7).make(8)
    for m in msgs:                           # one tier (no priority keywords)
        m.content, m.priority, m.queue_name = "plain request text", 3, "normal"
    now = time.monotonic_ns()
    for m in msgs[1::2]:                     # interleaved: live head, stale, live, stale ...
        m.arrival_ns, m.timeout = now - 5_000_000_000, 1_000_000_000
    gw.submit(msgs)
    gw.ingest()
    gw.dispatch()
    assert gw.counters["expired"] == 4 and gw.counters["dispatched"] == 4 and dlq.size() == 4
    assert all(m.status == "timeout" for m in msgs[1::2])


def test_residual_in_gemm_matches_fused_norm_path():
    """o/down accumulating into the residual stream (addmm, beta = 1) gives
    the same trunk output as F.linear + residual-add RMSNorm (bf16 rounding
    differs by one step)."""
    from llm_message_queue_amd.models.llama_stub import LlamaStub
    cfg = LlamaConfig(vocab=512, dim=2048, layers=2, heads=16, kv_heads=4, ffn=512)
    a = LlamaStub(cfg, slots=2, max_ctx=16, device="cpu", impl="ref", seed=5, residual_in_gemm=True)
    b = LlamaStub(cfg, slots=2, max_ctx=16, device="cpu", impl="ref", seed=5, residual_in_gemm=False)
    tok = torch.randint(0, cfg.vocab, (12,), generator=torch.Generator().manual_seed(0))
    pos = torch.tensor(list(range(6)) * 2, dtype=torch.int32)
    slot = torch.tensor([0] * 6 + [1] * 6, dtype=torch.int32)
    ha, hb = a.hidden(tok, pos, slot).float(), b.hidden(tok, pos, slot).float()
    assert torch.allclose(ha, hb, atol=5e-2, rtol=5e-2), (ha - hb).abs().max()
    assert torch.allclose(a.kcache[1], b.kcache[1], atol=5e-2, rtol=5e-2)


def test_split_qkv_matches_fused_qkv_gemm():
    """q and kv GEMMs written into column slices of one buffer == the fused
    QKV GEMM (same weight tensor, row-slice views): bitwise equal trunk."""
    from llm_message_queue_amd.models.llama_stub import LlamaStub
    cfg = LlamaConfig(vocab=512, dim=2048, layers=2, heads=16, kv_heads=4, ffn=512)
    a = LlamaStub(cfg, slots=2, max_ctx=16, device="cpu", impl="ref", seed=5, split_qkv=True)
    b = LlamaStub(cfg, slots=2, max_ctx=16, device="cpu", impl="ref", seed=5, split_qkv=False)
    tok = torch.randint(0, cfg.vocab, (12,), generator=torch.Generator().manual_seed(0))
    pos = torch.tensor(list(range(6)) * 2, dtype=torch.int32)
    slot = torch.tensor([0] * 6 + [1] * 6, dtype=torch.int32)
    ha, hb = a.hidden(tok, pos, slot).float(), b.hidden(tok, pos, slot).float()
    assert torch.allclose(ha, hb, atol=1e-2, rtol=1e-2), (ha - hb).abs().max()
    assert torch.allclose(a.kcache[1].float(), b.kcache[1].float(), atol=1e-2, rtol=1e-2)
