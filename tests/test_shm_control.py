"""Node-local shared-memory control plane (csrc/queue/shm_coll.h, ShmComm).

Multi-process on the CPU (gloo for setup barriers): all_gather /
all_to_all / broadcast semantics over many ops (both buffer parities reused),
per-rank variable payloads, a dead peer surfacing as PeerLost within the
timeout, and the multi-rank gateway dispatching through it.
"""
import os
import queue as _q
import socket
import time

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), LOCAL_RANK=str(rank), TORCHELASTIC_RUN_ID=f"t{port}")


def _coll_worker(rank, world, port, out):
    _env(rank, world, port)
    from llm_message_queue_amd.parallel.comm import ShmComm, init_from_env
    comm = init_from_env(backend="gloo", control="shm", timeout_s=20)
    assert isinstance(comm, ShmComm)
    ok = True
    for it in range(200):
        g = comm.all_gather_i64(np.array([rank, it, rank * it], dtype=np.int64))
        ok &= g.shape == (world, 3) and (g[:, 0] == np.arange(world)).all() and (g[:, 1] == it).all()
        # rank r sends (r + d + it) % 3 rows to rank d, each row = (r, d, it, k)
        send = [np.array([[rank, d, it, k] for k in range((rank + d + it) % 3)], dtype=np.int32).reshape(-1, 4)
                for d in range(world)]
        counts = [(s + rank + it) % 3 for s in range(world)]
        got = comm.all_to_all_rows(send, counts, 4)
        for s, rows in enumerate(got):
            ok &= rows.shape == (counts[s], 4)
            ok &= bool((rows[:, 0] == s).all() and (rows[:, 1] == rank).all() and (rows[:, 2] == it).all())
        # the variable form (receivers do not know the counts: KV-migration headers)
        var = comm.all_to_all_var(send, 4)
        for s, rows in enumerate(var):
            ok &= rows.shape == (counts[s], 4) and bool((rows[:, 0] == s).all() if len(rows) else True)
        root = it % world
        b = comm.broadcast_i64(np.array([root * 100 + it], dtype=np.int64), root=root)
        ok &= int(b[0]) == root * 100 + it
        if it % 50 == 0:
            comm.barrier()
    out.put((rank, bool(ok), comm.c.ops))


def _run(target, world, timeout=120, extra=()):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + tuple(extra)) for r in range(world)]
    for p in ps:
        p.start()
    res = []
    t0 = time.time()
    while len(res) < world and time.time() - t0 < timeout:
        try:
            res.append(q.get(timeout=1))
        except _q.Empty:
            if all(p.exitcode is not None for p in ps):
                break
    for p in ps:
        p.join(timeout=30)
        if p.is_alive():
            p.kill()
    return res, [p.exitcode for p in ps]


@pytest.mark.parametrize("world", [2, 4])
def test_shm_collectives_match_semantics(world):
    res, codes = _run(_coll_worker, world)
    assert len(res) == world, codes
    assert all(ok for _, ok, _ in res), res
    assert len({ops for _, _, ops in res}) == 1          # every rank ran the same op sequence


def _dead_peer_worker(rank, world, port, out):
    _env(rank, world, port)
    from llm_message_queue_amd.parallel.comm import PeerLost, init_from_env
    comm = init_from_env(backend="gloo", control="shm", timeout_s=3)
    comm.all_gather_i64(np.array([rank]))
    if rank == world - 1:
        os._exit(0)                                       # dies without a goodbye
    t0 = time.time()
    try:
        for _ in range(10):
            comm.all_gather_i64(np.array([rank]))
        out.put((rank, "no error", 0.0))
    except PeerLost:
        out.put((rank, "PeerLost", time.time() - t0))


def _overflow_worker(rank, world, port, out):
    _env(rank, world, port)
    from llm_message_queue_amd.parallel.comm import PeerLost, ShmComm, init_from_env
    comm = init_from_env(backend="gloo", control="shm", timeout_s=30)
    assert isinstance(comm, ShmComm)
    cap = comm.c.buf_bytes
    t0 = time.monotonic()
    try:                                   # rank 1's payload does not fit its buffer
        comm.all_gather_i64(np.zeros(cap // 8 + 16 if rank == 1 else 4, dtype=np.int64))
        res = "no error"
    except PeerLost as e:
        res = "overflow" if "overflow" in str(e) else f"other: {e}"
    out.put((rank, res, time.monotonic() - t0))


def test_shm_payload_overflow_fails_every_rank_at_once():
    """an oversized control payload used to raise on the
    sending rank only, while every other rank spun to its 60 s timeout; now
    the overflow is published and every rank raises PeerLost immediately."""
    res, codes = _run(_overflow_worker, 3, timeout=120)
    assert len(res) == 3, codes
    for rank, what, dt in res:
        assert what == "overflow", (rank, what)
        assert dt < 10.0, (rank, dt)


def test_shm_dead_peer_raises_peer_lost_within_timeout():
    res, codes = _run(_dead_peer_worker, 3, timeout=60)
    assert len(res) == 2, codes
    for _, what, dt in res:
        assert what == "PeerLost" and dt < 15, res


def _gateway_worker(rank, world, port, out):
    _env(rank, world, port)
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.parallel.comm import init_from_env
    from llm_message_queue_amd.utils.config import default_config
    comm = init_from_env(backend="gloo", control="shm", timeout_s=30)
    cfg = default_config()
    cfg.queue.enable_metrics = False
    micro = LlamaConfig(vocab=256, dim=256, layers=1, heads=2, kv_heads=1, ffn=256)
    eng = BackendEngine(micro, slots=4, max_ctx=64, token_budget=32, device="cpu", impl="ref", seed=rank)
    gw = Gateway(cfg, engine=eng, comm=comm, use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2)
    if rank == 0:
        gw.submit(Workload(seed=11).make(24))
    done = False
    for _ in range(400):
        gw.tick()
        if comm.all_gather_i64(np.array([gw.counters["completed"]])).sum() >= 24:
            done = True
            break
    g = comm.all_gather_i64(np.array([gw.counters["completed"], gw.counters["remote_recv"]]))
    out.put((rank, done, g.tolist()))


def _gateway_dead_peer_worker(rank, world, port, out):
    """Gateways on the shm control plane; the last rank dies after a few
    ticks.  The survivors' ticks wait in the split-phase overlap loop
    (``Gateway._overlap``: ingest while peers catch up), which must end at
    the collective's deadline and raise PeerLost -- not spin forever."""
    _env(rank, world, port)
    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.parallel.comm import PeerLost, ShmComm, init_from_env
    from llm_message_queue_amd.utils.config import default_config
    comm = init_from_env(backend="gloo", control="shm", timeout_s=3)
    assert isinstance(comm, ShmComm)
    cfg = default_config()
    cfg.queue.enable_metrics = False
    micro = LlamaConfig(vocab=256, dim=256, layers=1, heads=2, kv_heads=1, ffn=256)
    eng = BackendEngine(micro, slots=4, max_ctx=64, token_budget=32, device="cpu", impl="ref", seed=rank)
    gw = Gateway(cfg, engine=eng, comm=comm, use_gpu_preprocess=False, prompt_cap=8, gen_tokens=2)
    gw.submit(Workload(seed=rank).make(8))
    for _ in range(3):
        gw.tick()
    if rank == world - 1:
        os._exit(0)                                       # dies without a goodbye
    t0 = time.time()
    try:
        for _ in range(50):
            gw.submit(Workload(seed=100 + rank).make(2))  # arrivals keep the overlap loop busy
            gw.tick()
        out.put((rank, "no error", 0.0))
    except PeerLost:
        out.put((rank, "PeerLost", time.time() - t0))


def test_gateway_tick_with_dead_peer_raises_peer_lost():
    res, codes = _run(_gateway_dead_peer_worker, 3, timeout=120)
    assert len(res) == 2, codes
    for _, what, dt in res:
        assert what == "PeerLost" and dt < 15, res


def test_gateway_dispatch_over_shm_control_plane():
    res, codes = _run(_gateway_worker, 2, timeout=240)
    assert len(res) == 2, codes
    for _, done, g in res:
        assert done and sum(r[0] for r in g) == 24
    assert res[0][2][1][1] > 0                            # rank 1 received work from rank 0's ingress


def _fallback_worker(rank, world, port, out):
    _env(rank, world, port)
    from llm_message_queue_amd.parallel import comm as C
    real = C.ShmComm.__init__

    def broken_attach(self, data, name, timeout_s=60.0, buf_bytes=4 << 20):
        if data.rank == 1:                             # this rank cannot attach
            name = name + "_missing"
        real(self, data, name, timeout_s, buf_bytes)

    if rank == 1:
        C.ShmComm.__init__ = broken_attach
    else:
        C.ShmComm.__init__ = lambda self, data, name, timeout_s=60.0, buf_bytes=4 << 20: real(
            self, data, name, timeout_s, buf_bytes)
    comm = C.init_from_env(backend="gloo", control="shm", timeout_s=20)
    g = comm.all_gather_i64(np.array([rank]))
    out.put((rank, type(comm).__name__, g[:, 0].tolist()))


def test_shm_setup_failure_falls_back_to_torch_group_on_every_rank():
    res, codes = _run(_fallback_worker, 2, timeout=60)
    assert len(res) == 2, codes
    assert {kind for _, kind, _ in res} == {"TorchComm"}
    assert all(g == [0, 1] for _, _, g in res)


def _behind_worker(rank, world, port, out):
    _env(rank, world, port)
    from llm_message_queue_amd.parallel.comm import ShmComm, init_from_env
    comm = init_from_env(backend="gloo", control="shm", timeout_s=30)
    assert isinstance(comm, ShmComm)
    comm.all_gather_i64(np.array([rank]))
    if rank == 0:
        behind_before = comm.peers_behind()         # rank 1 sleeps before the next collective
        t0 = time.monotonic()
        while comm.peers_behind() and time.monotonic() - t0 < 20:
            time.sleep(0.005)
        waited = time.monotonic() - t0
        behind_after = comm.peers_behind()         # rank 1 now waits inside the collective
        comm.all_gather_i64(np.array([rank]))
        out.put((rank, behind_before, behind_after, waited))
    else:
        time.sleep(1.0)
        comm.all_gather_i64(np.array([rank]))
        out.put((rank, comm.peers_behind(), None, 0.0))


def test_shm_peers_behind_is_a_non_blocking_arrival_probe():
    """``ShmComm.peers_behind`` (the extra-local-step trigger) reports, without
    joining, whether some peer has not reached the next collective yet."""
    res, codes = _run(_behind_worker, 2, timeout=90)
    assert len(res) == 2, codes
    r0 = [r for r in res if r[0] == 0][0]
    assert r0[1] is True and r0[2] is False and 0.5 < r0[3] < 20, r0
