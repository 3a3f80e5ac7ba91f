"""Two ranks on the one MI355X of a GPU box: the multi-rank serving path with
the HIP backend (tiny Llama-shaped model), the shared-memory control plane
and cross-rank dispatch.  RCCL needs one device per rank, so with both ranks
on cuda:0 ``init_from_env`` puts every torch group on gloo (the rehearsal
layout of ``parallel/comm.py:local_device_index``); the per-tick exchange runs
through ``ShmComm`` exactly as on an 8-GPU node.
"""
import os
import queue as _q
import socket
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), LOCAL_RANK=str(rank), TORCHELASTIC_RUN_ID=f"g{port}",
                      HSA_ENABLE_IPC_MODE_LEGACY="0")
    try:
        import torch
        from llm_message_queue_amd.backend.engine import BackendEngine
        from llm_message_queue_amd.gateway.router import Gateway
        from llm_message_queue_amd.gateway.workload import Workload
        from llm_message_queue_amd.models.llama_stub import LlamaConfig
        from llm_message_queue_amd.parallel.comm import ShmComm, init_from_env, local_device_index
        from llm_message_queue_amd.utils.config import default_config
        dev = torch.device("cuda", local_device_index())
        torch.cuda.set_device(dev)
        comm = init_from_env(control="shm", timeout_s=60)
        cfg = default_config()
        cfg.queue.enable_metrics = False
        eng = BackendEngine(LlamaConfig.tiny(), slots=8, max_ctx=64, token_budget=128, device=dev, impl="hip",
                            seed=rank)
        gw = Gateway(cfg, engine=eng, comm=comm, use_gpu_preprocess=True, prompt_cap=16, gen_tokens=2)
        n = 40
        if rank == 0:                                   # one ingress (the cli serve topology)
            gw.submit(Workload(seed=5).make(n))
        done = False
        for _ in range(600):
            gw.tick()
            if comm.all_gather_i64(np.array([gw.counters["completed"]])).sum() >= n:
                done = True
                break
        torch.cuda.synchronize()
        g = comm.all_gather_i64(np.array([gw.counters["completed"], gw.counters["remote_recv"]]))
        out.put((rank, isinstance(comm, ShmComm), done, g.tolist()))
    except Exception as e:                              # surfaced by the parent
        out.put((rank, "error", repr(e), None))


def test_two_ranks_share_one_gpu_with_shm_control_plane():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res, t0 = [], time.time()
    while len(res) < 2 and time.time() - t0 < 100:
        try:
            res.append(q.get(timeout=1))
        except _q.Empty:
            if all(p.exitcode is not None for p in ps):
                break
    for p in ps:
        p.join(timeout=20)
        if p.is_alive():
            p.kill()
    assert len(res) == 2, [p.exitcode for p in ps]
    for rank, shm, done, g in res:
        assert shm is True, (rank, shm, done)
        assert done and sum(r[0] for r in g) == 40, (rank, g)
    assert res[0][3][1][1] > 0                          # rank 1 served work from rank 0's ingress
