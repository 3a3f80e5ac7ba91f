"""Per-tick control-plane cost at N ranks: the serving loop's two collectives
(``all_gather`` of the int64 load vectors + ``all_to_all`` of request
descriptors, ``parallel/comm.py``) with the planner in between -- everything
a rank does per tick besides its own GPU step -- on the gloo (host TCP) or
the nccl (RCCL on a high-priority side stream, HostLink staging) control
group.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29600 bench/control_plane_bench.py --iters 300 [--control nccl] [--busy-gpu]

``--busy-gpu`` keeps two large GEMMs queued on the default stream the whole
time (the serving engine's 2-deep forward run-ahead): the control plane must
not wait behind them.  ``--force-group`` builds a process group even at
world size 1 (one GPU box: measures the per-call cost of each backend; the
cross-GPU latency itself needs more ranks).

Rank 0 prints one JSON line: p50 / p99 / mean microseconds per tick.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=300)
    ap.add_argument("--remote-per-tick", type=int, default=16, help="descriptors sent to each peer per tick")
    ap.add_argument("--control", default="gloo", choices=["gloo", "nccl", "shm"])
    ap.add_argument("--busy-gpu", action="store_true")
    ap.add_argument("--force-group", action="store_true")
    a = ap.parse_args()
    import torch
    from llm_message_queue_amd.gateway.router import DESC_HDR
    from llm_message_queue_amd.parallel import planner
    from llm_message_queue_amd.parallel.comm import TorchComm, init_from_env
    gpu = torch.cuda.is_available()
    if a.force_group and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29633")
        os.environ.setdefault("RANK", "0")
        if gpu:
            torch.cuda.set_device(0)
        dist.init_process_group(backend="nccl" if gpu else "gloo", world_size=1, rank=0,
                                **({"device_id": torch.device("cuda", 0)} if gpu else {}))
        if a.control == "gloo":
            comm = TorchComm(group=dist.new_group(backend="gloo"), device=torch.device("cpu"))
        else:
            comm = TorchComm()
    else:
        comm = init_from_env(backend="nccl" if gpu else "gloo", control=a.control)
    if a.control == "shm" and int(os.environ.get("WORLD_SIZE", "1")) > 1:
        from llm_message_queue_amd.parallel.comm import ShmComm
        assert isinstance(comm, ShmComm), type(comm)
    W, me = comm.world, comm.rank
    width = DESC_HDR + 32
    rng = np.random.default_rng(me)
    busy = []
    if a.busy_gpu and gpu:
        x = torch.randn(8192, 8192, device="cuda", dtype=torch.bfloat16)

        def feed():
            while len(busy) < 2:
                y = x @ x
                ev = torch.cuda.Event()
                ev.record()
                busy.append((ev, y))
            while busy and busy[0][0].query():
                busy.pop(0)
    else:
        def feed():
            pass
    st = planner.PlanState("least_connections")
    times = []
    for it in range(a.iters + 20):
        feed()
        t0 = time.perf_counter()
        load = planner.make_load(int(rng.integers(0, 300)), 1200, [int(x) for x in rng.integers(0, 200, 4)],
                                 [int(x) for x in rng.integers(0, 50_000, 4)], healthy=True,
                                 done_for=[0] * W, pinned=np.zeros((W, 4), np.int64), stopping=False,
                                 slots_total=1536, slots_free=300)
        loads = comm.all_gather_i64(load)
        planner.plan_dispatch(loads, [50_000, 100_000, 150_000, 200_000], st)
        n = a.remote_per_tick
        send = [np.zeros((0 if j == me else n, width), dtype=np.int32) for j in range(W)]
        comm.all_to_all_rows(send, [0 if i == me else n for i in range(W)], width)
        if it >= 20:
            times.append(time.perf_counter() - t0)
    t = np.asarray(times) * 1e6
    agg = comm.all_gather_i64(np.array([int(np.percentile(t, 50)), int(np.percentile(t, 99)), int(t.mean())],
                                       dtype=np.int64))
    if gpu:
        torch.cuda.synchronize()
    if me == 0:
        print(json.dumps({"bench": f"control plane per tick ({a.control})", "world": W, "iters": a.iters,
                          "busy_gpu": bool(a.busy_gpu and gpu),
                          "p50_us": int(agg[:, 0].max()), "p99_us": int(agg[:, 1].max()),
                          "mean_us": int(agg[:, 2].max()),
                          "share_of_44ms_tick_pct": round(100 * agg[:, 2].max() / 44_000, 2)}), flush=True)


if __name__ == "__main__":
    main()
