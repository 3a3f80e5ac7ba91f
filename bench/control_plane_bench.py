"""Per-tick control-plane cost at N ranks: the serving loop's two collectives
(``all_gather`` of the int64 load vectors + ``all_to_all`` of request
descriptors, ``parallel/comm.py``) on the gloo group the bench uses by
default, with the planner in between -- everything a rank does per tick
besides its own GPU step.

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        --master-port 29600 bench/control_plane_bench.py --iters 300

Rank 0 prints one JSON line: p50 / p99 / mean microseconds per tick.  The
serving tick is ~44 ms of GPU work, so this is the share of a tick the
lockstep control plane costs at that world size (weak-scaling overhead).
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
    a = ap.parse_args()
    from llm_message_queue_amd.gateway.router import DESC_HDR
    from llm_message_queue_amd.parallel import planner
    from llm_message_queue_amd.parallel.comm import init_from_env
    comm = init_from_env(backend="gloo", control="gloo")
    W, me = comm.world, comm.rank
    width = DESC_HDR + 32
    rng = np.random.default_rng(me)
    times = []
    for it in range(a.iters + 20):
        t0 = time.perf_counter()
        load = planner.make_load(int(rng.integers(0, 300)), 1200, [int(x) for x in rng.integers(0, 200, 4)],
                                 [int(x) for x in rng.integers(0, 50_000, 4)], healthy=True,
                                 done_for=[0] * W, pinned=[0] * W, stopping=False)
        loads = comm.all_gather_i64(load)
        planner.plan_dispatch(loads, [50_000, 100_000, 150_000, 200_000])
        n = a.remote_per_tick
        send = [np.zeros((0 if j == me else n, width), dtype=np.int32) for j in range(W)]
        comm.all_to_all_rows(send, [0 if i == me else n for i in range(W)], width)
        if it >= 20:
            times.append(time.perf_counter() - t0)
    t = np.asarray(times) * 1e6
    agg = comm.all_gather_i64(np.array([int(np.percentile(t, 50)), int(np.percentile(t, 99)), int(t.mean())],
                                       dtype=np.int64))
    if me == 0:
        print(json.dumps({"bench": "control plane per tick (gloo)", "world": W, "iters": a.iters,
                          "p50_us": int(agg[:, 0].max()), "p99_us": int(agg[:, 1].max()),
                          "mean_us": int(agg[:, 2].max()),
                          "share_of_44ms_tick_pct": round(100 * agg[:, 2].max() / 44_000, 2)}), flush=True)


if __name__ == "__main__":
    main()
