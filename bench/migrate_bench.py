"""Conversation re-homing across GPU backends: KV migration vs dialog replay
(N11; BASELINE config 4 "long-dialog replay routed across GPUs").

C concurrent conversations, T turns each, closed loop, all entering at rank 0
(the `cli serve` ingress).  In the migrate and replay modes every turn after the first is placed on a GPU
other than the one holding its KV (``Gateway.rehome_every_turn``) -- the
worst case for re-homing (a rebalance on every turn).
Modes (one per launch, the job's collectives stop together):

  * migrate -- the turn's KV moves from its home GPU (two-phase p2p on the
    data group: token counts, then packed K/V) and only the new tokens are
    prefilled;
  * replay  -- no migration: the new GPU prefills the whole dialog again;
  * pinned  -- affinity on (turns go home while it has room): the reference
    point without re-homing.

    python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 \\
        --master-port 29700 bench/migrate_bench.py --mode migrate

On a 1-GPU box both ranks share the device and torch.distributed runs on gloo
(RCCL needs one device per rank), so the KV moves through host memory -- a
functional rehearsal and an upper bound on the migration cost, not an xGMI
measurement.  Rank 0 prints one JSON line.
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="migrate", choices=["migrate", "replay", "pinned"])
    ap.add_argument("--convs", type=int, default=512)
    ap.add_argument("--turns", type=int, default=8)
    ap.add_argument("--slots", type=int, default=768)
    ap.add_argument("--max-ctx", type=int, default=512)
    ap.add_argument("--token-budget", type=int, default=4096)
    ap.add_argument("--gen-tokens", type=int, default=16)
    ap.add_argument("--prompt-cap", type=int, default=32)
    ap.add_argument("--timeout-s", type=float, default=150.0)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--cpu", action="store_true", help="tiny model on CPU (rehearsal of the control flow)")
    a = ap.parse_args()
    import torch

    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.parallel.comm import init_from_env, local_device_index
    from llm_message_queue_amd.preprocess.preprocessor import Preprocessor
    from llm_message_queue_amd.utils.config import default_config

    if a.cpu:
        dev = torch.device("cpu")
        comm = init_from_env(backend="gloo", control="gloo")
        a.model, a.slots, a.max_ctx, a.token_budget, a.prompt_cap = "tiny", 32, 128, 256, 12
        a.gen_tokens = min(a.gen_tokens, 4)
    else:
        torch.cuda.set_device(local_device_index())
        dev = torch.device("cuda", local_device_index())
        comm = init_from_env(control="gloo")
    W, rank = comm.world, comm.rank
    cfg = default_config()
    cfg.queue.enable_metrics = False
    cfg.backend.max_ctx = a.max_ctx
    cfg.loadbalancer.algorithm = "round_robin"
    cfg.gpu.kv_migration = a.mode == "migrate"
    for lv in cfg.queue.levels:
        lv.max_concurrent = 0
    # replicas of ONE model: identical weights on every GPU (a migrated KV is
    # only meaningful against the same weights)
    engine = BackendEngine(LlamaConfig.by_name(a.model), slots=a.slots, max_ctx=a.max_ctx,
                           token_budget=a.token_budget, device=dev, impl="ref" if a.cpu else "hip", seed=1234)
    engine.warm_shapes()
    pre = Preprocessor(cfg.preprocessor, use_gpu=not a.cpu, device=str(dev))
    gw = Gateway(cfg, preprocessor=pre, engine=engine, comm=comm, use_gpu_preprocess=not a.cpu,
                 prompt_cap=a.prompt_cap, gen_tokens=a.gen_tokens)
    gw.affinity = a.mode == "pinned"
    gw.rehome_every_turn = a.mode != "pinned"
    wl = Workload(seed=11)
    done_turns = {c: 0 for c in range(a.convs)}
    due = []
    finished = [0]
    t_start = time.monotonic()
    if rank == 0:
        for c in range(a.convs):
            heapq.heappush(due, (t_start + (c % 64) * 1e-3, c))

    def on_complete(m):
        c = m.metadata.get("_conv")
        if c is None:
            return
        done_turns[c] += 1
        finished[0] += 1
        if done_turns[c] < a.turns:
            heapq.heappush(due, (time.monotonic(), c))

    gw.on_complete = on_complete

    def pump():
        t = time.monotonic()
        batch = []
        while due and due[0][0] <= t:
            _, c = heapq.heappop(due)
            m = wl.make(1)[0]
            m.conversation_id = f"dlg-{c}"
            m.metadata["_conv"] = c
            m.arrival_ns = time.monotonic_ns()
            batch.append(m)
        if batch:
            gw.submit(batch)

    target = a.convs * a.turns
    tok0 = engine.total_tokens
    if not a.cpu:
        torch.cuda.synchronize()
    comm.barrier()
    t0 = time.perf_counter()
    while not gw.peers_stopping:
        if rank == 0 and (finished[0] >= target or time.perf_counter() - t0 > a.timeout_s):
            gw.request_stop()
        pump()
        gw.tick(pump=pump)
    if not a.cpu:
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    gw.flush_latency()
    st = np.array([engine.total_tokens - tok0, engine.kv_reused_tokens, engine.kv_imported,
                   gw.counters["kv_migrated"], gw.counters["kv_migrate_replays"], gw.counters["remote_sent"],
                   int(gw.migrator.bytes_sent) if gw.migrator is not None else 0,
                   int(gw.migrator.host_ns) if gw.migrator is not None else 0,
                   int(gw.migrator.ticks) if gw.migrator is not None else 0,
                   int(gw.migrator.host_max_ns) if gw.migrator is not None else 0], dtype=np.int64)
    rows = comm.all_gather_i64(st)
    agg = rows.sum(axis=0)
    lat = gw.rec_done.summary()
    if rank == 0:
        print(json.dumps({
            "bench": "re-homing: KV migration vs dialog replay", "mode": a.mode, "world": W,
            "model": a.model, "convs": a.convs, "turns": a.turns, "gen_tokens": a.gen_tokens,
            "turns_completed": finished[0], "seconds": round(el, 3), "turns_per_s": round(finished[0] / el, 1),
            "p50_turn_ms": round(lat["p50_ms"], 2), "p99_turn_ms": round(lat["p99_ms"], 2),
            "forward_tokens": int(agg[0]), "forward_tokens_per_turn": round(int(agg[0]) / max(1, finished[0]), 1),
            "kv_reused_tokens": int(agg[1]), "kv_imported": int(agg[2]), "kv_migrated": int(agg[3]),
            "migrate_replays": int(agg[4]), "remote_dispatched": int(agg[5]), "kv_bytes_moved": int(agg[6]),
            # host time inside KVMigrator.execute per migration tick (header
            # exchange + pack / enqueue or, on gloo, the staged copies), by rank
            "migrator_host_ms_per_tick_by_rank": [round(float(r[7]) / max(1, int(r[8])) / 1e6, 3) for r in rows],
            "migrator_host_ms_max_by_rank": [round(float(r[9]) / 1e6, 3) for r in rows],
            "migration_ticks_by_rank": [int(r[8]) for r in rows],
            "data_plane": "gloo (host staging; ranks share one GPU)" if not a.cpu else "gloo (CPU rehearsal)"}),
            flush=True)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
