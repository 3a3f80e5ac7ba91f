"""Long-dialog replay across the job's GPUs (BASELINE config 4: "conversation
state_manager with per-GPU KV-residency hints, long-dialog replay routed
across 8 GPUs").

One process per GPU (``--gpus N`` starts the ranks itself, as bench.py).
C concurrent conversations per router (``--ingress per-rank``) or C x N at
rank 0 alone (``--ingress rank0``, the `cli serve` topology: every
conversation turn enters the front door), T turns each, closed loop: a turn
is submitted when the conversation's previous turn completed.  Every turn's
prompt is its message in the context of the whole dialog so far:

  * ``residency`` -- conversation affinity: a turn goes to the GPU whose slot
    holds the dialog's KV (KV-residency pins in the plan) and prefills only
    its new tokens; a turn the plan places elsewhere (its home GPU full)
    moves the KV there (KV migration over the data plane, N11) instead of
    replaying the dialog;
  * ``replay`` -- no residency: every turn re-prefills the whole dialog on
    whatever GPU the plan picks (what a gateway without KV residency sends).

Reported per mode, job-wide and per rank: turns/s, turn latency, forward
tokens per turn, KV tokens reused, KV migrations and migration replays,
requests placed on another rank's GPU.  The reference keeps sessions sticky
to an endpoint (`internal/loadbalancer/load_balancer.go:501-558`) but has no
KV to keep.

    python bench/dialog_bench.py --gpus 8 [--convs 512 --turns 6]
    python bench/dialog_bench.py --gpus 8 --cpu-dry-run --sim-gpu 1,0.97,1.03   # CPU rehearsal
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402

from llm_message_queue_amd.utils.harness import comm_evidence, self_launch  # noqa: E402


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--convs", type=int, default=1024, help="conversations per router (rank0: x N at rank 0)")
    ap.add_argument("--turns", type=int, default=6)
    ap.add_argument("--slots", type=int, default=1536)
    ap.add_argument("--max-ctx", type=int, default=512)
    ap.add_argument("--token-budget", type=int, default=4096)
    ap.add_argument("--gen-tokens", type=int, default=16)
    ap.add_argument("--prompt-cap", type=int, default=32)
    ap.add_argument("--think-ms", type=float, default=0.0)
    ap.add_argument("--timeout-s", type=float, default=240.0)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--modes", default="residency,replay")
    ap.add_argument("--ingress", default="per-rank", choices=["per-rank", "rank0"])
    ap.add_argument("--lb", default="least_connections")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--cpu-dry-run", action="store_true",
                    help="rehearse on CPU (gloo, tiny model unless --sim-gpu); not a measurement")
    ap.add_argument("--sim-gpu", default="",
                    help="with --cpu-dry-run: per-rank relative GPU speeds (SimEngine at the serving config)")
    ap.add_argument("--control-plane", default="shm", choices=["shm", "gloo", "nccl"])
    ap.add_argument("--cpu-bind", default="auto", choices=["auto", "gpu", "core", "off"],
                    help="host placement of each rank (parallel/placement.py; auto = its GPU's socket cores "
                         "when the job has more than one rank)")
    return ap.parse_args(argv)


def main(argv=None) -> int:
    a = parse(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and a.gpus > 1:
        return self_launch(a, argv, __file__)
    if env_world is not None and int(env_world) != a.gpus:
        print(f"dialog_bench: --gpus {a.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        return 3
    import torch

    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.backend.slot_page import SlotPage
    from llm_message_queue_amd.balancer.load_balancer import Endpoint, LoadBalancer
    from llm_message_queue_amd.gateway.router import Gateway, LatencyRecorder
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.parallel.comm import init_from_env, local_device_index
    from llm_message_queue_amd.preprocess.preprocessor import Preprocessor
    from llm_message_queue_amd.utils.config import default_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dry = a.cpu_dry_run
    if dry:
        dev = torch.device("cpu")
        comm = init_from_env(backend="gloo", control="gloo" if a.control_plane == "nccl" else a.control_plane)
        if not a.sim_gpu:
            a.model, a.slots, a.max_ctx, a.token_budget, a.prompt_cap = "tiny", 32, 128, 256, 12
            a.gen_tokens = min(a.gen_tokens, 4)
            a.convs = min(a.convs, 16)
    else:
        if not torch.cuda.is_available():
            print("dialog_bench needs a GPU (or --cpu-dry-run)", file=sys.stderr)
            return 2
        local = local_device_index()
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        from llm_message_queue_amd.parallel.placement import bind_rank
        binding = bind_rank(a.cpu_bind)              # this rank's threads on its GPU's socket
        comm = init_from_env(control=a.control_plane)
    evidence = comm_evidence(comm, dev, world, dry, binding=None if dry else binding)

    def dsync():
        if not dry:
            torch.cuda.synchronize(dev)

    cfg = default_config()
    cfg.queue.enable_metrics = False
    cfg.backend.max_ctx = a.max_ctx
    cfg.loadbalancer.algorithm = a.lb
    cfg.loadbalancer.health_check_interval = 0
    for lv in cfg.queue.levels:
        lv.max_concurrent = a.slots * world
    job = os.environ.get("TORCHELASTIC_RUN_ID", str(os.getpid() if world == 1 else "dlg"))
    page = SlotPage(f"dlg{job}", rank)
    if dry and a.sim_gpu:
        from llm_message_queue_amd.backend.sim_engine import SimEngine
        speeds = [float(x) for x in a.sim_gpu.split(",")]
        engine = SimEngine(speed=speeds[rank % len(speeds)], slots=a.slots, max_ctx=a.max_ctx,
                           token_budget=a.token_budget, page=page, gpu_index=rank, seed=1234)
    else:
        # replicas of ONE model: identical weights on every GPU (a migrated KV
        # is only meaningful against the same weights)
        engine = BackendEngine(LlamaConfig.by_name(a.model), slots=a.slots, max_ctx=a.max_ctx,
                               token_budget=a.token_budget, device=dev, impl="ref" if dry else "hip", seed=1234,
                               page=page, gpu_index=rank)
    engine.warm_shapes()
    pre = Preprocessor(cfg.preprocessor, use_gpu=not dry, device=str(dev))
    lb = LoadBalancer(cfg.loadbalancer)
    for j in range(world):
        lb.add_endpoint(Endpoint(id=f"gpu{j}", type="llm", gpu_index=j, page=page if j == rank else None,
                                 max_connections=a.slots))
    gw = Gateway(cfg, preprocessor=pre, engine=engine, comm=comm, load_balancer=lb, use_gpu_preprocess=not dry,
                 prompt_cap=a.prompt_cap, gen_tokens=a.gen_tokens)
    wl = Workload(seed=5 + rank)
    my_convs = (a.convs * world if rank == 0 else 0) if a.ingress == "rank0" else a.convs

    def run_mode(mode: str, convs: int, turns: int, tag: str) -> dict:
        residency = mode == "residency"
        gw.kv_residency = residency
        gw.affinity = residency
        gw.kv_migrate = residency and bool(cfg.gpu.kv_migration)   # replay: never move a dialog's KV
        gw.conv_home.clear()
        gw.conv_hist.clear()
        gw.reset_latency()
        done_turns = {c: 0 for c in range(convs)}
        due = []
        t_start = time.monotonic()
        for c in range(convs):
            heapq.heappush(due, (t_start + (c % 64) * 1e-3, c))
        finished = [0]

        def on_complete(m):
            c = m.metadata.get("_conv")
            if c is None or not str(m.conversation_id).startswith(tag):
                return
            done_turns[c] += 1
            finished[0] += 1
            if done_turns[c] < turns:
                heapq.heappush(due, (time.monotonic() + a.think_ms / 1e3, c))

        gw.on_complete = on_complete

        def pump():
            t = time.monotonic()
            batch = []
            while due and due[0][0] <= t:
                _, c = heapq.heappop(due)
                m = wl.make(1)[0]
                m.conversation_id = f"{tag}-{rank}-{c}"
                m.metadata["_conv"] = c
                m.arrival_ns = time.monotonic_ns()
                batch.append(m)
            if batch:
                gw.submit(batch)

        keys = ("kv_migrated", "kv_migrate_replays", "remote_sent", "remote_recv", "dispatched",
                "dialog_ids_real", "dialog_ids_placeholder", "hist_tokens_sent", "hist_tokens_recv")
        c0 = {k: gw.counters[k] for k in keys}
        tok0, reuse0, imp0 = engine.total_tokens, engine.kv_reused_tokens, engine.kv_imported
        rp0 = (getattr(engine, "replay_tokens", 0), getattr(engine, "replay_nonzero", 0))
        bytes0 = gw.migrator.bytes_sent if gw.migrator is not None else 0
        dsync()
        comm.barrier()
        t0 = time.perf_counter()
        target = convs * turns
        while True:
            pump()
            gw.tick(pump=pump)
            if engine.inflight() == 0 and gw.pending() == 0 and due and due[0][0] > time.monotonic():
                time.sleep(min(due[0][0] - time.monotonic(), 0.002))
            # the run ends on every rank at the same tick (each tick is a collective)
            left = 0 if (finished[0] >= target or time.perf_counter() - t0 > a.timeout_s) else 1
            busy = engine.inflight() + gw.pending() + len(gw.remote_out) + gw.awaiting_kv()
            if comm.all_gather_i64(np.array([left + busy], dtype=np.int64)).max() == 0:
                break
        dsync()
        el = time.perf_counter() - t0
        gw.flush_latency()
        row = [finished[0], engine.total_tokens - tok0, engine.kv_reused_tokens - reuse0,
               engine.kv_imported - imp0,
               (gw.migrator.bytes_sent - bytes0) if gw.migrator is not None else 0] \
            + [gw.counters[k] - c0[k] for k in keys] \
            + [getattr(engine, "replay_tokens", 0) - rp0[0], getattr(engine, "replay_nonzero", 0) - rp0[1]] \
            + [target, int(el * 1e6)]
        rows = comm.all_gather_i64(np.array(row, dtype=np.int64))
        done = comm.all_gather_i64(gw.rec_done.arr.reshape(-1)).sum(axis=0).reshape(gw.rec_done.arr.shape)
        lat = LatencyRecorder(len(gw.tiers)).summary(done, done)
        tot = rows.sum(axis=0)
        elapsed = rows[:, -1].max() / 1e6
        return {"mode": mode, "turns_completed": int(tot[0]), "turns_offered": int(tot[-2]),
                "seconds": round(elapsed, 3), "turns_per_s": round(int(tot[0]) / elapsed, 1),
                "forward_tokens_per_turn": round(int(tot[1]) / max(1, int(tot[0])), 1),
                "kv_reused_tokens": int(tot[2]), "kv_imported": int(tot[3]), "kv_bytes_moved": int(tot[4]),
                **{k: int(tot[5 + i]) for i, k in enumerate(keys)},
                # real dialog context: replayed history tokens and how many are
                # not 0 (the round-5 placeholders were all 0)
                "replay_history_tokens": int(tot[5 + len(keys)]),
                "replay_history_nonzero": int(tot[6 + len(keys)]),
                "p50_turn_ms": round(lat["p50_ms"], 2), "p99_turn_ms": round(lat["p99_ms"], 2),
                "by_rank": {"turns_completed": rows[:, 0].tolist(), "forward_tokens": rows[:, 1].tolist(),
                            "kv_reused_tokens": rows[:, 2].tolist(),
                            **{k: rows[:, 5 + i].tolist() for i, k in enumerate(keys)}}}

    run_mode("residency", min(my_convs, 64), 2, "warm")            # kernels, allocator, first shapes
    modes = {m: run_mode(m, my_convs, a.turns, f"d{k}") for k, m in enumerate(a.modes.split(","))}
    out = {"bench": "long-dialog replay across GPUs" + (" (CPU rehearsal, not a measurement)" if dry else ""),
           "n_gpus": world, "model": a.model if not (dry and a.sim_gpu) else "sim-8b (SimEngine)",
           "sim_gpu": a.sim_gpu or None, "ingress": a.ingress, "convs_per_router": a.convs,
           "turns": a.turns, "gen_tokens": a.gen_tokens, "slots": a.slots, "placement": a.lb,
           "data_plane": evidence.get("data_backend"), "comm": evidence, "modes": modes}
    if "residency" in modes and "replay" in modes:
        out["speedup_turns_per_s"] = round(modes["residency"]["turns_per_s"]
                                           / max(1e-9, modes["replay"]["turns_per_s"]), 2)
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as fh:
                fh.write(line + "\n")
    page.close(unlink=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
