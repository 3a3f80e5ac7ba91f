"""Sustained overload across the job's GPUs (BASELINE config 5: "dead-letter
+ delayed_queue under sustained overload; resource_scheduler dynamic worker
rebalancing across 8 GPUs").

One process per GPU (``--gpus N`` starts the ranks itself, as bench.py), each
rank a router + backend, the per-tick load exchange and plan of the serving
bench.  Every rank offers Poisson load at ``--overload`` x the calibrated
per-GPU capacity, every request carrying a ``--deadline-ms`` timeout, every
tier queue bounded at ``--queue-max``.  Reported per phase, job-wide and per
rank:

  * goodput (requests/s served by the backends; should stay at capacity);
  * shedding per tier: requests rejected at ingress (queue full) and expired
    in the queue (deadline passed -> dead-letter queue, status ``timeout``) --
    strict priority + aging must shed the low tiers and serve realtime and
    high in full;
  * latency of the SERVED requests per tier (bounded by the deadline);
  * retries: ``--fault-every N`` injects a backend launch failure on one rank
    every N ticks; its in-flight requests wait out ``queue.retry``'s backoff
    in the delayed queue and return to their tier, or go to the dead-letter
    queue once their retries are spent (the reference's intended retry path,
    `internal/priorityqueue/worker.go:202-239`);
  * accounting: every offered request ends completed, rejected, shed or
    dead-lettered -- none lost.

``--autoscale`` then runs load steps (e.g. ``1.5:6,0.1:6,1.5:6`` = 6 s at
1.5x, 6 s at 0.1x, 6 s at 1.5x) with rank 0's ResourceScheduler acting on
the job (`internal/scheduler/resource_scheduler.go:525-571`): a light load
parks a GPU (its endpoint leaves placement on every rank), the return of the
overload -- queued demand no active GPU has room for -- unparks it.

    python bench/overload_bench.py --gpus 8 [--overload 1.5 --seconds 10]
    python bench/overload_bench.py --gpus 8 --cpu-dry-run --sim-gpu 1,0.97,1.03   # CPU rehearsal
"""
from __future__ import annotations

import argparse
import gc
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
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--slots", type=int, default=1536)
    ap.add_argument("--max-ctx", type=int, default=512)
    ap.add_argument("--token-budget", type=int, default=4096)
    ap.add_argument("--prompt-cap", type=int, default=32)
    ap.add_argument("--gen-tokens", type=int, default=4)
    ap.add_argument("--overload", type=float, default=1.5, help="offered load / calibrated capacity (per GPU)")
    ap.add_argument("--seconds", type=float, default=10.0, help="per policy phase")
    ap.add_argument("--deadline-ms", type=float, default=1000.0, help="per-request timeout (queue deadline)")
    ap.add_argument("--queue-max", type=int, default=10000, help="per-tier queue bound (QUEUE_FULL beyond)")
    ap.add_argument("--fault-every", type=int, default=0, help="inject a backend launch fault every N ticks")
    ap.add_argument("--fault-rank", type=int, default=1, help="the rank whose backend the faults hit")
    ap.add_argument("--retry-backoff-ms", type=float, default=50.0, help="backoff of a backend-failure retry")
    ap.add_argument("--max-retries", type=int, default=2)
    ap.add_argument("--policies", default="fifo,adaptive_lifo", help="comma list: fifo, adaptive_lifo")
    ap.add_argument("--lifo-after-ms", type=float, default=0.0,
                    help="adaptive LIFO threshold (0 = each tier's aging deadline)")
    ap.add_argument("--autoscale", default="",
                    help="load steps 'mult:seconds,...' run with the resource scheduler acting (e.g. "
                         "1.5:6,0.1:6,1.5:6); empty = skip")
    ap.add_argument("--scale-cooldown-s", type=float, default=1.0)
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
        print(f"overload_bench: --gpus {a.gpus} but WORLD_SIZE={env_world}", file=sys.stderr)
        return 3
    import torch

    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.backend.slot_page import SlotPage
    from llm_message_queue_amd.balancer.load_balancer import Endpoint, LoadBalancer
    from llm_message_queue_amd.gateway.router import Gateway, LatencyRecorder
    from llm_message_queue_amd.gateway.workload import PoissonArrivals, Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.parallel.comm import init_from_env, local_device_index
    from llm_message_queue_amd.preprocess.preprocessor import Preprocessor
    from llm_message_queue_amd.queue.dead_letter import DeadLetterQueue
    from llm_message_queue_amd.queue.delayed import DelayedQueue
    from llm_message_queue_amd.queue.worker import FixedBackoff
    from llm_message_queue_amd.scheduler.resource_scheduler import ResourceScheduler, ResourceSchedulerConfig
    from llm_message_queue_amd.utils.config import default_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dry = a.cpu_dry_run
    if dry:
        dev = torch.device("cpu")
        comm = init_from_env(backend="gloo", control="gloo" if a.control_plane == "nccl" else a.control_plane)
        if not a.sim_gpu:
            a.model, a.slots, a.max_ctx, a.token_budget, a.prompt_cap = "tiny", 16, 64, 128, 16
    else:
        if not torch.cuda.is_available():
            print("overload_bench needs a GPU (or --cpu-dry-run)", file=sys.stderr)
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
    cfg.queue.default_max_size = a.queue_max
    for lv, ms in zip(sorted(cfg.queue.levels, key=lambda lv: lv.priority), (50, 100, 150, 200)):
        lv.max_concurrent = a.slots * world
        lv.max_wait_time = int(ms * 1e6)
    job = os.environ.get("TORCHELASTIC_RUN_ID", str(os.getpid() if world == 1 else "ovl"))
    page = SlotPage(f"ovl{job}", rank)
    if dry and a.sim_gpu:
        from llm_message_queue_amd.backend.sim_engine import SimEngine
        speeds = [float(x) for x in a.sim_gpu.split(",")]
        engine = SimEngine(speed=speeds[rank % len(speeds)], slots=a.slots, max_ctx=a.max_ctx,
                           token_budget=a.token_budget, page=page, gpu_index=rank, seed=1000 + rank)
    else:
        engine = BackendEngine(LlamaConfig.by_name(a.model), slots=a.slots, max_ctx=a.max_ctx,
                               token_budget=a.token_budget, device=dev, impl="ref" if dry else "hip",
                               seed=1000 + rank, page=page, gpu_index=rank)
    pre = Preprocessor(cfg.preprocessor, use_gpu=not dry, device=str(dev))
    lbcfg = cfg.loadbalancer
    lbcfg.algorithm = a.lb
    lbcfg.health_check_interval = 0
    lb = LoadBalancer(lbcfg)
    for j in range(world):
        lb.add_endpoint(Endpoint(id=f"gpu{j}", type="llm", gpu_index=j, page=page if j == rank else None,
                                 max_connections=a.slots))
    dlq = DeadLetterQueue()
    gw = Gateway(cfg, preprocessor=pre, engine=engine, comm=comm, load_balancer=lb, use_gpu_preprocess=not dry,
                 prompt_cap=a.prompt_cap, gen_tokens=a.gen_tokens, dead_letter=dlq)
    delayed = DelayedQueue()                 # polled by the tick (no drain thread)
    gw.attach_retry_queue(delayed, FixedBackoff(int(a.retry_backoff_ms * 1e6), a.max_retries))
    wl = Workload(seed=11 + rank)
    ntier = len(gw.tiers)
    engine.warm_shapes()

    def busy_local() -> int:
        return (engine.inflight() + engine.queued_steps() + len(gw.remote_out) + gw.pending() + gw.inbox_size()
                + sum(len(v) for v in gw._done_owed.values()) + gw.preprocessing() + gw.awaiting_kv()
                + gw.retrying())

    def drain(drop: bool) -> None:
        if drop:
            gw.drop_pending()
        busy = comm.all_gather_i64(np.array([busy_local()], dtype=np.int64))
        n = 0
        while busy.max() > 0 and n < 5000:
            gw.tick()
            n += 1
            busy = comm.all_gather_i64(np.array([busy_local()], dtype=np.int64))

    # ---- calibrate (saturated, fixed tick counts on every rank: each tick is a collective)
    for i in range(80):
        need = max(0, 2 * a.slots - gw.pending() - engine.inflight())
        if need:
            gw.submit(wl.make(need))
        gw.tick()
        if i == 19:
            dsync()
            t0, tok0, rt0, d0 = time.perf_counter(), engine.total_tokens, engine.completed_tokens, engine.completed_total
    dsync()
    t1 = time.perf_counter()
    cap_local = (engine.total_tokens - tok0) / (t1 - t0) / max(1.0, (engine.completed_tokens - rt0)
                                                               / max(1, engine.completed_total - d0))
    cap = float(comm.all_gather_i64(np.array([int(cap_local * 1000)], dtype=np.int64))[:, 0].mean() / 1000.0)
    drain(drop=True)

    deadline_ns = int(a.deadline_ms * 1e6)
    lifo = [int(a.lifo_after_ms * 1e6) if a.lifo_after_ms > 0 else int(lv.max_wait_time)
            for lv in sorted(cfg.queue.levels, key=lambda lv: lv.priority)]
    served_tier = np.zeros(ntier, dtype=np.int64)
    expired_tier = np.zeros(ntier, dtype=np.int64)

    def on_complete(m):
        served_tier[m.tier] += 1

    def on_expire(m):
        expired_tier[gw.tier_of_queue.get(m.queue_name, ntier - 1)] += 1

    gw.on_complete = on_complete
    gw.on_expire = on_expire
    KEYS = ("submitted", "completed", "dispatched", "rejected", "expired", "retried", "retry_exhausted",
            "evacuated", "handed_back", "remote_sent")

    def run(steps, seed: int, policy: str, rs=None) -> dict:
        """Serve ``steps`` = [(load multiplier, seconds)] back to back; one
        report per step (job-wide sums and per-rank rows)."""
        gw.lifo_ns = lifo if policy == "adaptive_lifo" else None
        out = []
        arrivals = PoissonArrivals(0.0, seed=seed * 100 + rank)
        gc.collect()
        gc.freeze()
        gc.disable()

        def pump():
            due = arrivals.due(time.monotonic())
            if due:
                msgs = wl.make(len(due))
                for m, ts in zip(msgs, due):
                    m.arrival_ns = int(ts * 1e9)
                    m.timeout = deadline_ns
                gw.submit(msgs)

        comm.barrier()
        for k, (mult, secs) in enumerate(steps):
            gw.reset_latency()
            c0 = {x: gw.counters[x] for x in KEYS}
            s0, e0, q0 = served_tier.copy(), expired_tier.copy(), dlq.size()
            ev0 = len(rs.scale_events) if rs is not None else 0
            start = time.monotonic()
            arrivals.reset(start, mult * cap)
            ticks = faults = 0
            while True:
                pump()
                if a.fault_every and rank == a.fault_rank % world and ticks and ticks % a.fault_every == 0:
                    engine.inject(fail_launch=1)
                    faults += 1
                gw.tick(pump=pump)
                if not gw.healthy:          # an injected fault evacuated the backend: bring it back
                    gw.set_healthy(True)
                ticks += 1
                # the phase ends on every rank at the same tick (each tick is a collective)
                if comm.all_gather_i64(np.array([time.monotonic() - start >= secs], dtype=np.int64)).max():
                    break
            el = time.monotonic() - start
            gw.flush_latency()
            row = [gw.counters[x] - c0[x] for x in KEYS] + (served_tier - s0).tolist() \
                + (expired_tier - e0).tolist() + [dlq.size() - q0, delayed.size(), faults, int(el * 1e6)]
            rows = comm.all_gather_i64(np.array(row, dtype=np.int64))
            lat = LatencyRecorder(ntier).summary(
                comm.all_gather_i64(gw.rec.arr.reshape(-1)).sum(axis=0).reshape(gw.rec.arr.shape),
                comm.all_gather_i64(gw.rec.enq.reshape(-1)).sum(axis=0).reshape(gw.rec.enq.shape))
            done = comm.all_gather_i64(gw.rec_done.arr.reshape(-1)).sum(axis=0).reshape(gw.rec_done.arr.shape)
            lat_d = LatencyRecorder(ntier).summary(done, done)
            nk = len(KEYS)
            tot = rows.sum(axis=0)
            elapsed = rows[:, -1].max() / 1e6
            rep = {"load": mult, "seconds": round(elapsed, 2), "offered_rps": round(mult * cap * world, 1),
                   "goodput_rps": round(int(tot[1]) / elapsed, 1),
                   **{x: int(tot[i]) for i, x in enumerate(KEYS)},
                   "served_by_tier": tot[nk:nk + ntier].tolist(),
                   "expired_to_dlq_by_tier": tot[nk + ntier:nk + 2 * ntier].tolist(),
                   "dlq_added": int(tot[nk + 2 * ntier]), "faults_injected": int(tot[nk + 2 * ntier + 2]),
                   "served_p99_arrival_to_dispatch_ms_by_tier": [round(x, 1) for x in lat["p99_by_tier_ms"]],
                   "served_p50_arrival_to_dispatch_ms": round(lat["p50_ms"], 1),
                   "served_p99_e2e_ms_by_tier": [round(x, 1) for x in lat_d["p99_by_tier_ms"]],
                   "by_rank": {x: rows[:, i].tolist() for i, x in enumerate(KEYS)}}
            rep["by_rank"]["dlq_added"] = rows[:, nk + 2 * ntier].tolist()
            rep["by_rank"]["delayed_at_end"] = rows[:, nk + 2 * ntier + 1].tolist()
            if rs is not None:
                ev = rs.scale_events[ev0:]
                rep["scale_events"] = [{"action": e["action"], "average_load": round(e["average_load"], 3),
                                        "pending": e["pending"]} for e in ev]
                rep["parked_at_end"] = list(rs.parked)
            out.append(rep)
        arrivals.rate = 0.0
        gc.enable()
        return out

    def accounting(c0) -> dict:
        acc = comm.all_gather_i64(np.array([gw.counters[x] - c0[x] for x in ("submitted", "completed", "rejected",
                                                                           "expired", "retry_exhausted")],
                                           dtype=np.int64)).sum(axis=0)
        return {"offered": int(acc[0]), "completed": int(acc[1]), "rejected": int(acc[2]), "shed": int(acc[3]),
                "dead_lettered_after_retries": int(acc[4]),
                "lost": int(acc[0] - acc[1] - acc[2] - acc[3] - acc[4])}

    results = {}
    for i, policy in enumerate(a.policies.split(",")):
        c0 = dict(gw.counters)
        rep = run([(a.overload, a.seconds)], 3 + i, policy)[0]
        drain(drop=False)            # finish (or shed at deadline) everything offered
        rep["policy"] = policy
        rep["requests_accounted"] = accounting(c0)
        results[policy] = rep
    auto = None
    if a.autoscale:
        steps = [(float(x.split(":")[0]), float(x.split(":")[1])) for x in a.autoscale.split(",")]
        rs = None
        if rank == 0:
            rs = ResourceScheduler(ResourceSchedulerConfig(
                enable_auto_scaling=True, scale_cooldown=int(a.scale_cooldown_s * 1e9), min_resources=1,
                max_resources=world, resource_check_period=100_000_000), start=True)
            rs._last_scale = time.monotonic()     # first decision after one cooldown (heartbeats in)
            gw.attach_resource_scheduler(rs, act=True)
        c0 = dict(gw.counters)
        auto = {"steps": run(steps, 17, "fifo", rs)}
        drain(drop=False)
        auto["requests_accounted"] = accounting(c0)
        if rs is not None:
            auto["scale_events"] = [dict(e, average_load=round(e["average_load"], 3)) for e in rs.scale_events]
            rs.stop()
        auto["scale_events"] = auto.get("scale_events") if rank == 0 else None
    out = {
        "bench": "sustained overload across GPUs" + (" (CPU rehearsal, not a measurement)" if dry else ""),
        "n_gpus": world, "model": a.model if not (dry and a.sim_gpu) else "sim-8b (SimEngine)",
        "sim_gpu": a.sim_gpu or None, "slots": a.slots, "calibrated_capacity_per_gpu_rps": round(cap, 1),
        "overload": a.overload, "deadline_ms": a.deadline_ms, "queue_max_per_tier": a.queue_max,
        "retry": {"backoff_ms": a.retry_backoff_ms, "max_retries": a.max_retries, "fault_every": a.fault_every,
                  "fault_rank": a.fault_rank % world},
        "lifo_after_ns": lifo, "comm": evidence, "policies": results, "autoscale": auto,
    }
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as fh:
                fh.write(line + "\n")
    page.close(unlink=True)
    delayed.close()
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
