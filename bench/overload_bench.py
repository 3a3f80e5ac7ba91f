"""Sustained overload (BASELINE config 5: "dead-letter + delayed_queue under
sustained overload").

Offers Poisson load at ``--overload`` x the backend's calibrated capacity for
``--seconds``, with every request carrying a ``--deadline-ms`` timeout and
every tier queue bounded at ``--queue-max``.  Reports what a production
gateway must show under overload:

  * goodput: requests/s served by the 8B backend (should stay at capacity);
  * shedding: requests rejected at ingress (queue full, 503) and requests
    expired in the queue (deadline passed -> dead-letter queue, status
    ``timeout``), per tier -- strict priority + aging should shed the low
    tiers first and keep serving realtime;
  * latency of the SERVED requests (arrival -> dispatch, arrival -> last
    token) per tier: bounded by the deadline, not by the backlog;
  * ordering: each run compares FIFO within a tier (the reference's order)
    with adaptive LIFO (``queue.adaptive_lifo``: an overloaded tier serves
    its newest request, the stale head is shed at its deadline);
  * failures: ``--fault-every N`` injects a backend launch failure every N
    ticks; the evacuated in-flight requests are re-queued (and shed to the
    DLQ like any other request if their deadline passes).

    python bench/overload_bench.py [--overload 1.5 --seconds 20]
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--slots", type=int, default=1536)
    ap.add_argument("--max-ctx", type=int, default=512)
    ap.add_argument("--token-budget", type=int, default=4096)
    ap.add_argument("--prompt-cap", type=int, default=32)
    ap.add_argument("--gen-tokens", type=int, default=4)
    ap.add_argument("--overload", type=float, default=1.5, help="offered load / calibrated capacity")
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--deadline-ms", type=float, default=1000.0, help="per-request timeout (queue deadline)")
    ap.add_argument("--queue-max", type=int, default=10000, help="per-tier queue bound (QUEUE_FULL beyond)")
    ap.add_argument("--fault-every", type=int, default=0, help="inject a backend launch fault every N ticks")
    ap.add_argument("--policies", default="fifo,adaptive_lifo", help="comma list: fifo, adaptive_lifo")
    ap.add_argument("--lifo-after-ms", type=float, default=0.0,
                    help="adaptive LIFO threshold (0 = each tier's aging deadline)")
    ap.add_argument("--json-out", default="")
    ap.add_argument("--cpu", action="store_true", help="control-flow check on CPU (tiny model); not a measurement")
    a = ap.parse_args()
    import numpy as np
    import torch

    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import PoissonArrivals, Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.preprocess.preprocessor import Preprocessor
    from llm_message_queue_amd.queue.dead_letter import DeadLetterQueue
    from llm_message_queue_amd.utils.config import default_config

    dev = torch.device("cpu") if a.cpu else torch.device("cuda", 0)
    if a.cpu:
        a.model, a.slots, a.max_ctx, a.token_budget, a.prompt_cap = "tiny", 16, 64, 128, 16
    sync = (lambda: None) if a.cpu else torch.cuda.synchronize
    cfg = default_config()
    cfg.queue.enable_metrics = False
    cfg.queue.default_max_size = a.queue_max
    for lv, ms in zip(sorted(cfg.queue.levels, key=lambda lv: lv.priority), (50, 100, 150, 200)):
        lv.max_concurrent = a.slots
        lv.max_wait_time = int(ms * 1e6)
    engine = BackendEngine(LlamaConfig.by_name(a.model), slots=a.slots, max_ctx=a.max_ctx,
                           token_budget=a.token_budget, device=dev, impl="ref" if a.cpu else "hip")
    pre = Preprocessor(cfg.preprocessor, use_gpu=not a.cpu, device=str(dev))
    dlq = DeadLetterQueue()
    gw = Gateway(cfg, preprocessor=pre, engine=engine, use_gpu_preprocess=not a.cpu, prompt_cap=a.prompt_cap,
                 gen_tokens=a.gen_tokens, dead_letter=dlq)
    wl = Workload(seed=11)
    ntier = len(gw.tiers)

    # ---- calibrate (saturated, as bench.py)
    for i in range(80):
        need = max(0, 2 * a.slots - gw.pending() - engine.inflight())
        if need:
            gw.submit(wl.make(need))
        gw.tick()
        if i == 19:
            sync()
            t0, tok0, rt0, d0 = time.perf_counter(), engine.total_tokens, engine.completed_tokens, engine.completed_total
    sync()
    t1 = time.perf_counter()
    cap = (engine.total_tokens - tok0) / (t1 - t0) / max(1.0, (engine.completed_tokens - rt0)
                                                          / max(1, engine.completed_total - d0))
    gw.drop_pending()
    while engine.inflight() or gw.pending():
        gw.tick()
    rate = a.overload * cap

    # ---- overload phases: FIFO within a tier (the reference's order), then adaptive LIFO
    deadline_ns = int(a.deadline_ms * 1e6)
    lifo = [int(a.lifo_after_ms * 1e6) if a.lifo_after_ms > 0 else int(lv.max_wait_time)
            for lv in sorted(cfg.queue.levels, key=lambda lv: lv.priority)]

    def phase(policy: str, seed: int) -> dict:
        gw.lifo_ns = lifo if policy == "adaptive_lifo" else None
        served_tier = np.zeros(ntier, dtype=np.int64)
        expired_tier = np.zeros(ntier, dtype=np.int64)
        gw.on_complete = lambda m: served_tier.__setitem__(m.tier, served_tier[m.tier] + 1)

        def on_expire(m):
            t = gw.tier_of_queue.get(m.queue_name, ntier - 1)
            expired_tier[t] += 1
        gw.on_expire = on_expire
        gw.rec.reset()
        gw.rec_done.reset()
        c0 = dict(gw.counters)
        d0 = dlq.size()
        arrivals = PoissonArrivals(rate, seed=seed)
        faults = 0
        gc.collect()
        gc.freeze()
        gc.disable()
        start = time.monotonic()
        arrivals.reset(start)

        def pump():
            due = arrivals.due(time.monotonic())
            if due:
                msgs = wl.make(len(due))
                for m, ts in zip(msgs, due):
                    m.arrival_ns = int(ts * 1e9)
                    m.timeout = deadline_ns
                gw.submit(msgs)

        ticks = 0
        while time.monotonic() - start < a.seconds:
            pump()
            if a.fault_every and ticks and ticks % a.fault_every == 0:
                engine.inject(fail_launch=1)
                faults += 1
            gw.tick(pump=pump)
            if not gw.healthy:          # an injected fault evacuated the backend: bring it back
                gw.set_healthy(True)
            ticks += 1
        elapsed = time.monotonic() - start
        gc.enable()
        c1 = gw.counters
        lat = gw.rec.summary()
        gw.flush_latency()
        done = gw.rec_done.summary()
        res = {
            "policy": policy, "seconds": round(elapsed, 2),
            "goodput_rps": round((c1["completed"] - c0["completed"]) / elapsed, 1),
            "dispatched_rps": round((c1["dispatched"] - c0["dispatched"]) / elapsed, 1),
            "submitted": c1["submitted"] - c0["submitted"],
            "rejected_queue_full": c1["rejected"] - c0["rejected"],
            "expired_to_dlq": c1["expired"] - c0["expired"], "dlq_added": dlq.size() - d0,
            "served_by_tier": served_tier.tolist(), "expired_by_tier": expired_tier.tolist(),
            "served_p50_arrival_to_dispatch_ms": round(lat["p50_ms"], 1),
            "served_p99_arrival_to_dispatch_ms_by_tier": [round(x, 1) for x in lat["p99_by_tier_ms"]],
            "served_p99_e2e_ms_by_tier": [round(x, 1) for x in done["p99_by_tier_ms"]],
            "served_p50_e2e_ms": round(done["p50_ms"], 1),
            "faults_injected": faults, "evacuated": c1["evacuated"] - c0["evacuated"],
        }
        # drain between phases (untimed): drop the backlog, finish in-flight work
        gw.drop_pending()
        while engine.inflight() or gw.pending():
            gw.tick()
        return res

    phases = [phase(p, 3 + i) for i, p in enumerate(a.policies.split(","))]
    out = {
        "bench": "sustained overload" + (" (CPU control-flow check, not a measurement)" if a.cpu else ""),
        "model": a.model, "slots": a.slots,
        "calibrated_capacity_rps": round(cap, 1), "offered_rps": round(rate, 1), "overload": a.overload,
        "deadline_ms": a.deadline_ms, "queue_max_per_tier": a.queue_max, "lifo_after_ns": lifo,
        "phases": phases,
    }
    line = json.dumps(out)
    print(line, flush=True)
    if a.json_out:
        with open(a.json_out, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
