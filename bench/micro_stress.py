#!/usr/bin/env python3
"""Realtime micro-forwards under load: does a micro-forward stream running
next to the serving steps complete (no cross-stream stall), and how long does
a micro-forward take while the big steps run?

Drives ``BackendEngine`` (Llama-3-8B stub) directly: the serving pool is kept
saturated (4,096-token steps), and realtime requests arrive at ``--rt-rate``
per second into the micro pool.  Every ``--report-s`` seconds it prints one
JSON line (steps, micro-forwards, mean device ms of each, realtime
admission -> last token p50/p99); a forward incomplete after
``--step-timeout`` seconds ends the run with BackendHung (exit 3).

    python bench/micro_stress.py --stream high --blas lt --seconds 40
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--stream", default="high", choices=["high", "same", "partition"])
    ap.add_argument("--micro-cus", type=int, default=64)
    ap.add_argument("--micro-gemm", default="hip", choices=["hip", "rocblas"])
    ap.add_argument("--budget", type=int, default=4096)
    ap.add_argument("--slots", type=int, default=1536)
    ap.add_argument("--blas", default="", choices=["", "lt", "rocblas"],
                    help="library GEMM backend for F.linear / addmm (torch preferred_blas_library)")
    ap.add_argument("--mode", default="micro", choices=["micro", "off"])
    ap.add_argument("--seconds", type=float, default=40.0)
    ap.add_argument("--rt-rate", type=float, default=560.0)
    ap.add_argument("--micro-inflight", type=int, default=1)
    ap.add_argument("--step-timeout", type=float, default=15.0)
    ap.add_argument("--report-s", type=float, default=5.0)
    ap.add_argument("--no-graph", action="store_true", help="decode micro-forwards launched eagerly (no HIP graphs)")
    a = ap.parse_args()
    import numpy as np
    import torch

    from llm_message_queue_amd.backend.engine import BackendEngine, BackendHung, Request
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    if a.blas:
        torch.backends.cuda.preferred_blas_library("cublaslt" if a.blas == "lt" else "cublas")
    dev = torch.device("cuda", 0)
    eng = BackendEngine(LlamaConfig.llama3_8b(), slots=a.slots, max_ctx=512, token_budget=a.budget, device=dev,
                        impl="hip", realtime_mode=a.mode, micro_stream=a.stream, micro_cus=a.micro_cus, micro_gemm=a.micro_gemm,
                        micro_inflight=a.micro_inflight, step_timeout_s=a.step_timeout, micro_graph=not a.no_graph)
    eng.warm_shapes()
    eng.time_steps = True
    rng = np.random.default_rng(0)
    rid = [0]

    def req(tier):
        rid[0] += 1
        return Request(req_id=rid[0], prompt=rng.integers(0, 128000, size=int(rng.integers(8, 24))).astype(np.int32),
                       gen_tokens=4, tier=tier)

    t0 = time.monotonic()
    t_rep = t0
    rt_next = [t0]
    lat = []

    def rt_poll() -> bool:
        """Realtime arrivals due now are admitted (micro pool) and the
        micro-forwards pumped / reaped while the serving step runs."""
        now = time.monotonic()
        rts = []
        while rt_next[0] <= now:
            rts.append(req(0))
            rt_next[0] += rng.exponential(1.0 / a.rt_rate)
        for r in rts:
            r.meta = time.monotonic_ns()
        if rts:
            eng.admit(rts)
        n = eng.pump_micro()
        res = eng.finish_micro()
        t = time.monotonic_ns()
        for r in res.completed:
            if r.tier == 0 and isinstance(r.meta, int):
                lat.append((t - r.meta) / 1e6)
        return bool(rts or n or res.completed)

    try:
        while time.monotonic() - t0 < a.seconds:
            rt_poll()
            cap = eng.admit_capacity()
            if cap:
                eng.admit([req(2) for _ in range(cap)])
            eng.launch(wait_cb=rt_poll)
            rt_poll()
            res = eng.finish()
            t_done = time.monotonic_ns()
            for r in res.completed:
                if r.tier == 0 and isinstance(r.meta, int):
                    lat.append((t_done - r.meta) / 1e6)
            if time.monotonic() - t_rep >= a.report_s:
                t_rep = time.monotonic()
                la = np.asarray(lat) if lat else np.zeros(1)
                print(json.dumps({"t_s": round(t_rep - t0, 1), "steps": eng.gpu_steps,
                                  "step_ms": round(eng.gpu_step_ms / max(1, eng.gpu_steps), 2),
                                  "micro": eng.micro_timed,
                                  "micro_ms": round(eng.micro_gpu_ms / max(1, eng.micro_timed), 2),
                                  "rt_done": len(lat), "rt_p50_ms": round(float(np.percentile(la, 50)), 1),
                                  "rt_p99_ms": round(float(np.percentile(la, 99)), 1),
                                  "tok_s": round(eng.total_tokens / (t_rep - t0), 0),
                                  "graph_steps": eng.micro_graph_steps}), flush=True)
        eng.finish(block=True)
        eng.close()
        if a.stream == "partition":
            from llm_message_queue_amd.backend.cu_partition import release_streams
            del eng, res
            release_streams()
    except BackendHung as e:
        print(json.dumps({"hung": str(e), "t_s": round(time.monotonic() - t0, 1), "micro": eng.micro_steps}),
              flush=True)
        return 3
    return 0


if __name__ == "__main__":
    sys.exit(main())
