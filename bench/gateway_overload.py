"""Gateway-only (null backend) behaviour past its capacity: served rate every
0.5 s and a cProfile of the serve loop, to find what grows with the backlog.

    python bench/gateway_overload.py --rate 200000 --seconds 4 [--cpu]
"""
from __future__ import annotations

import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--rate", type=float, default=200000.0)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--cpu", action="store_true", help="CPU oracle preprocess instead of the GPU pipeline")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    from llm_message_queue_amd.backend.null_engine import NullEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import PoissonArrivals, Workload
    from llm_message_queue_amd.preprocess.preprocessor import Preprocessor
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.enable_metrics = False
    pre = Preprocessor(cfg.preprocessor, use_gpu=not a.cpu, device="cpu" if a.cpu else "cuda:0")
    gw = Gateway(cfg, preprocessor=pre, engine=NullEngine(), use_gpu_preprocess=not a.cpu, prompt_cap=32,
                 gen_tokens=1)
    wl = Workload(seed=3)
    arr = PoissonArrivals(a.rate, seed=1)
    prof = cProfile.Profile()
    g0 = time.monotonic()
    arr.reset(g0)
    last, d_last, s_last = g0, 0, 0
    t_gen = t_tick = 0.0
    prof.enable()
    while time.monotonic() - g0 < a.seconds:
        t = time.perf_counter()
        due = arr.due(time.monotonic(), limit=8192)
        if due:
            msgs = wl.make(len(due))
            for m, ts in zip(msgs, due):
                m.arrival_ns = int(ts * 1e9)
            gw.submit(msgs)
        t2 = time.perf_counter()
        gw.tick()
        t3 = time.perf_counter()
        t_gen += t2 - t
        t_tick += t3 - t2
        now = time.monotonic()
        if now - last > 0.5:
            d, sub = gw.counters["dispatched"], gw.counters["submitted"]
            print(f"t={now - g0:4.1f}s submitted/s={(sub - s_last) / (now - last):8.0f} "
                  f"dispatched/s={(d - d_last) / (now - last):8.0f} queued={gw.pending():7d} "
                  f"inbox={gw.inbox_size():7d} gen={t_gen:.2f}s tick={t_tick:.2f}s", flush=True)
            last, d_last, s_last = now, d, sub
            t_gen = t_tick = 0.0
    prof.disable()
    pstats.Stats(prof).sort_stats("tottime").print_stats(a.top)


if __name__ == "__main__":
    main()
