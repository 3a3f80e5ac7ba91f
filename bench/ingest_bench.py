"""Gateway ingest cost (GPU preprocess + queue push) per message, with the GPU
idle and with the GPU saturated by a concurrent bf16 GEMM stream (what the
backend forward does to the preprocess side stream).

    python bench/ingest_bench.py [--sizes 64,256,1024,4096] [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="64,256,1024,4096")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--split", action="store_true",
                    help="time begin_batch / end_batch host work separately (the serve loop's async ingest: "
                         "the GPU wait is not on the host), plus a cProfile of both")
    ap.add_argument("--profile", action="store_true", help="with --split: cProfile the host work")
    a = ap.parse_args()
    import torch

    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.preprocess.preprocessor import Preprocessor
    from llm_message_queue_amd.utils.config import default_config

    cfg = default_config()
    pre = Preprocessor(cfg.preprocessor, use_gpu=True, device="cuda:0")
    wl = Workload(seed=3)
    busy = threading.Event()
    stop = threading.Event()

    def load():
        x = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
        w = torch.randn(28672, 4096, device="cuda", dtype=torch.bfloat16)
        while not stop.is_set():
            if busy.is_set():
                for _ in range(8):
                    torch.nn.functional.linear(x, w)
                torch.cuda.current_stream().synchronize()
            else:
                time.sleep(0.001)

    th = threading.Thread(target=load, daemon=True)
    th.start()
    if a.split:
        import cProfile
        import pstats
        for B in [int(s) for s in a.sizes.split(",")]:
            for mode in ("idle", "busy"):
                (busy.set if mode == "busy" else busy.clear)()
                time.sleep(0.05)
                pre.process_batch(wl.make(B), use_gpu=True, prompt_cap=32)
                tb = te = 0.0
                prof = cProfile.Profile() if a.profile else None
                for _ in range(a.reps):
                    msgs = wl.make(B)
                    t0 = time.perf_counter()
                    if prof:
                        prof.enable()
                    tok = pre.begin_batch(msgs, prompt_cap=32)
                    if prof:
                        prof.disable()
                    tb += time.perf_counter() - t0
                    while not pre.batch_ready(tok):
                        time.sleep(0.0002)
                    t0 = time.perf_counter()
                    if prof:
                        prof.enable()
                    pre.end_batch(tok)
                    if prof:
                        prof.disable()
                    te += time.perf_counter() - t0
                print(json.dumps({"batch": B, "gpu": mode, "begin_us": round(tb / a.reps * 1e6, 1),
                                  "end_us": round(te / a.reps * 1e6, 1),
                                  "host_us_per_msg": round((tb + te) / a.reps / B * 1e6, 2)}), flush=True)
                if prof:
                    st = pstats.Stats(prof)
                    print(f"--- cProfile B={B} {mode} (tottime, per 1 batch = /{a.reps})")
                    st.sort_stats("tottime").print_stats(14)
        stop.set()
        th.join(timeout=5)
        return
    for B in [int(s) for s in a.sizes.split(",")]:
        for mode in ("idle", "busy"):
            (busy.set if mode == "busy" else busy.clear)()
            time.sleep(0.05)
            pre.process_batch(wl.make(B), use_gpu=True, prompt_cap=32)    # warm
            t_py = t_gpu = 0.0
            for _ in range(a.reps):
                msgs = wl.make(B)
                g0 = pre.stats.get("gpu_ms_total", 0.0)
                t0 = time.perf_counter()
                pre.process_batch(msgs, use_gpu=True, prompt_cap=32)
                t_py += time.perf_counter() - t0
                t_gpu += pre.stats.get("gpu_ms_total", 0.0) - g0
            print(json.dumps({"batch": B, "gpu": mode, "total_us_per_msg": round(t_py / a.reps / B * 1e6, 2),
                              "pipeline_ms": round(t_gpu / a.reps, 3),
                              "batch_ms": round(t_py / a.reps * 1e3, 3)}), flush=True)
    stop.set()
    th.join(timeout=5)


if __name__ == "__main__":
    main()
