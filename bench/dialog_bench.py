"""Long-dialog replay (BASELINE config 4: "conversation state manager with
per-GPU KV-residency hints, long-dialog replay").

C concurrent conversations each run T turns, closed loop: a turn is submitted
when the conversation's previous turn completed.  Every turn's prompt is its
message (GPU tokenizer, <= --prompt-cap tokens) in the context of the whole
dialog so far, so the backend must attend over the dialog:

  * residency ON  -- the turn goes to the GPU whose slot still holds the
    dialog's KV (conversation affinity) and prefills only its new tokens;
  * residency OFF -- the dialog is replayed: all previous tokens are
    prefilled again with the new ones (what a gateway without KV residency
    has to send).

Both modes run back to back on the same engine; prints one JSON line.

    python bench/dialog_bench.py [--convs 1024 --turns 6]
"""
from __future__ import annotations

import argparse
import heapq
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_mode(gw, engine, wl, convs, turns, residency, think_s, timeout_s, tag):
    import torch
    gw.kv_residency = residency
    gw.conv_home.clear()
    gw.conv_hist.clear()
    gw.rec_done.reset()
    done_turns = {}
    due = []                                  # (time, conv index)
    now = time.monotonic()
    for c in range(convs):
        heapq.heappush(due, (now + (c % 64) * 1e-3, c))
        done_turns[c] = 0
    finished = [0]

    def on_complete(m):
        c = m.metadata.get("_conv")
        if c is None:
            return
        done_turns[c] += 1
        finished[0] += 1
        if done_turns[c] < turns:
            heapq.heappush(due, (time.monotonic() + think_s, c))

    gw.on_complete = on_complete

    def pump():
        t = time.monotonic()
        batch = []
        while due and due[0][0] <= t:
            _, c = heapq.heappop(due)
            m = wl.make(1)[0]
            m.conversation_id = f"{tag}-{c}"
            m.metadata["_conv"] = c
            m.arrival_ns = time.monotonic_ns()
            batch.append(m)
        if batch:
            gw.submit(batch)

    tok0, reuse0 = engine.total_tokens, engine.kv_reused_tokens
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    target = convs * turns
    while finished[0] < target and time.perf_counter() - t0 < timeout_s:
        pump()
        gw.tick(pump=pump)
        if engine.inflight() == 0 and gw.pending() == 0 and due and due[0][0] > time.monotonic():
            time.sleep(min(due[0][0] - time.monotonic(), 0.01))
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    gw.flush_latency()
    lat = gw.rec_done.summary()
    return {"residency": residency, "turns_completed": finished[0], "seconds": round(el, 3),
            "turns_per_s": round(finished[0] / el, 1), "forward_tokens": engine.total_tokens - tok0,
            "forward_tokens_per_turn": round((engine.total_tokens - tok0) / max(1, finished[0]), 1),
            "kv_reused_tokens": engine.kv_reused_tokens - reuse0,
            "p50_turn_ms": round(lat["p50_ms"], 2), "p99_turn_ms": round(lat["p99_ms"], 2)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--convs", type=int, default=1024)
    ap.add_argument("--turns", type=int, default=6)
    ap.add_argument("--slots", type=int, default=1536)
    ap.add_argument("--max-ctx", type=int, default=512)
    ap.add_argument("--token-budget", type=int, default=4096)
    ap.add_argument("--gen-tokens", type=int, default=16)
    ap.add_argument("--prompt-cap", type=int, default=32)
    ap.add_argument("--think-ms", type=float, default=0.0)
    ap.add_argument("--timeout-s", type=float, default=240.0)
    ap.add_argument("--model", default="llama3-8b")
    a = ap.parse_args()
    import torch

    from llm_message_queue_amd.backend.engine import BackendEngine
    from llm_message_queue_amd.gateway.router import Gateway
    from llm_message_queue_amd.gateway.workload import Workload
    from llm_message_queue_amd.models.llama_stub import LlamaConfig
    from llm_message_queue_amd.preprocess.preprocessor import Preprocessor
    from llm_message_queue_amd.utils.config import default_config

    dev = torch.device("cuda", 0)
    cfg = default_config()
    cfg.queue.enable_metrics = False
    cfg.backend.max_ctx = a.max_ctx
    for lv in cfg.queue.levels:
        lv.max_concurrent = a.slots
    engine = BackendEngine(LlamaConfig.by_name(a.model), slots=a.slots, max_ctx=a.max_ctx,
                           token_budget=a.token_budget, device=dev, impl="hip")
    pre = Preprocessor(cfg.preprocessor, use_gpu=True, device=str(dev))
    gw = Gateway(cfg, preprocessor=pre, engine=engine, use_gpu_preprocess=True, prompt_cap=a.prompt_cap,
                 gen_tokens=a.gen_tokens)
    wl = Workload(seed=5)
    # warm-up (kernels, allocator)
    run_mode(gw, engine, wl, 64, 2, True, 0.0, 60, "warm")
    res = [run_mode(gw, engine, wl, a.convs, a.turns, r, a.think_ms / 1e3, a.timeout_s, f"m{int(r)}")
           for r in (True, False)]
    on, off = res
    print(json.dumps({"bench": "long-dialog replay", "model": a.model, "convs": a.convs, "turns": a.turns,
                      "gen_tokens": a.gen_tokens, "slots": a.slots, "residency_on": on, "residency_off": off,
                      "speedup_turns_per_s": round(on["turns_per_s"] / max(1e-9, off["turns_per_s"]), 2)}))


if __name__ == "__main__":
    main()
