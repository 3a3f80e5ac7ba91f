"""gRPC ingest rate: submissions/s accepted through ``SubmitBatch`` (512 per
call), ``SubmitStream`` (one bidirectional stream per client) and unary
``Submit`` calls (client processes separate from the server),
against a CPU gateway (no GPU; dispatch simulated at 1 ms per request).

    python bench/grpc_bench.py [--n 20000] [--clients 4]

Prints one JSON line per mode.  This measures the front-end (HTTP/2 framing,
protobuf, the micro-batched preprocess + queue push), not the GPU backend.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


WORDS = ["hello", "urgent", "status", "please", "asap", "report", "summary", "question?"]


def _client(port: int, mode: str, per: int, c: int) -> int:
    from llm_message_queue_amd.api.grpc_server import GrpcClient, pb
    cli = GrpcClient(f"127.0.0.1:{port}")
    cli.health()
    ok = 0
    if mode == "stream":
        reqs = (pb["SubmitRequest"](content=f"{WORDS[i % 8]} {WORDS[(i * 3) % 8]} {i}", user_id=f"u{c}-{i % 97}")
                for i in range(per))
        ok = sum(r.code == 202 for r in cli.submit_stream(reqs, timeout=600))
    elif mode == "batch":
        for b0 in range(0, per, 512):
            reqs = [pb["SubmitRequest"](content=f"{WORDS[i % 8]} {WORDS[(i * 3) % 8]} {i}", user_id=f"u{c}-{i % 97}")
                    for i in range(b0, min(per, b0 + 512))]
            ok += sum(r.code == 202 for r in cli.submit_batch(reqs))
    else:
        for i in range(per):
            ok += cli.submit(f"{WORDS[i % 8]} {i}", user_id=f"u{c}").code == 202
    cli.close()
    return ok


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=20000, help="messages per mode")
    ap.add_argument("--clients", type=int, default=4)
    a = ap.parse_args()
    from llm_message_queue_amd.api.grpc_server import GrpcServer
    from llm_message_queue_amd.gateway.app import GatewayApp
    from llm_message_queue_amd.utils.config import default_config
    cfg = default_config()
    cfg.queue.worker.process_interval = 2_000_000
    gw = GatewayApp(cfg, use_gpu=False, simulate_ms=(1, 1, 1, 1))
    srv = GrpcServer(gw, 0, "127.0.0.1", max_workers=4 * a.clients)
    port = srv.start()
    try:
        for mode in ("batch", "stream", "unary"):
            per = a.n // a.clients if mode != "unary" else a.n // (4 * a.clients)

            # clients in their own processes (spawned: no fork after gRPC
            # init), so the measurement is the server's, not one shared GIL's
            ctx = mp.get_context("spawn")
            with ctx.Pool(a.clients) as pool:
                t0 = time.perf_counter()
                ok = pool.starmap(_client, [(port, mode, per, c) for c in range(a.clients)])
            dt = time.perf_counter() - t0
            print(json.dumps({"bench": "grpc ingest", "mode": mode, "clients": a.clients, "accepted": sum(ok),
                              "seconds": round(dt, 3), "msgs_per_s": round(sum(ok) / dt, 1)}), flush=True)
    finally:
        srv.stop()
        gw.stop()


if __name__ == "__main__":
    main()
