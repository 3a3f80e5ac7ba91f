"""Command line (components C18-C21): the reference's four binaries as modes
of one entry point.

    python -m llm_message_queue_amd.cli serve [--config DIR] [--model llama3-8b|tiny] [--no-gpu]
    python -m llm_message_queue_amd.cli api-gateway ...   # ingress + queue + dispatcher, no local backend
    python -m llm_message_queue_amd.cli queue-manager ... # backend rank (GPU engine), no HTTP
    python -m llm_message_queue_amd.cli scheduler --gateway http://host:8080
    python -m llm_message_queue_amd.cli validate-config [--config DIR]
    python -m llm_message_queue_amd.cli bench [bench.py args]

Multi-GPU: launch under ``torch.distributed.run`` (one rank per GPU, RCCL).
Rank 0 hosts HTTP; every rank runs the gateway tick loop and the ranks share
work through the RCCL planner (all_gather of load vectors + all_to_all of
request descriptors).  Split deployment: any number of ``api-gateway``
processes (HTTP + preprocess) push into a shared-memory request ring that the
``queue-manager`` process (dispatcher + GPU backend) drains, with status
events flowing back -- the reference's microservices never shared their
queues (D14).
"""
from __future__ import annotations

import argparse
import json
import os
import signal
import sys
import threading
import time


def _load_cfg(path):
    from ..utils.config import load_config
    return load_config(path)


def _build_engine(cfg, model: str, device):
    from ..backend.engine import BackendEngine
    from ..backend.slot_page import SlotPage
    from ..models.llama_stub import LlamaConfig
    rank = int(os.environ.get("RANK", "0"))
    page = SlotPage(f"serve{os.environ.get('TORCHELASTIC_RUN_ID', os.getpid())}", rank)
    return BackendEngine(LlamaConfig.by_name(model), slots=cfg.gpu.slots_per_gpu, max_ctx=cfg.backend.max_ctx,
                         token_budget=cfg.backend.token_budget, device=device, impl="hip", page=page, gpu_index=rank), page


def cmd_native_ingress(a) -> int:
    """``api-gateway --native``: the C++ HTTP ingress for POST /api/v1/messages
    feeding the shared request ring (no Python request handling at all)."""
    from ..gateway.native_ingress import NativeIngress
    cfg = _load_cfg(a.config)
    port = a.port or cfg.server.port
    ing = NativeIngress(port, a.ring or cfg.server.shared_ring, a.ingress_threads, a.host or cfg.server.host,
                        cfg=cfg)
    port = ing.start()
    print(json.dumps({"event": "listening", "host": a.host or cfg.server.host, "port": port, "role": "native-ingress",
                      "ring": ing.ring, "threads": a.ingress_threads}), flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    while not stop.is_set():
        stop.wait(0.5)
    print(json.dumps({"event": "stopped", **ing.stats()}), flush=True)
    ing.stop()
    return 0


def cmd_serve(a, role: str = "serve") -> int:
    import torch
    from ..balancer.load_balancer import Endpoint
    from ..gateway.app import GatewayApp
    from ..parallel.comm import init_from_env, local_device_index
    from ..utils import logging as ulog

    cfg = _load_cfg(a.config)
    if a.port:
        cfg.server.port = a.port
    if getattr(a, "grpc_port", 0):
        cfg.server.grpc_port = a.grpc_port
    if a.host:
        cfg.server.host = a.host
    ulog.configure(cfg.logging.level, cfg.logging.format, cfg.logging.output)
    rank = int(os.environ.get("RANK", "0"))
    use_gpu = torch.cuda.is_available() and not a.no_gpu
    comm = init_from_env(control=cfg.gpu.control_plane) if use_gpu else None
    engine = page = None
    if use_gpu and role in ("serve", "queue-manager"):
        local = local_device_index()
        torch.cuda.set_device(local)
        engine, page = _build_engine(cfg, a.model, torch.device("cuda", local))
        engine.warm_shapes()      # cold-start GEMM shapes before the first request (idle -> busy)
    ring, app_role = None, "serve"
    if role in ("api-gateway", "queue-manager") and not a.no_ring:
        # the split deployment shares ONE request queue through shared memory (D14)
        from ..gateway.shm_bridge import RingPair
        ring = RingPair(a.ring or cfg.server.shared_ring, cfg.server.shared_ring_bytes, "open")
        app_role = "ingress" if role == "api-gateway" else "dispatcher"
    gapp = GatewayApp(cfg, use_gpu=use_gpu, engine=engine, comm=comm, start=False, role=app_role, ring=ring)
    if engine is not None:
        # every rank's balancer lists EVERY GPU of the job (its own bound to
        # the zero-copy load page): the multi-GPU planner reads the view of
        # these endpoints -- an operator or the autoscaler removing /
        # marking one on rank 0 takes that GPU out of placement everywhere
        world = comm.world if comm is not None else 1
        for j in range(world):
            gapp.lb.add_endpoint(Endpoint(id=f"gpu{j}", type="llm", gpu_index=j, page=page if j == rank else None,
                                          max_connections=cfg.gpu.slots_per_gpu))
        gapp.resources.register_gpu(rank, a.model, cfg.gpu.slots_per_gpu,
                                    torch.cuda.get_device_properties(engine.device).total_memory,
                                    cfg.gpu.slots_per_gpu * cfg.backend.max_ctx)
    if page is not None:
        gapp.start_telemetry({rank: page})
    gapp.start()
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())

    def _watch_fatal():            # a lost peer rank ends this process too
        while not stop.is_set():
            if gapp.fatal is not None:
                stop.set()
            stop.wait(0.2)
    threading.Thread(target=_watch_fatal, daemon=True).start()
    if rank == 0 and role in ("serve", "api-gateway", "queue-manager"):
        # queue-manager serves the full API too: with a native ingress in
        # front, status / conversation / admin routes live with the dispatcher
        import uvicorn
        from ..api.server import create_app
        app = create_app(gapp)
        server = uvicorn.Server(uvicorn.Config(app, host=cfg.server.host, port=cfg.server.port, log_level="warning"))
        t = threading.Thread(target=server.run, daemon=True)
        t.start()
        print(json.dumps({"event": "listening", "host": cfg.server.host, "port": cfg.server.port,
                          "gpu": use_gpu, "role": role}), flush=True)
        grpc_srv = None
        if cfg.server.grpc_port:
            from ..api.grpc_server import GrpcServer
            grpc_srv = GrpcServer(gapp, cfg.server.grpc_port, cfg.server.host, cfg.server.grpc_max_workers,
                                  tls_cert=cfg.server.grpc_tls_cert, tls_key=cfg.server.grpc_tls_key)
            print(json.dumps({"event": "listening", "host": cfg.server.host, "port": grpc_srv.start(),
                              "protocol": "grpc", "service": "llmq.v1.MessageQueue"}), flush=True)
        while not stop.is_set() and t.is_alive():
            stop.wait(0.5)
        if grpc_srv is not None:
            grpc_srv.stop()
        server.should_exit = True
        t.join(timeout=5)
    else:
        while not stop.is_set():
            stop.wait(0.5)
    gapp.stop()
    if page is not None:
        page.close(unlink=True)
    if gapp.fatal is not None:
        print(json.dumps({"event": "fatal", "error": str(gapp.fatal)}), flush=True)
        return 3
    return 0


def cmd_scheduler(a) -> int:
    """The autoscaler service: polls a gateway's queue stats over HTTP and
    adds/removes endpoints through its REST API (reference cmd/scheduler,
    which instead ran against an empty private queue, D13)."""
    import urllib.request
    from ..balancer.load_balancer import Endpoint
    from ..scheduler.scheduler import Scheduler, SchedulerConfig

    cfg = _load_cfg(a.config)
    base = a.gateway.rstrip("/")

    def get(path):
        with urllib.request.urlopen(base + path, timeout=5) as r:
            return json.loads(r.read())

    def send(method, path, body=None):
        req = urllib.request.Request(base + path, method=method, data=json.dumps(body).encode() if body else None,
                                     headers={"Content-Type": "application/json"})
        with urllib.request.urlopen(req, timeout=5) as r:
            return json.loads(r.read() or b"{}")

    class RemoteLB:
        def get_all_endpoints(self):
            return [Endpoint.from_dict(e) for e in get("/api/v1/endpoints")["endpoints"]]

        def add_endpoint(self, ep):
            send("POST", "/api/v1/endpoints", {"id": ep.id, "url": ep.url, "name": ep.name, "type": ep.type,
                                              "weight": ep.weight, "max_connections": ep.max_connections})

        def remove_endpoint(self, eid):
            send("DELETE", f"/api/v1/endpoints/{eid}")

    def stats():
        st = get("/api/v1/queues/stats").get("standard", {})
        return {q: v.get("PendingCount", 0) for q, v in st.items()}

    sc = cfg.scheduler
    s = Scheduler(SchedulerConfig(strategy=sc.strategy, monitor_interval=sc.check_interval,
                                  scaling_thresholds={"scale_up_queue_length": sc.scale_up_threshold,
                                                      "scale_down_queue_length": sc.scale_down_threshold},
                                  resource_limits={"min_endpoints": sc.min_endpoints,
                                                   "max_endpoints": sc.max_endpoints}), stats, RemoteLB())
    n = 0
    while a.iterations <= 0 or n < a.iterations:
        try:
            act = s.schedule_resources()
            print(json.dumps({"action": act, "recommendation": s.recommendation}), flush=True)
        except Exception as e:
            print(json.dumps({"error": str(e)}), flush=True)
        n += 1
        time.sleep(sc.check_interval / 1e9)
    return 0


def cmd_validate(a) -> int:
    from ..utils.config import ConfigError
    try:
        cfg = _load_cfg(a.config)
    except (ConfigError, FileNotFoundError) as e:
        print(json.dumps({"valid": False, "error": str(e)}))
        return 1
    print(json.dumps({"valid": True, "levels": [lv.name for lv in cfg.queue.levels],
                      "strategy": cfg.scheduler.strategy, "lb": cfg.loadbalancer.algorithm}))
    return 0


def cmd_token(a) -> int:
    """Issue an HS256 JWT with the configured secret/issuer (jwt authentication)."""
    from ..api.security import issue_token
    cfg = _load_cfg(a.config)
    jwt = cfg.security.authentication.jwt
    secret = a.secret or jwt.secret
    if not secret:
        print(json.dumps({"error": "no jwt secret (security.authentication.jwt.secret or --secret)"}))
        return 1
    ttl = int(a.ttl_hours * 3600) if a.ttl_hours > 0 else int(jwt.expiration) * 3600
    print(issue_token(secret, a.subject, a.role, ttl_s=ttl, issuer=jwt.issuer))
    return 0


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="llmq")
    sub = ap.add_subparsers(dest="cmd", required=True)
    for name in ("serve", "server", "api-gateway", "queue-manager"):
        p = sub.add_parser(name)
        p.add_argument("--config", default=None, help="config dir or file (default: ./configs)")
        p.add_argument("--host", default="")
        p.add_argument("--port", type=int, default=0)
        p.add_argument("--grpc-port", type=int, default=0, help="also serve llmq.v1.MessageQueue over gRPC")
        p.add_argument("--model", default="llama3-8b")
        p.add_argument("--no-gpu", action="store_true")
        p.add_argument("--ring", default="", help="shared request ring name (api-gateway/queue-manager)")
        p.add_argument("--no-ring", action="store_true", help="api-gateway/queue-manager without the shared ring")
        p.add_argument("--native", action="store_true", help="api-gateway: C++ HTTP ingress for POST /messages")
        p.add_argument("--ingress-threads", type=int, default=4)
    p = sub.add_parser("scheduler")
    p.add_argument("--config", default=None)
    p.add_argument("--gateway", default="http://127.0.0.1:8080")
    p.add_argument("--iterations", type=int, default=0)
    p = sub.add_parser("validate-config")
    p.add_argument("--config", default=None)
    p = sub.add_parser("token", help="issue a JWT for security.authentication.method=jwt")
    p.add_argument("--config", default=None)
    p.add_argument("--subject", required=True)
    p.add_argument("--role", default="")
    p.add_argument("--secret", default="", help="override the configured secret")
    p.add_argument("--ttl-hours", type=float, default=0.0, help="default: jwt.expiration")
    sub.add_parser("bench", add_help=False)
    a, rest = ap.parse_known_args(argv)
    if a.cmd in ("serve", "server"):
        return cmd_serve(a, "serve")
    if a.cmd == "api-gateway":
        return cmd_native_ingress(a) if a.native else cmd_serve(a, "api-gateway")
    if a.cmd == "queue-manager":
        return cmd_serve(a, "queue-manager")
    if a.cmd == "scheduler":
        return cmd_scheduler(a)
    if a.cmd == "validate-config":
        return cmd_validate(a)
    if a.cmd == "token":
        return cmd_token(a)
    if a.cmd == "bench":
        root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        sys.path.insert(0, root)
        import bench
        return bench.main(rest)
    return 2


if __name__ == "__main__":
    sys.exit(main())
