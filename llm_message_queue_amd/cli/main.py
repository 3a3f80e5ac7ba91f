"""Command line (components C18-C21): the reference's four binaries as modes
of one entry point.

    python -m llm_message_queue_amd.cli serve [--config DIR] [--model llama3-8b|tiny] [--no-gpu]
    python -m llm_message_queue_amd.cli api-gateway ...   # ingress + queue + dispatcher, no local backend
    python -m llm_message_queue_amd.cli queue-manager ... # backend rank (GPU engine), no HTTP
    python -m llm_message_queue_amd.cli scheduler --gateway http://host:8080
    python -m llm_message_queue_amd.cli validate-config [--config DIR]
    python -m llm_message_queue_amd.cli bench [bench.py args]

Multi-GPU: launch under ``torch.distributed.run`` (one rank per GPU).  Rank
0 hosts the public port: the C++ front door (``server.front_door: native``)
takes ``POST /api/v1/messages`` into a shared-memory ring that EVERY rank
drains (so ingest and GPU preprocessing spread over the GPUs), routes
conversation turns to rank 0 (owner of conversation state) and
reverse-proxies every other route to rank 0's API server; status queries for
messages another rank popped are answered through ``gateway.peers``.  Every
rank runs the gateway tick loop; per tick the ranks exchange load vectors
and request descriptors over the node-local shared-memory control plane
(``parallel.comm.ShmComm``) and compute the same placement plan, and KV
migrations move over RCCL / xGMI.  Split deployment: any number of ``api-gateway``
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


def _build_engine(cfg, model: str, device, job: str = ""):
    import torch
    from ..backend.engine import BackendEngine
    from ..backend.slot_page import SlotPage
    from ..models.llama_stub import LlamaConfig
    rank = int(os.environ.get("RANK", "0"))
    page = SlotPage(f"serve{job or os.getpid()}", rank)
    mcfg = LlamaConfig.by_name(model)
    slots = fit_slots(mcfg, cfg.gpu.slots_per_gpu, cfg.backend.max_ctx, cfg.gpu.hbm_reserve_gb,
                      torch.cuda.get_device_properties(device).total_memory)
    return BackendEngine(mcfg, slots=slots, max_ctx=cfg.backend.max_ctx,
                         token_budget=cfg.backend.token_budget, device=device, impl="hip", page=page, gpu_index=rank,
                         step_timeout_s=cfg.backend.step_timeout / 1e9,
                         realtime_step_tokens=cfg.backend.realtime_step_tokens,
                         realtime_mode=cfg.backend.realtime_mode, micro_slots=cfg.backend.micro_slots,
                         micro_inflight=cfg.backend.micro_inflight, micro_stream=cfg.backend.micro_stream,
                         micro_cus=cfg.backend.micro_cus, micro_gemm=cfg.backend.micro_gemm,
                         library_gemm=cfg.backend.library_gemm, micro_graph=cfg.backend.micro_graph), page


def fit_slots(mcfg, slots: int, max_ctx: int, reserve_gb: float, total_bytes: int) -> int:
    """``gpu.hbm_reserve_gb``: batch slots whose KV cache (slots x max_ctx x
    K/V bytes per token) fits next to the bf16 weights with that much HBM
    left free; fewer than configured -> capped, with a warning."""
    per_slot = max_ctx * mcfg.layers * 2 * mcfg.kv_heads * mcfg.head_dim * 2
    room = total_bytes - int(reserve_gb * (1 << 30)) - mcfg.param_count() * 2
    fit = max(0, room // per_slot) if per_slot > 0 else slots
    if fit < slots:
        from ..utils.logging import get_logger
        get_logger("serve").warning("gpu.slots_per_gpu capped to fit HBM", configured=slots, fitted=int(fit),
                    hbm_gib=round(total_bytes / (1 << 30), 1), reserve_gib=reserve_gb,
                    kv_gib_per_slot=round(per_slot / (1 << 30), 4))
        if fit < 1:
            raise SystemExit("gpu.hbm_reserve_gb leaves no HBM for the KV cache")
        return int(fit)
    return slots


def _build_cpu_engine(cfg, sim_gpu: str = "", job: str = ""):
    """``--cpu-ranks``: a tiny Llama-shaped engine on the CPU reference ops
    (the multi-rank control flow without a GPU; never a measurement).  With
    ``--sim-gpu SPEEDS`` each rank runs a SimEngine instead: the engine's
    host side at the serving config, the 8B step as a simulated device
    clock at the rank's relative speed (front-door rehearsals at the
    8-GPU request rate on a CPU box)."""
    from ..backend.engine import BackendEngine
    from ..backend.slot_page import SlotPage
    from ..models.llama_stub import LlamaConfig
    rank = int(os.environ.get("RANK", "0"))
    page = SlotPage(f"serve{job or os.getpid()}", rank)
    if sim_gpu:
        from ..backend.sim_engine import SimEngine
        speeds = [float(x) for x in sim_gpu.split(",")]
        return SimEngine(speed=speeds[rank % len(speeds)], slots=cfg.gpu.slots_per_gpu, max_ctx=cfg.backend.max_ctx,
                         token_budget=cfg.backend.token_budget, page=page, gpu_index=rank,
                         seed=1000 + rank), page
    return BackendEngine(LlamaConfig.tiny(), slots=min(cfg.gpu.slots_per_gpu, 16), max_ctx=64, token_budget=128,
                         device="cpu", impl="ref", seed=1000 + rank, page=page, gpu_index=rank), page


def _free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def _wait_port(host: str, port: int, thread, timeout_s: float = 30.0) -> None:
    import socket
    deadline = time.monotonic() + timeout_s
    while time.monotonic() < deadline and thread.is_alive():
        try:
            with socket.create_connection((host, port), timeout=0.5):
                return
        except OSError:
            time.sleep(0.05)
    raise RuntimeError(f"API server did not come up on {host}:{port}")


def cmd_native_ingress(a) -> int:
    """``api-gateway --native``: the C++ HTTP ingress for POST /api/v1/messages
    feeding the shared request ring (no Python request handling at all)."""
    from ..gateway.native_ingress import NativeIngress
    cfg = _load_cfg(a.config)
    port = a.port or cfg.server.port
    threads = a.ingress_threads or cfg.server.ingress_threads
    ing = NativeIngress(port, a.ring or cfg.server.shared_ring, threads, a.host or cfg.server.host,
                        cfg=cfg, gateway_compat=True)
    port = ing.start()
    print(json.dumps({"event": "listening", "host": a.host or cfg.server.host, "port": port, "role": "native-ingress",
                      "ring": ing.ring, "threads": threads}), flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())
    while not stop.is_set():
        stop.wait(0.5)
    print(json.dumps({"event": "stopped", **ing.stats()}), flush=True)
    ing.stop()
    return 0


def _start_tracemalloc(path: str, every_s: float = 60.0) -> None:
    """``LLMQ_TRACEMALLOC=<file>``: a memory-growth probe for soaks.  Python
    allocations are traced (8 frames), and every ``LLMQ_TRACEMALLOC_EVERY_S``
    seconds (default 60) the 25 call sites that grew most since the first
    snapshot are appended to ``<file>.<pid>``.  Costs ~2x interpreter time:
    diagnosis only."""
    import tracemalloc
    tracemalloc.start(8)
    out = f"{path}.{os.getpid()}"

    def loop():
        base = None
        t0 = time.monotonic()
        while True:
            time.sleep(every_s)
            snap = tracemalloc.take_snapshot().filter_traces(
                (tracemalloc.Filter(False, tracemalloc.__file__), tracemalloc.Filter(False, "<frozen importlib._bootstrap>")))
            if base is None:
                base = snap
                continue
            cur, peak = tracemalloc.get_traced_memory()
            with open(out, "a") as fh:
                fh.write(f"=== t={time.monotonic() - t0:.0f}s traced={cur / 2**20:.1f} MiB peak={peak / 2**20:.1f} MiB\n")
                for st in snap.compare_to(base, "traceback")[:25]:
                    fh.write(f"{st.size_diff / 2**20:+.2f} MiB  {st.count_diff:+d} blocks\n")
                    for line in st.traceback.format()[-8:]:
                        fh.write(f"    {line}\n")
    threading.Thread(target=loop, name="tracemalloc-probe", daemon=True).start()


def cmd_serve(a, role: str = "serve") -> int:
    import torch
    if os.environ.get("LLMQ_TRACEMALLOC"):
        _start_tracemalloc(os.environ["LLMQ_TRACEMALLOC"], float(os.environ.get("LLMQ_TRACEMALLOC_EVERY_S", "60")))
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
    world = int(os.environ.get("WORLD_SIZE", "1"))
    cpu_ranks = bool(getattr(a, "cpu_ranks", False))
    if getattr(a, "front_door", ""):
        cfg.server.front_door = a.front_door
    use_gpu = torch.cuda.is_available() and not a.no_gpu and not cpu_ranks
    comm = None
    if use_gpu:
        from ..parallel.comm import set_device_list
        set_device_list(cfg.gpu.devices)                    # gpu.devices (empty: every visible GPU)
        comm = init_from_env(backend=cfg.gpu.comm_backend, control=cfg.gpu.control_plane)
    elif cpu_ranks and world > 1:
        # CPU rehearsal of the multi-GPU job: gloo data plane, the same
        # control plane, tiny reference-op engines (tests / CI)
        comm = init_from_env(backend="gloo", control=cfg.gpu.control_plane)
    # every node-shared segment of this job INCARNATION is named by a token
    # no earlier job or restart can share (run id + restart count + a nonce
    # rank 0 broadcasts) and stamped with its generation
    from ..parallel.comm import job_token
    multi = comm is not None and comm.world > 1
    job, gen = job_token(comm if multi else None)
    engine = page = None
    if use_gpu and role in ("serve", "queue-manager"):
        local = local_device_index()
        torch.cuda.set_device(local)
        from ..parallel.placement import bind_rank
        binding = bind_rank(cfg.gpu.cpu_bind)    # before the serving threads start (they inherit it)
        if binding.get("cpus"):
            print(json.dumps({"event": "cpu_binding", "rank": rank, **{k: v for k, v in binding.items()
                                                                       if k != "shared_with"}}), flush=True)
        engine, page = _build_engine(cfg, a.model, torch.device("cuda", local), job)
        engine.warm_shapes()      # cold-start GEMM shapes before the first request (idle -> busy)
    elif cpu_ranks and role in ("serve", "queue-manager"):
        engine, page = _build_cpu_engine(cfg, getattr(a, "sim_gpu", ""), job)
    if page is not None:
        page.unlink_name()        # read through this mapping only; a SIGKILL leaves no file behind
    ring, app_role = None, "serve"
    # the C++ front door fronts every `serve` with a backend -- one GPU or a
    # whole node (the Python ASGI stack tops out at ~2k req/s for POST
    # /api/v1/messages); `server.front_door: python` keeps uvicorn on the port
    front = role == "serve" and engine is not None and cfg.server.front_door == "native"
    conv_ring = None
    if front:
        # the front door: ONE shared request ring every rank drains
        # (MPMC), plus rank 0's ring for conversation turns (rank 0 owns
        # conversation state); the C++ ingress on rank 0 feeds both.  The
        # rings belong to this job incarnation: rank 0 creates them (stamped
        # with the generation), the others attach after a barrier and refuse
        # a ring of any other generation; once rank 0's ingress has mapped
        # them too their names are dropped (nothing survives a SIGKILL)
        from ..gateway.shm_bridge import RingPair
        shared = f"{a.ring or cfg.server.shared_ring}-{job}"
        if rank == 0:
            ring = RingPair(shared, cfg.server.shared_ring_bytes, "create", gen)
            conv_ring = RingPair(f"{shared}-conv", cfg.server.shared_ring_bytes, "create", gen)
        if multi:
            comm.barrier()
        if rank != 0:
            ring = RingPair(shared, 0, "attach", gen)
        app_role = "rank"
    elif role in ("api-gateway", "queue-manager") and not a.no_ring:
        # the split deployment shares ONE request queue through shared memory (D14)
        from ..gateway.shm_bridge import RingPair
        ring = RingPair(a.ring or cfg.server.shared_ring, cfg.server.shared_ring_bytes, "open")
        app_role = "ingress" if role == "api-gateway" else "dispatcher"
    gapp = GatewayApp(cfg, use_gpu=use_gpu, engine=engine, comm=comm, start=False, role=app_role, ring=ring)
    if conv_ring is not None:
        gapp.extra_rings.append(conv_ring)
    # every GPU rank that drains a ring answers rank 0's API through the peer
    # directory: status queries for the messages it popped, and the
    # preprocessor's admin state (it preprocesses what it pops)
    peered = front or (role == "queue-manager" and ring is not None and comm is not None and comm.world > 1)
    if peered:
        from ..gateway.peers import PeerDirectory
        gapp.peers = PeerDirectory(ring.name, rank, comm.world if comm is not None else 1, handler=gapp.peer_op,
                                   comm=comm if multi else None, gen=gen)
    if engine is not None:
        # every rank's balancer lists EVERY GPU of the job (its own bound to
        # the zero-copy load page): the multi-GPU planner reads the view of
        # these endpoints -- an operator or the autoscaler removing /
        # marking one on rank 0 takes that GPU out of placement everywhere
        world = comm.world if comm is not None else 1
        for j in range(world):
            gapp.lb.add_endpoint(Endpoint(id=f"gpu{j}", type="llm", gpu_index=j, page=page if j == rank else None,
                                          max_connections=cfg.gpu.slots_per_gpu))
        hbm = (torch.cuda.get_device_properties(engine.device).total_memory if engine.cuda
               else engine.weight_bytes + engine.kv_token_capacity() * engine.kv_bytes_per_token())
        gapp.resources.register_gpu(rank, a.model, engine.slots, hbm, engine.kv_token_capacity())
    if page is not None:
        gapp.start_telemetry({rank: page})
    gapp.start()
    print(json.dumps({"event": "rank", "rank": rank, "pid": os.getpid(), "job": job,
                      "restart": int(os.environ.get("TORCHELASTIC_RESTART_COUNT", "0"))}), flush=True)
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *_: stop.set())
    signal.signal(signal.SIGINT, lambda *_: stop.set())

    # under torchrun the launcher is our parent: if it dies (SIGKILLed) the
    # ranks -- each in a session of its own -- would live on, holding their
    # GPU and port, so a rank whose launcher is gone stops like on SIGTERM
    launcher = os.getppid() if os.environ.get("TORCHELASTIC_RUN_ID") else 0

    def _watch_fatal():            # a lost peer rank / a stalled loop ends this process too
        while not stop.is_set():
            if launcher and os.getppid() != launcher:
                print(json.dumps({"event": "launcher_gone", "rank": rank}), flush=True)
                stop.set()
                break
            if gapp.fatal is not None:
                print(json.dumps({"event": "fatal", "rank": rank, "error": str(gapp.fatal)}), flush=True)
                stop.set()
                # the orderly shutdown below joins threads; a thread stuck in
                # whatever stalled the loop must not keep the process alive:
                # leave with the failure status regardless after a grace period
                # (os._exit, never an exec -- the launcher starts the new one)
                t = threading.Timer(float(os.environ.get("LLMQ_FATAL_EXIT_GRACE_S", "20")),
                                    lambda: os._exit(3))
                t.daemon = True
                t.start()
            stop.wait(0.2)
    threading.Thread(target=_watch_fatal, daemon=True).start()
    ingress = None
    if rank == 0 and role in ("serve", "api-gateway", "queue-manager"):
        # queue-manager serves the full API too: with a native ingress in
        # front, status / conversation / admin routes live with the dispatcher
        import uvicorn
        from ..api.server import create_app
        # behind the C++ front door every proxied request arrives from loopback
        app = create_app(gapp, trusted_proxies=("127.0.0.1", "::1") if front else ())
        api_host, api_port = cfg.server.host, cfg.server.port
        if front:
            # the public port belongs to the C++ front door; the API server
            # listens on loopback behind it (reverse-proxied routes)
            api_host, api_port = "127.0.0.1", _free_port()
        # server.mode (gin's debug / release in the reference): debug logs
        # every request the API server answers, release only warnings
        debug = cfg.server.mode == "debug"
        server = uvicorn.Server(uvicorn.Config(app, host=api_host, port=api_port,
                                               log_level="info" if debug else "warning", access_log=debug))
        t = threading.Thread(target=server.run, daemon=True)
        t.start()
        port = api_port
        _wait_port(api_host, api_port, t)          # "listening" means accepting connections
        if front:
            from ..gateway.native_ingress import NativeIngress
            ingress = NativeIngress(cfg.server.port, ring.name, getattr(a, "ingress_threads", 0)
                                    or cfg.server.ingress_threads, cfg.server.host, cfg=cfg,
                                    conv_ring=f"{ring.name}-conv", upstream=(api_host, api_port))
            port = ingress.start()
            gapp.front_door = ingress
            for r in (ring, conv_ring):           # every process of the job has them mapped now
                r.unlink_names()
        print(json.dumps({"event": "listening", "host": cfg.server.host, "port": port,
                          "gpu": use_gpu, "role": role, "world": world,
                          "front_door": "native" if front else "python", "api_port": api_port}), flush=True)
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
        if ingress is not None:
            ingress.stop()
        server.should_exit = True
        t.join(timeout=5)
    else:
        while not stop.is_set():
            stop.wait(0.5)
    gapp.stop()
    if page is not None:
        page.close(unlink=True)
    if gapp.peers is not None:
        gapp.peers.close(unlink=rank == 0)
    if front:
        for r in (ring, conv_ring):
            if r is not None:
                r.close(unlink=rank == 0)
    if gapp.fatal is not None:
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
        st = get("/api/v1/queues/stats")
        job = st.get("job")
        if job and "pending_by_tier" in job:      # multi-GPU gateway: every rank's queues
            return {q: int(n) for q, n in job["pending_by_tier"].items()}
        return {q: v.get("PendingCount", 0) for q, v in st.get("standard", {}).items()}

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
        p.add_argument("--ingress-threads", type=int, default=0,
                       help="native ingress epoll threads (default: server.ingress_threads)")
        p.add_argument("--front-door", default="", choices=["", "native", "python"],
                       help="multi-GPU serve: C++ front door feeding a ring every rank drains (native, "
                            "default) or every route on rank 0's ASGI server (python)")
        p.add_argument("--sim-gpu", default="",
                       help="with --cpu-ranks: per-rank relative GPU speeds; each rank's backend is a SimEngine "
                            "at the serving config (rehearsal, not a measurement)")
        p.add_argument("--cpu-ranks", action="store_true",
                       help="serve / queue-manager: tiny CPU engines per rank over gloo (multi-rank rehearsal "
                            "without a GPU)")
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
