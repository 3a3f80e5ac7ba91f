"""Monolith wiring (component C18, `cmd/server/main.go`), fixed:
  * the four level queues exist before the first request (D1);
  * a dispatcher always runs (D2): with a GPU, the gateway tick loop feeds
    the local Llama-stub backend (and, under torchrun, the other ranks' GPUs
    through the per-tick planner on the shared-memory control plane); without
    a GPU, QueueFactory workers drain the level
    queues with a simulated LLM call that goes through the LoadBalancer's
    GetEndpoint/ReleaseEndpoint (what `cmd/queue-manager/main.go:141-166`
    simulates);
  * defaults merged / intervals validated (D3) by ``utils.config``.
"""
from __future__ import annotations

import collections
import itertools
import os
import threading
import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from ..balancer.load_balancer import Endpoint, LoadBalancer
from ..conversation.persistence import make_store
from ..conversation.state_manager import StateManager
from ..models.message import Message, MessageStatus, priority_name
from ..preprocess.preprocessor import Preprocessor
from ..queue.core import QueueError, QueueFull
from ..queue.factory import QueueFactory, QueueType
from ..scheduler.resource_scheduler import ResourceScheduler
from ..utils.logging import get_logger
from ..utils.metrics import QueueMetrics, default_metrics
from .app_health import HealthMixin
from .app_jobwide import JobWideMixin
from .ingress import MicroBatcher
from .router import Gateway

# reference fixed estimates (api/handlers.go:729-744), used before rates exist
_REF_WAIT_NS = {1: 1_000_000_000, 2: 5_000_000_000, 3: 15_000_000_000, 4: 30_000_000_000}


class MessageStore:
    """Bounded id -> Message index for GET /messages (stubs in the reference).
    Per-user and per-conversation sub-indexes (insertion-ordered like the
    main one) keep filtered listings off a full scan."""

    _FIELDS = ("user_id", "conversation_id")

    def __init__(self, max_items: int = 200_000):
        self._d: "collections.OrderedDict[str, Message]" = collections.OrderedDict()
        self._by: Dict[str, Dict[str, Dict[str, None]]] = {f: {} for f in self._FIELDS}
        # the keys each id is indexed under: a message re-put after its
        # user_id / conversation_id changed is unindexed from the keys it was
        # filed under, not from its live attributes
        self._keys: Dict[str, Tuple[str, ...]] = {}
        self._lock = threading.Lock()
        self.max_items = max_items

    def _unindex(self, mid: str) -> None:
        keys = self._keys.pop(mid, None)
        if keys is None:
            return
        for f, k in zip(self._FIELDS, keys):
            idx = self._by[f]
            ids = idx.get(k) if k else None
            if ids is not None:
                ids.pop(mid, None)
                if not ids:
                    del idx[k]

    def put(self, m: Message) -> None:
        with self._lock:
            self._unindex(m.id)
            self._d[m.id] = m
            self._d.move_to_end(m.id)
            keys = tuple(getattr(m, f, "") or "" for f in self._FIELDS)
            self._keys[m.id] = keys
            for f, k in zip(self._FIELDS, keys):
                if k:
                    self._by[f].setdefault(k, {})[m.id] = None
            while len(self._d) > self.max_items:
                mid, _ev = self._d.popitem(last=False)
                self._unindex(mid)

    def get(self, mid: str) -> Optional[Message]:
        with self._lock:
            return self._d.get(mid)

    def values(self) -> List[Message]:
        with self._lock:
            return list(self._d.values())

    def remove(self, mid: str) -> Optional[Message]:
        with self._lock:
            m = self._d.pop(mid, None)
            if m is not None:
                self._unindex(mid)
            return m

    def query(self, user_id: str = "", conversation_id: str = "", status: str = "", limit: int = 10,
              offset: int = 0) -> Tuple[int, List[Message]]:
        """Filtered page (oldest first) and the match count.  Unfiltered, only
        the page is touched; by user or conversation, only that sub-index (the
        full index is 200k messages at serving rates: a scan is ~100 ms of
        interpreter time the serve loop shares).  A status-only filter scans."""
        offset, limit = max(0, offset), max(0, limit)
        if not (user_id or conversation_id or status):
            with self._lock:
                return len(self._d), list(itertools.islice(self._d.values(), offset, offset + limit))
        with self._lock:
            if user_id or conversation_id:
                subs = [self._by[f].get(v, {}) for f, v in (("user_id", user_id), ("conversation_id", conversation_id))
                        if v]
                ids = min(subs, key=len)
                items = [self._d[i] for i in ids if i in self._d]
            else:
                items = list(self._d.values())
        sel = [m for m in items if (not user_id or m.user_id == user_id)
               and (not conversation_id or m.conversation_id == conversation_id)
               and (not status or m.status == status)]
        return len(sel), sel[offset:offset + limit]


class GatewayApp(JobWideMixin, HealthMixin):
    def __init__(self, cfg, *, use_gpu: Optional[bool] = None, engine=None, comm=None,
                 simulate_ms: Sequence[float] = (5, 10, 20, 30), start: bool = True,
                 role: str = "serve", ring=None):
        """``role``: "serve" (monolith), "ingress" (HTTP + preprocess, pushes
        into the shared request ring ``ring``), "dispatcher" (pops the ring
        into its queue and runs the backend; reports status via the event
        ring), or "rank" (one GPU rank of the multi-GPU front door: drains
        ``ring`` -- the shared ring every rank pops -- plus ``extra_rings``
        into its gateway inbox, so ingest and preprocessing spread over the
        GPUs; status queries for its messages come through ``peers``).  See
        ``shm_bridge`` and ``peers``."""
        import torch
        if role not in ("serve", "ingress", "dispatcher", "rank"):
            raise ValueError(f"unknown gateway role {role!r}")
        if role != "serve" and ring is None:
            raise ValueError(f"role {role!r} needs a shared ring")
        self.role = role
        self.ring = ring
        self.extra_rings: List[object] = []       # role "rank": e.g. rank 0's conversation ring
        self.peers = None                          # gateway.peers.PeerDirectory (multi-rank front door)
        self.front_door = None                     # gateway.native_ingress.NativeIngress (rank 0 of cli serve)
        self._ring_thread: Optional[threading.Thread] = None
        self._snap_thread: Optional[threading.Thread] = None
        self.telemetry = None
        self._accepted = 0
        self.fatal: Optional[BaseException] = None     # PeerLost from the serve loop
        self.stalled = ""                              # serve-loop stall (watchdog): /health 503
        self.cfg = cfg
        self.log = get_logger("app")
        self._bound = threading.local()
        self._main_device = torch.cuda.current_device() if torch.cuda.is_available() else None
        self.metrics: QueueMetrics = default_metrics()
        gpu = torch.cuda.is_available() if use_gpu is None else use_gpu
        self.gpu = gpu
        self.preprocessor = Preprocessor(cfg.preprocessor, use_gpu=gpu and cfg.preprocessor.use_gpu)
        # raw requests (C++ ingress) are preprocessed here, not in the API
        # handler that records metadata["analysis"] for the other paths
        self.preprocessor.record_analysis = bool(cfg.queue.enable_metrics) and role in ("rank", "dispatcher")
        self.factory = QueueFactory(cfg.queue, metrics=self.metrics)
        if getattr(self.metrics, "registry", None) is not None:
            # read at scrape time, so every path that changes the DLQ counts
            self.metrics.dead_letter.labels("factory").set_function(self.factory.dead_letter_queue.size)
        self.standard = self.factory.create_queue_manager("standard", QueueType.STANDARD)
        self.factory.create_queue_manager("delayed", QueueType.DELAYED)
        self.factory.create_queue_manager("dead_letter", QueueType.DEAD_LETTER)
        self.factory.create_queue_manager("priority", QueueType.PRIORITY)
        self.lb = LoadBalancer(cfg.loadbalancer)
        self.resources = ResourceScheduler.from_config(cfg.scheduler)
        store = make_store(cfg)
        summary = None
        if cfg.conversation.summarise_on_evict:
            from ..conversation.summarise import SummaryEngine
            summary = SummaryEngine(cfg.preprocessor, device="cuda" if gpu else "cpu",
                                    k=cfg.conversation.salient_tokens, alpha=cfg.conversation.summary_alpha,
                                    dim=cfg.conversation.summary_dim)
        self.state = StateManager.from_config(cfg, persistence=store, summary_engine=summary)
        self.messages = MessageStore()
        self.engine = engine
        self.gateway = Gateway(cfg, preprocessor=self.preprocessor, engine=engine, comm=comm,
                               load_balancer=self.lb if engine is not None else None, metrics=self.metrics,
                               state_manager=self.state, use_gpu_preprocess=self.preprocessor.gpu_enabled(),
                               queue_manager=self.standard, dead_letter=self.factory.dead_letter_queue)
        self.gateway.on_complete = self._on_complete
        # backend-failure retries wait out queue.retry's backoff in the
        # delayed queue; exhausted ones go to the dead-letter queue
        self.gateway.attach_retry_queue(self.factory.delayed_queue)
        if engine is not None:
            # per-GPU usage (in-flight slots, HBM) from every tick's load
            # exchange -> /api/v1/resources (multi-rank; one rank keeps its
            # own resource current through the same path)
            # with several GPUs, rank 0's autoscale decisions park / unpark
            # GPU endpoints (its L_EXCLUDE view reaches every rank's planner)
            self.gateway.attach_resource_scheduler(self.resources,
                                                   act=self.gateway.rank == 0 and self.gateway.world > 1)
        self.batcher = MicroBatcher(self._flush, cfg.preprocessor.batch_window_us, cfg.preprocessor.max_batch)
        self._stop = threading.Event()
        self._wake = threading.Event()
        self._loop_thread: Optional[threading.Thread] = None
        self.simulate_ns = [int(x * 1e6) for x in simulate_ms]
        self._workers = []
        self._dispatch_times: "collections.deque[Tuple[float, int]]" = collections.deque(maxlen=64)
        if start:
            self.start()

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        self.state.start()
        snap = self.cfg.queue.snapshot_path
        if snap and self.role != "ingress":
            from ..queue.snapshot import read_snapshot
            resumed = 0
            for path in self._snapshots_to_resume():
                counts = read_snapshot(self.factory, path)
                if counts is not None:
                    self.log.info("Resumed queue snapshot", path=path, **counts)
                    os.replace(path, path + ".resumed")
                    resumed += 1
            if resumed:
                for mgr in self.factory.managers().values():
                    for q in mgr.queue_names():
                        for m in mgr.mlq.messages(q):
                            self.messages.put(m)
            if self.cfg.queue.snapshot_interval > 0:
                self._snap_thread = threading.Thread(target=self._snapshot_loop, name="queue-snapshot",
                                                     daemon=True)
                self._snap_thread.start()
        if self.role == "ingress":
            self._ring_thread = threading.Thread(target=self._event_loop, name="ring-events", daemon=True)
            self._ring_thread.start()
            return
        if self.role == "dispatcher":
            self._ring_thread = threading.Thread(target=self._ring_loop, name="ring-ingest", daemon=True)
            self._ring_thread.start()
        elif self.role == "rank":
            self._ring_thread = threading.Thread(target=self._rank_ring_loop, name="ring-ingest", daemon=True)
            self._ring_thread.start()
        if self.engine is not None:
            self._loop_thread = threading.Thread(target=self._serve_loop, name="gateway-loop", daemon=True)
            self._loop_thread.start()
            if self.cfg.server.stall_dump_after > 0 or self.cfg.server.stall_fatal_after > 0:
                threading.Thread(target=self._stall_watchdog, name="stall-watchdog", daemon=True).start()
        else:
            if not self.lb.get_all_endpoints():
                self.lb.add_endpoint(Endpoint(id="local-sim", url="", name="simulated LLM", type="llm",
                                              max_connections=self.cfg.queue.worker.max_concurrent))
            for tier in self.gateway.tiers:
                self._workers += self.factory.create_workers("standard", 1, self._simulate, queue_name=tier) or []

    def stop(self) -> None:
        self._stop.set()
        self._wake.set()
        if self.ring is not None:
            self.ring.wake_all()
        if self.telemetry is not None:
            self.telemetry.stop()
        if self.peers is not None:
            self.peers.stop()
        for t in (self._loop_thread, self._ring_thread, self._snap_thread):
            if t is not None:
                t.join(timeout=10)
        if self.cfg.queue.snapshot_path and self.role != "ingress":
            self.snapshot()
        self.batcher.close()
        self.factory.close()
        self.state.stop()
        self.resources.stop()
        self.lb.stop()

    # ------------------------------------------------------------------ threads
    def _bind_device(self) -> None:
        """Make this thread's current HIP device the backend's GPU.  The
        current device (and with it ``torch.cuda.Event()`` / current-stream
        defaults) is per THREAD: a serve-loop thread of rank 3 would
        otherwise record its step events on device 0's stream."""
        if self._bound.__dict__.get("ok"):
            return
        self._bound.ok = True
        dev = getattr(self.engine, "device", None) if self.engine is not None else None
        if dev is not None and getattr(dev, "type", "") == "cuda":
            import torch
            torch.cuda.set_device(dev)
        elif self.gpu:
            import torch
            if torch.cuda.is_available():
                torch.cuda.set_device(torch.cuda.current_device() if self._main_device is None
                                      else self._main_device)

    # ------------------------------------------------------------------ ingest
    def _flush(self, msgs: Sequence[Message]) -> List[Optional[QueueError]]:
        self._bind_device()
        self.preprocessor.process_batch(msgs, use_gpu=self.preprocessor.gpu_enabled(),
                                        prompt_cap=self.gateway.prompt_cap)
        for m in msgs:
            if not m.queue_name:
                m.queue_name = priority_name(m.priority)
        if self.role == "ingress":
            n = self.ring.put_messages(msgs)
            errs = [None] * n + [QueueFull(f"shared request ring {self.ring.name} is full")] * (len(msgs) - n)
        else:
            errs = self.standard.push_routed(msgs)
        for m, e in zip(msgs, errs):
            if e is None:
                self.messages.put(m)
                self._accepted += 1
        self._wake.set()
        return errs

    def submit(self, msg: Message, timeout_s: float = 30.0) -> Optional[QueueError]:
        """Preprocess (micro-batched on the GPU) and enqueue one message."""
        return self.submit_future(msg).result(timeout=timeout_s)

    def submit_future(self, msg: Message):
        """Non-blocking ``submit``: a concurrent Future of the queue error
        (None on success).  HTTP handlers await it instead of blocking the
        event loop for the micro-batch window."""
        if not msg.arrival_ns:
            msg.arrival_ns = time.monotonic_ns()
        return self.batcher.submit(msg)

    def messages_seen(self) -> int:
        """Messages accepted through this app's ingress (micro-batcher)."""
        return self._accepted

    def estimated_wait_ns(self, msg: Message) -> int:
        """Requests ahead of this one / observed dispatch rate (reference:
        fixed per-tier constants, used until a rate is known)."""
        rate = self._dispatch_rate()
        if rate <= 0:
            return _REF_WAIT_NS.get(msg.priority, 15_000_000_000)
        ahead = 0
        for t, name in enumerate(self.gateway.tiers):
            if self.gateway.tier_prio[t] <= msg.priority:
                ahead += self.standard.size(name)
        return int(ahead / rate * 1e9)

    def _dispatch_rate(self) -> float:
        d = list(self._dispatch_times)
        if len(d) < 2 or d[-1][0] <= d[0][0]:
            return 0.0
        return (d[-1][1] - d[0][1]) / (d[-1][0] - d[0][0])

    # ------------------------------------------------------------------ health
    def set_endpoint_status(self, eid: str, status: str) -> None:
        """LB endpoint status; for this process's own GPU endpoint also the
        gateway's health (unhealthy evacuates the backend, healthy re-admits)."""
        self.lb.update_endpoint_status(eid, status)
        if self.engine is not None and eid == f"gpu{self.gateway.rank}":
            self.gateway.set_healthy(status == "healthy", f"operator set {status}", failure=False)

    def _gpu_unhealthy(self, gpu: int, reason: str) -> None:
        """Telemetry callback (ECC / amd-smi failure)."""
        try:
            self.lb.update_endpoint_status(f"gpu{gpu}", "unhealthy")
        except Exception:
            pass
        if self.engine is not None and gpu == getattr(self.engine, "gpu_index", -1):
            self.gateway.set_healthy(False, reason)

    def start_telemetry(self, pages: Dict[int, object]):
        """N8 amd-smi poller -> load pages, metrics, ResourceScheduler, health."""
        from ..backend.telemetry import TelemetryService
        self.telemetry = TelemetryService(self.cfg.gpu.telemetry_period_ms, pages=pages, metrics=self.metrics,
                                          resource_scheduler=self.resources, on_unhealthy=self._gpu_unhealthy)
        if self.telemetry.available:
            self.telemetry.start()
        return self.telemetry

    # ------------------------------------------------------------------ checkpoint
    def snapshot_file(self) -> str:
        """This process's snapshot: ``queue.snapshot_path`` for one rank,
        ``<path>.rank<r>`` for rank r of a multi-GPU job (every rank holds
        the queues of the requests it popped; one shared file would be
        overwritten by each rank in turn and replayed N times)."""
        path, gw = self.cfg.queue.snapshot_path, self.gateway
        return path if gw.world <= 1 else f"{path}.rank{gw.rank}"

    def _snapshots_to_resume(self) -> List[str]:
        """The snapshots this rank replays at start: its own, plus those of
        ranks a previous job of a different size had (rank k's file goes to
        rank k mod world; a single-rank file to rank 0)."""
        import glob
        import re
        path, gw = self.cfg.queue.snapshot_path, self.gateway
        out = [path] if gw.rank == 0 else []
        for f in sorted(glob.glob(glob.escape(path) + ".rank*")):
            m = re.fullmatch(re.escape(path) + r"\.rank(\d+)", f)
            if m and int(m.group(1)) % max(1, gw.world) == gw.rank:
                out.append(f)
        return out

    def snapshot(self, path: str = "") -> Dict[str, int]:
        """Write queued + in-flight + delayed + dead-lettered messages (JSONL)."""
        from ..queue.snapshot import write_snapshot
        inflight = [m for m in self.messages.values() if m.status == MessageStatus.PROCESSING]
        return write_snapshot(self.factory, path or self.snapshot_file(), inflight)

    def _snapshot_loop(self) -> None:
        period = self.cfg.queue.snapshot_interval / 1e9
        while not self._stop.wait(period):
            try:
                self.snapshot()
            except OSError as e:
                self.log.error("Queue snapshot failed", error=str(e))

    # ------------------------------------------------------------------ shared rings
    def _ring_loop(self) -> None:
        """Dispatcher: drain the request ring into the local queue.  Records
        from a Python ingress are already preprocessed; RAW records from the
        native HTTP ingress are preprocessed here in one batch per drain."""
        from .shm_bridge import TAG_RAW, decode_message, decode_raw
        self._bind_device()
        while not self._stop.is_set():
            recs = self.ring.get_records(self.cfg.preprocessor.max_batch, timeout_ms=100)
            if not recs:
                continue
            now = time.time_ns()
            ready, raw, bad = [], [], []
            undecodable: List[Message] = []
            for tag, b in recs:
                if tag == TAG_RAW:
                    try:
                        m = decode_raw(b)
                    except Exception as e:
                        # the native scanner already refuses what json.loads /
                        # Message.from_dict refuse (400 at the door); a record
                        # that still fails here was acknowledged (202), so it
                        # is accounted for, never silently dropped: status
                        # failed, dead-letter queue, metric, event to the ingress
                        undecodable.append(self._undecodable(b, e))
                        continue
                    m.created_at = m.updated_at = now
                    raw.append(m)
                else:
                    ready.append(decode_message(b))
            if raw:
                self.preprocessor.process_batch(raw, use_gpu=self.preprocessor.gpu_enabled(),
                                                prompt_cap=self.gateway.prompt_cap)
                ready.extend(raw)
            for m in ready:
                if not m.queue_name:
                    m.queue_name = priority_name(m.priority)
            errs = self.standard.push_routed(ready)
            for m, e in zip(ready, errs):
                if e is None:
                    self.messages.put(m)
                    self._accepted += 1
                else:
                    m.status = MessageStatus.FAILED
                    bad.append(m)
            if bad:
                self.ring.put_events(bad, error="queue full")
            if undecodable:
                self.factory.dead_letter_queue.push_many(undecodable, "undecodable request body", "ingress")
                self.metrics.requests_rejected.labels("undecodable").inc(len(undecodable))
                for m in undecodable:
                    self.messages.put(m)
                self.ring.put_events(undecodable, error="undecodable request body")
            self._wake.set()

    def _rank_ring_loop(self) -> None:
        """Role "rank": pop raw requests from the shared ring (and this
        rank's extra rings) into the gateway inbox.  Preprocessing runs in the
        serve loop's ingest (one overlapped GPU batch per tick on THIS rank's
        GPU), and queueing goes through the gateway, so conversation pins and
        the per-tick planner see every message -- the same path bench.py
        measures.  Messages with a conversation_id arrive on rank 0's ring
        (the native front door routes them there): rank 0 owns conversation
        state and records the turn like ``POST /api/v1/messages`` does."""
        from .shm_bridge import TAG_RAW, decode_message, decode_raw
        # No backpressure: the ring is FIFO and the per-rank queues are
        # priority queues, so requests leave the ring as fast as the ranks can
        # take them (a per-rank backpressure threshold was measured to hold
        # realtime requests behind normal ones in the ring: realtime p99 160
        # -> 214 ms, profiles/r3_http_multirank_2ranks_1gpu_5000_backpressure.json).
        # Every rank's ring thread wakes on the same push and takes what
        # brings its total up to an even 1/world share of the ring's traffic
        # (``ShmRing::pop`` balanced: ``share`` + ``who``); a rank that has
        # not polled for 2 ms is skipped, so a busy or dead rank never
        # strands records.  Greedy pops gave 47-74k per rank at 33k req/s,
        # a per-pop 1/world split 37-69k
        # (profiles/r4_http_frontdoor_8ranks_box16{,_fair}.jsonl).
        mb = self.cfg.preprocessor.max_batch
        share = max(1, self.gateway.world)
        while not self._stop.is_set():
            got = []
            for r in self.extra_rings:               # rank 0's conversation ring
                got.extend(r.get_records(mb, timeout_ms=0))
            got.extend(self.ring.get_records(mb, timeout_ms=0 if got else (5 if self.extra_rings else 20),
                                             share=share, who=self.gateway.rank if share > 1 else -1))
            if not got:
                continue
            now = time.time_ns()
            msgs, undecodable = [], []
            for tag, b in got:
                try:
                    m = decode_raw(b) if tag == TAG_RAW else decode_message(b)
                except Exception as e:               # noqa: BLE001 -- accounted for below
                    undecodable.append(self._undecodable(b, e))
                    continue
                if tag == TAG_RAW:
                    m.created_at = m.updated_at = now
                m.metadata["ingest_rank"] = self.gateway.rank
                if m.conversation_id:
                    self._record_turn(m)
                msgs.append(m)
                self.messages.put(m)
            if undecodable:
                self.factory.dead_letter_queue.push_many(undecodable, "undecodable request body", "ingress")
                self.metrics.requests_rejected.labels("undecodable").inc(len(undecodable))
                for m in undecodable:
                    self.messages.put(m)
            if msgs:
                self._accepted += len(msgs)
                self.gateway.submit(msgs)
                self._wake.set()

    def _record_turn(self, m: Message) -> None:
        """Conversation bookkeeping of a submitted turn (``POST
        /api/v1/messages`` with a conversation_id, `api/handlers.go:700`)."""
        from ..conversation.state_manager import ConversationNotFound
        cid = m.conversation_id
        self.state.get_conversation(cid, m.user_id)
        home = self.state.home_gpu(cid)
        if home >= 0:
            m.metadata.setdefault("home_gpu", home)
        try:
            self.state.add_message(cid, m)
        except ConversationNotFound:
            pass

    @staticmethod
    def _undecodable(b: bytes, err: BaseException) -> Message:
        mid = b[8:44].rstrip(b"\x00").decode("ascii", "replace") if len(b) >= 44 else ""
        m = Message(id=mid, status=MessageStatus.FAILED, metadata={"error": f"undecodable body: {err}"})
        m.arrival_ns = int.from_bytes(b[0:8], "little", signed=True) if len(b) >= 8 else 0
        return m

    def reset_latency(self) -> None:
        """Start a fresh latency window (operators / load tests)."""
        self.gateway.reset_latency()

    def _event_loop(self) -> None:
        """Ingress: apply status events from the dispatcher to the message store."""
        while not self._stop.is_set():
            for ev in self.ring.get_events(4096, timeout_ms=100):
                m = self.messages.get(ev["id"])
                if m is None:
                    continue
                m.status = ev["status"]
                m.endpoint_id = ev["endpoint_id"]
                m.dispatched_at = ev["dispatched_at"]
                m.completed_at = ev["completed_at"]
                m.retry_count = ev["retry_count"]
                if ev["error"]:
                    m.metadata["error"] = ev["error"]

    # ------------------------------------------------------------------ dispatch
    def _gc_maintenance(self, now: float) -> None:
        """See ``server.gc_freeze_interval``: keep full GC scans off the
        request path."""
        import gc
        sc = self.cfg.server
        fi, fu = sc.gc_freeze_interval / 1e9, sc.gc_full_interval / 1e9
        if fi <= 0:
            return
        if fu > 0 and now - self._gc_full_at >= fu:
            gc.unfreeze()
            gc.collect()
            self._gc_full_at = now
        if now - self._gc_freeze_at >= fi:
            gc.freeze()
            self._gc_freeze_at = now

    def _serve_loop(self) -> None:
        import gc
        from ..backend.engine import BackendHung
        from ..parallel.comm import PeerLost
        gw = self.gateway
        self._bind_device()
        if self.cfg.server.gc_freeze_interval > 0:
            gc.collect()
            gc.freeze()
        self._gc_freeze_at = self._gc_full_at = time.monotonic()
        while True:
            self._gc_maintenance(time.monotonic())
            if self._stop.is_set():
                gw.request_stop()
            if gw.peers_stopping:
                break
            try:
                gw.tick()
            except (PeerLost, BackendHung) as e:
                # a peer rank died, or this GPU stopped completing steps: this
                # job cannot tick any more; leave with a failure status so the
                # launcher restarts a fresh group
                self.fatal = e
                self.log.error("peer rank lost; stopping" if isinstance(e, PeerLost)
                               else "GPU step hung; stopping", error=str(e))
                self._stop.set()
                break
            except Exception as e:                    # noqa: BLE001 -- a bug must not leave a zombie
                # anything else is a defect: without this the dispatcher thread
                # would die silently and the API keep accepting requests that
                # nothing dispatches; fail the process so it is restarted
                import traceback
                self.fatal = e
                self.log.error("serve loop failed; stopping", error=repr(e),
                               traceback=traceback.format_exc(limit=20))
                self._stop.set()
                break
            self._dispatch_times.append((time.monotonic(), gw.counters["dispatched"]))
            idle = (gw.cluster_idle if gw.world > 1 else
                    self.engine.inflight() == 0 and gw.pending() == 0)
            if idle:                      # (multi-rank: only when every rank is idle)
                self._wake.wait(0.01)
                self._wake.clear()

    def _simulate(self, ctx, msg: Message):
        """CPU mode process function: LB pick -> simulated LLM latency -> release."""
        ep = self.lb.get_endpoint(msg, msg.conversation_id)
        msg.endpoint_id = ep.id
        t0 = time.monotonic_ns()
        if msg.dispatched_at == 0:
            msg.dispatched_at = t0
            self.gateway.rec.record(np.array([min(max(msg.priority, 1), 4) - 1]),
                                    np.array([t0 - (msg.arrival_ns or t0)]),
                                    np.array([t0 - (msg.enqueued_at or t0)]))
            self.gateway.counters["dispatched"] += 1
            self._dispatch_times.append((time.monotonic(), self.gateway.counters["dispatched"]))
        dur = self.simulate_ns[min(max(msg.priority, 1), 4) - 1] / 1e9
        err = None
        if ctx.err() is None:
            time.sleep(dur)
        fail = msg.metadata.get("simulate_error") if isinstance(msg.metadata, dict) else None
        if fail:
            err = RuntimeError(str(fail))
        self.lb.release_endpoint(ep.id, time.monotonic_ns() - t0, err is not None)
        if err is None:
            self._on_complete(msg)
        return err

    def _on_complete(self, msg: Message) -> None:
        msg.status = MessageStatus.COMPLETED
        msg.completed_at = time.time_ns()
        if self.role == "dispatcher":
            self.ring.put_events([msg])
        if msg.conversation_id:
            conv = self.state.find_conversation(msg.conversation_id)
            if conv is not None and msg.endpoint_id.startswith("gpu"):
                try:
                    self.state.set_home_gpu(msg.conversation_id, int(msg.endpoint_id[3:]))
                except ValueError:
                    pass

    # ------------------------------------------------------------------ stats
    def queue_stats(self) -> Dict[str, object]:
        out: Dict[str, object] = {}
        for name, mgr in self.factory.managers().items():
            out[name] = {q: s.to_dict() for q, s in mgr.get_all_queue_stats().items()}
        out["workers"] = {q: [w.to_dict() for w in ws] for q, ws in self.factory.get_worker_stats().items()}
        out["dispatch"] = dict(self.gateway.counters)
        out["latency"] = self.gateway.rec.summary()          # arrival -> dispatch (and enqueue -> dispatch)
        self.gateway.flush_latency()
        out["latency_e2e"] = self.gateway.rec_done.summary()  # arrival -> completion
        out["dead_letter"] = self.factory.dead_letter_queue.size()
        if self.ring is not None:
            out["rings"] = self.ring.stats()
        out["delayed"] = self.factory.delayed_queue.size()
        if self.peers is not None:
            out["job"] = self.job_stats()         # every GPU rank of the multi-GPU front door
        return out
