"""gRPC front-end: service ``llmq.v1.MessageQueue`` next to the REST API.

The reference only *documents* a gRPC server (`docs/performance.md:716-749`:
keepalive 30 s / 5 s, 4 MiB message caps, 1000 concurrent streams, gzip) --
there is no gRPC code in it.  Here it is a real service on
the same gateway the REST routes drive:

  * ``Submit`` (unary), ``SubmitBatch`` (many messages per call -- the
    high-rate path: per-message gRPC costs are paid once per batch) and
    ``SubmitStream`` (bidirectional: a client keeps one HTTP/2 stream open and
    pipelines submissions; replies come back in order, and concurrent
    submissions share the gateway's GPU preprocess micro-batch);
  * ``GetMessage`` / ``WatchMessage`` (server-streaming status changes until
    the message reaches a terminal state -- result delivery without polling);
  * ``QueueStats`` and ``Health``.

No ``protoc`` in the image, so the descriptors are built at import time from
the table below (``descriptor_pb2`` + ``message_factory``) -- real protobuf
wire format; ``proto/llmq.proto`` is generated from the same table
(``proto_source()``, a test keeps the checked-in file in sync).

Authentication / RBAC / rate limits reuse the native guard of the REST API and
the native ingress (``api/security.py``): credentials come from the call
metadata (``authorization: Bearer <jwt>`` or the configured API-key header),
each RPC is checked as its REST twin (``Submit`` = ``POST /api/v1/messages``)
and failures map to UNAUTHENTICATED / PERMISSION_DENIED / RESOURCE_EXHAUSTED.
"""
from __future__ import annotations

import json
import queue as _queue
import threading
import time
from concurrent import futures
from typing import Any, Dict, List, Optional, Tuple

import grpc
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

from ..models.message import Message, MessageStatus, PriorityParseError, format_time
from .security import guard_from_config

PACKAGE = "llmq.v1"
SERVICE = "MessageQueue"
VERSION = "1.0.0"
TERMINAL = (MessageStatus.COMPLETED, MessageStatus.FAILED, MessageStatus.TIMEOUT)

_S, _I32, _I64, _BOOL, _MSG = "string", "int32", "int64", "bool", "message"
# message -> [(field, number, type, repeated, message type)]
MESSAGES: Dict[str, List[Tuple[str, int, str, bool, str]]] = {
    "Empty": [],
    "SubmitRequest": [("id", 1, _S, False, ""), ("content", 2, _S, False, ""), ("user_id", 3, _S, False, ""),
                      ("conversation_id", 4, _S, False, ""),
                      # 0 = let the preprocessor decide; else 1 (realtime) .. 4 (low)
                      ("priority", 5, _I32, False, ""), ("priority_name", 6, _S, False, ""),
                      ("metadata", 7, _MSG, True, "SubmitRequest.MetadataEntry"),
                      ("timeout_ms", 8, _I64, False, "")],
    "SubmitReply": [("message_id", 1, _S, False, ""), ("priority", 2, _I32, False, ""),
                    ("queue_time", 3, _S, False, ""), ("estimated_wait_ns", 4, _I64, False, ""),
                    # per-item outcome on SubmitStream (unary calls use the status instead)
                    ("code", 5, _I32, False, ""), ("error", 6, _S, False, "")],
    "SubmitBatchRequest": [("items", 1, _MSG, True, "SubmitRequest")],
    "SubmitBatchReply": [("items", 1, _MSG, True, "SubmitReply")],
    "MessageRef": [("message_id", 1, _S, False, ""), ("timeout_ms", 2, _I64, False, "")],
    "MessageInfo": [("id", 1, _S, False, ""), ("conversation_id", 2, _S, False, ""),
                    ("user_id", 3, _S, False, ""), ("content", 4, _S, False, ""),
                    ("priority", 5, _I32, False, ""), ("status", 6, _S, False, ""),
                    ("queue_name", 7, _S, False, ""), ("retry_count", 8, _I32, False, ""),
                    ("created_at", 9, _S, False, ""), ("updated_at", 10, _S, False, ""),
                    ("completed_at", 11, _S, False, ""), ("metadata_json", 12, _S, False, "")],
    "TierStats": [("name", 1, _S, False, ""), ("priority", 2, _I32, False, ""), ("pending", 3, _I64, False, ""),
                  ("processing", 4, _I64, False, ""), ("completed", 5, _I64, False, ""),
                  ("failed", 6, _I64, False, "")],
    "QueueStatsReply": [("tiers", 1, _MSG, True, "TierStats"), ("total_pending", 2, _I64, False, ""),
                        ("dead_letter", 3, _I64, False, ""), ("delayed", 4, _I64, False, "")],
    "HealthReply": [("status", 1, _S, False, ""), ("version", 2, _S, False, ""), ("time", 3, _S, False, "")],
}
MAPS = {"SubmitRequest.MetadataEntry": (_S, _S)}
# rpc -> (request, response, client streams, server streams, REST twin for the guard)
RPCS: Dict[str, Tuple[str, str, bool, bool, Tuple[str, str]]] = {
    "Submit": ("SubmitRequest", "SubmitReply", False, False, ("POST", "/api/v1/messages")),
    "SubmitStream": ("SubmitRequest", "SubmitReply", True, True, ("POST", "/api/v1/messages")),
    "SubmitBatch": ("SubmitBatchRequest", "SubmitBatchReply", False, False, ("POST", "/api/v1/messages")),
    "GetMessage": ("MessageRef", "MessageInfo", False, False, ("GET", "/api/v1/messages/{id}")),
    "WatchMessage": ("MessageRef", "MessageInfo", False, True, ("GET", "/api/v1/messages/{id}")),
    "QueueStats": ("Empty", "QueueStatsReply", False, False, ("GET", "/api/v1/queues/stats")),
    "Health": ("Empty", "HealthReply", False, False, ("GET", "/api/v1/health")),
}
_FT = descriptor_pb2.FieldDescriptorProto
_TYPES = {_S: _FT.TYPE_STRING, _I32: _FT.TYPE_INT32, _I64: _FT.TYPE_INT64, _BOOL: _FT.TYPE_BOOL,
          _MSG: _FT.TYPE_MESSAGE}


def _file_descriptor() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name="llmq/v1/queue.proto", package=PACKAGE, syntax="proto3")
    for name, fields in MESSAGES.items():
        mp = fd.message_type.add(name=name)
        for fname, num, typ, rep, tname in fields:
            f = mp.field.add(name=fname, number=num, type=_TYPES[typ],
                             label=_FT.LABEL_REPEATED if rep else _FT.LABEL_OPTIONAL)
            if tname:
                f.type_name = f".{PACKAGE}.{tname}"
        for entry, (kt, vt) in MAPS.items():
            parent, ename = entry.split(".")
            if parent == name:
                e = mp.nested_type.add(name=ename)
                e.options.map_entry = True
                e.field.add(name="key", number=1, type=_TYPES[kt], label=_FT.LABEL_OPTIONAL)
                e.field.add(name="value", number=2, type=_TYPES[vt], label=_FT.LABEL_OPTIONAL)
    svc = fd.service.add(name=SERVICE)
    for rpc, (req, resp, cs, ss, _) in RPCS.items():
        svc.method.add(name=rpc, input_type=f".{PACKAGE}.{req}", output_type=f".{PACKAGE}.{resp}",
                       client_streaming=cs, server_streaming=ss)
    return fd


_POOL = descriptor_pool.DescriptorPool()
_FILE = _POOL.Add(_file_descriptor())
pb: Dict[str, Any] = {n: message_factory.GetMessageClass(_POOL.FindMessageTypeByName(f"{PACKAGE}.{n}"))
                      for n in MESSAGES}


def proto_source() -> str:
    """``proto/llmq.proto``: the schema for clients in other languages."""
    out = ["// Generated from llm_message_queue_amd/api/grpc_server.py (MESSAGES / RPCS); do not edit.",
           'syntax = "proto3";', "", f"package {PACKAGE};", ""]
    for name, fields in MESSAGES.items():
        out.append(f"message {name} {{")
        for fname, num, typ, rep, tname in fields:
            if tname in MAPS:
                kt, vt = MAPS[tname]
                out.append(f"  map<{kt}, {vt}> {fname} = {num};")
            else:
                t = tname if typ == _MSG else typ
                out.append(f"  {'repeated ' if rep else ''}{t} {fname} = {num};")
        out.append("}")
        out.append("")
    out.append(f"service {SERVICE} {{")
    for rpc, (req, resp, cs, ss, _) in RPCS.items():
        out.append(f"  rpc {rpc}({'stream ' if cs else ''}{req}) returns ({'stream ' if ss else ''}{resp});")
    out.append("}")
    return "\n".join(out) + "\n"


def server_options(max_streams: int = 1000, max_msg_bytes: int = 4 << 20) -> List[Tuple[str, int]]:
    """The documented server tuning (`docs/performance.md:720-746` of the reference)."""
    return [("grpc.keepalive_time_ms", 30_000), ("grpc.keepalive_timeout_ms", 5_000),
            ("grpc.keepalive_permit_without_calls", 1), ("grpc.http2.min_ping_interval_without_data_ms", 5_000),
            ("grpc.max_receive_message_length", max_msg_bytes), ("grpc.max_send_message_length", max_msg_bytes),
            ("grpc.max_concurrent_streams", max_streams)]


class _Service:
    def __init__(self, gw_app, guard):
        self.G = gw_app
        self.guard = guard

    # ------------------------------------------------------------------ guard
    def _check(self, context, rpc: str, user: str = ""):
        """Guard verdict for one call / one item: (code, reason, retry_after)."""
        if self.guard is None or rpc == "Health":
            return 0, "", 0.0
        md = {k.lower(): v for k, v in context.invocation_metadata()}
        method, path = RPCS[rpc][4]
        peer = context.peer() or ""                       # "ipv4:1.2.3.4:port" / "ipv6:[::1]:port"
        ip = peer.split(":", 1)[1].rsplit(":", 1)[0].strip("[]") if ":" in peer else ""
        code, _, _, reason, retry = self.guard.check(method, path.replace("{id}", "x"), ip,
                                                     md.get(self.guard.key_header.lower(), ""),
                                                     md.get("authorization", ""), user or md.get("x-user-id", ""))
        return code, reason, retry

    def _admit(self, context, rpc: str, user: str = "") -> None:
        code, reason, retry = self._check(context, rpc, user)
        if code == 401:
            context.abort(grpc.StatusCode.UNAUTHENTICATED, reason)
        if code == 403:
            context.abort(grpc.StatusCode.PERMISSION_DENIED, reason)
        if code == 429:
            context.set_trailing_metadata((("retry-after", str(max(1, int(retry + 0.999)))),))
            context.abort(grpc.StatusCode.RESOURCE_EXHAUSTED, reason)

    # ------------------------------------------------------------------ submit
    def _bind(self, req) -> Message:
        d: Dict[str, Any] = {"id": req.id, "content": req.content, "user_id": req.user_id,
                             "conversation_id": req.conversation_id, "metadata": dict(req.metadata)}
        if req.priority:
            if not 1 <= req.priority <= 4:
                raise ValueError(f"priority {req.priority} outside 1 (realtime) .. 4 (low)")
            d["priority"] = int(req.priority)
        elif req.priority_name:
            d["priority"] = req.priority_name
        if req.timeout_ms > 0:
            d["timeout"] = int(req.timeout_ms) * 1_000_000
        m = Message.from_dict(d)
        if not m.id:
            import uuid
            m.id = str(uuid.uuid4())
        m.created_at = m.updated_at = time.time_ns()
        return m

    def _reply(self, m: Message, err) -> Any:
        if err is not None:
            return pb["SubmitReply"](message_id=m.id, code=500, error=f"Failed to queue message: {err}")
        if m.conversation_id:
            self.G.state.get_conversation(m.conversation_id, m.user_id)
            try:
                self.G.state.add_message(m.conversation_id, m)
            except Exception:
                pass
        return pb["SubmitReply"](message_id=m.id, priority=int(m.priority), queue_time=format_time(time.time_ns()),
                                 estimated_wait_ns=int(self.G.estimated_wait_ns(m)), code=202)

    def Submit(self, req, context):
        self._admit(context, "Submit", req.user_id)
        try:
            m = self._bind(req)
        except (ValueError, PriorityParseError, TypeError) as e:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, f"Invalid message format: {e}")
        try:
            err = self.G.submit_future(m).result(timeout=30.0)
        except Exception as e:                              # noqa: BLE001 - reported to the caller
            err = e
        r = self._reply(m, err)
        if r.code != 202:
            context.abort(grpc.StatusCode.UNAVAILABLE, r.error)
        return r

    def _submit_many(self, reqs, context):
        """Bind + submit every item first (one micro-batch), then collect.
        Every item is its own request to the guard (global / IP / user
        buckets are charged per message, so batching does not bypass them);
        a rejected item gets its status in ``code`` / ``error``."""
        staged = []
        for req in reqs:
            code, reason, _ = self._check(context, "Submit", req.user_id)
            if code:
                staged.append((None, req.id, code, reason))
                continue
            try:
                m = self._bind(req)
            except (ValueError, PriorityParseError, TypeError) as e:
                staged.append((None, req.id, 400, f"Invalid message format: {e}"))
                continue
            staged.append((m, self.G.submit_future(m), 0, ""))
        return staged

    def _collect(self, item):
        m, fut, code, why = item
        if m is None:
            return pb["SubmitReply"](message_id=fut, code=code, error=why)
        try:
            err = fut.result(timeout=30.0)
        except Exception as e:                              # noqa: BLE001
            err = e
        return self._reply(m, err)

    def SubmitBatch(self, req, context):
        """Many submissions per RPC: per-message gRPC costs (HTTP/2 frames,
        completion-queue round trips) are paid once per batch."""
        if len(req.items) > 10_000:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "at most 10000 items per batch")
        staged = self._submit_many(req.items, context)
        if staged and all(x[0] is None and x[2] in (401, 403) for x in staged):
            # bad credentials for the whole call: fail it as a unary call would
            code, why = staged[0][2], staged[0][3]
            context.abort(grpc.StatusCode.UNAUTHENTICATED if code == 401 else grpc.StatusCode.PERMISSION_DENIED, why)
        return pb["SubmitBatchReply"](items=[self._collect(x) for x in staged])

    def SubmitStream(self, request_iterator, context):
        """Replies in request order.  A reader thread submits as requests arrive
        so a pipelining client fills the micro-batch; this generator waits on
        each future in turn.  Per-item failures ride in ``code``/``error``."""
        self._admit(context, "SubmitStream")
        pending: "_queue.Queue" = _queue.Queue(maxsize=4096)
        END = object()

        def put(item) -> bool:
            # bounded queue: a client that stops reading replies must not pin
            # this thread forever once the call is gone
            while context.is_active():
                try:
                    pending.put(item, timeout=0.5)
                    return True
                except _queue.Full:
                    continue
            return False

        def reader():
            try:
                for req in request_iterator:
                    if not all(put(item) for item in self._submit_many((req,), context)):
                        return
            except grpc.RpcError:
                pass
            finally:
                put(END)

        threading.Thread(target=reader, daemon=True, name="grpc-submit-reader").start()
        while context.is_active():
            try:
                item = pending.get(timeout=0.5)
            except _queue.Empty:
                continue
            if item is END:
                return
            yield self._collect(item)

    # ------------------------------------------------------------------ read side
    @staticmethod
    def _info(m: Message):
        return pb["MessageInfo"](id=m.id, conversation_id=m.conversation_id, user_id=m.user_id, content=m.content,
                                 priority=int(m.priority), status=m.status, queue_name=m.queue_name,
                                 retry_count=int(m.retry_count), created_at=format_time(m.created_at),
                                 updated_at=format_time(m.updated_at), completed_at=format_time(m.completed_at),
                                 metadata_json=json.dumps(m.metadata, default=str, separators=(",", ":")))

    def _lookup(self, mid: str) -> Optional[Message]:
        """This process's message, else a copy from the GPU rank that popped
        it (multi-GPU front door)."""
        m = self.G.messages.get(mid)
        if m is None and getattr(self.G, "peers", None) is not None:
            d = self.G.find_message(mid)
            if d is not None:
                m = Message.from_dict(d)
                m.status = d.get("status", m.status)
        return m

    def GetMessage(self, req, context):
        self._admit(context, "GetMessage")
        m = self._lookup(req.message_id)
        if m is None:
            context.abort(grpc.StatusCode.NOT_FOUND, "Message not found")
        return self._info(m)

    def WatchMessage(self, req, context):
        """One ``MessageInfo`` per observed status change; ends at a terminal
        status, at ``timeout_ms`` (default 60 s) or when the client leaves.
        Each open watch holds one handler thread (``server.grpc_max_workers``
        bounds concurrent watches plus in-flight calls)."""
        self._admit(context, "WatchMessage")
        deadline = time.monotonic() + (req.timeout_ms / 1e3 if req.timeout_ms > 0 else 60.0)
        last = None
        nap = 0.002                                   # poll backoff 2 -> 50 ms, reset on change
        while context.is_active() and time.monotonic() < deadline:
            m = self._lookup(req.message_id)
            if m is None:
                if last is None:
                    context.abort(grpc.StatusCode.NOT_FOUND, "Message not found")
                return
            if m.status != last:
                last = m.status
                nap = 0.002
                yield self._info(m)
                if last in TERMINAL:
                    return
            time.sleep(nap)
            nap = min(0.05, nap * 2)

    def QueueStats(self, req, context):
        self._admit(context, "QueueStats")
        G = self.G
        job = G.job_stats() if getattr(G, "peers", None) is not None else None    # every GPU rank
        tiers = []
        for t, name in enumerate(G.gateway.tiers):
            c = job["tiers"][name] if job else dict(zip(("pending", "processing", "completed", "failed"),
                                                        G._tier_counts(name)))
            tiers.append(pb["TierStats"](name=name, priority=int(G.gateway.tier_prio[t]), pending=c["pending"],
                                         processing=c["processing"], completed=c["completed"], failed=c["failed"]))
        return pb["QueueStatsReply"](tiers=tiers, total_pending=sum(x.pending for x in tiers),
                                     dead_letter=job["dead_letter"] if job else G.factory.dead_letter_queue.size(),
                                     delayed=job["delayed"] if job else G.factory.delayed_queue.size())

    def Health(self, req, context):
        return pb["HealthReply"](status="ok", version=VERSION, time=format_time(time.time_ns()))


def _counted(fn, rpc: str, streaming: bool, metrics):
    """Count each call in ``llm_grpc_requests_total{method, code}``."""
    if metrics is None or not hasattr(metrics, "grpc_requests"):
        return fn

    def code_of(context, exc) -> str:
        c = context.code() if hasattr(context, "code") else None
        if c is None:
            return "OK" if exc is None else "UNKNOWN"
        return c.name

    if streaming:
        def gen(req, context):
            exc = None
            try:
                yield from fn(req, context)
            except BaseException as e:        # abort() / cancel / GeneratorExit
                exc = e
                raise
            finally:
                metrics.grpc_requests.labels(rpc, code_of(context, exc)).inc()
        return gen

    def unary(req, context):
        exc = None
        try:
            return fn(req, context)
        except BaseException as e:
            exc = e
            raise
        finally:
            metrics.grpc_requests.labels(rpc, code_of(context, exc)).inc()
    return unary


def _handler(svc: _Service) -> grpc.GenericRpcHandler:
    table = {}
    metrics = getattr(svc.G, "metrics", None)
    for rpc, (req, resp, cs, ss, _) in RPCS.items():
        make = {(False, False): grpc.unary_unary_rpc_method_handler,
                (False, True): grpc.unary_stream_rpc_method_handler,
                (True, True): grpc.stream_stream_rpc_method_handler,
                (True, False): grpc.stream_unary_rpc_method_handler}[(cs, ss)]
        table[rpc] = make(_counted(getattr(svc, rpc), rpc, ss, metrics), request_deserializer=pb[req].FromString,
                          response_serializer=pb[resp].SerializeToString)
    return grpc.method_handlers_generic_handler(f"{PACKAGE}.{SERVICE}", table)


class GrpcServer:
    """``llmq.v1.MessageQueue`` on ``host:port`` (0 = ephemeral; ``start``
    returns the bound port)."""

    def __init__(self, gw_app, port: int = 0, host: str = "0.0.0.0", max_workers: int = 32,
                 gzip: bool = True, tls_cert: str = "", tls_key: str = ""):
        """``tls_cert`` / ``tls_key``: PEM files -> TLS on the port
        (``server.grpc_tls_cert`` / ``server.grpc_tls_key``); empty = plaintext."""
        self.G = gw_app
        self.host, self.port = host, port
        self.creds = None
        if tls_cert or tls_key:
            if not (tls_cert and tls_key):
                raise ValueError("gRPC TLS needs both a certificate and a key")
            with open(tls_key, "rb") as k, open(tls_cert, "rb") as c:
                self.creds = grpc.ssl_server_credentials([(k.read(), c.read())])
        self._server = grpc.server(futures.ThreadPoolExecutor(max_workers=max_workers,
                                                              thread_name_prefix="grpc"),
                                   options=server_options(),
                                   compression=grpc.Compression.Gzip if gzip else None)
        self._server.add_generic_rpc_handlers((_handler(_Service(gw_app, guard_from_config(gw_app.cfg))),))

    def start(self) -> int:
        addr = f"{self.host}:{self.port}"
        self.port = (self._server.add_secure_port(addr, self.creds) if self.creds is not None
                     else self._server.add_insecure_port(addr))
        self._server.start()
        return self.port

    def stop(self, grace: float = 1.0) -> None:
        self._server.stop(grace).wait()


class GrpcClient:
    """Thin client for ``llmq.v1.MessageQueue`` (no generated stubs needed)."""

    def __init__(self, target: str, token: str = "", api_key: str = "", api_key_header: str = "x-api-key",
                 gzip: bool = False, root_cert: str = ""):
        """``root_cert``: PEM file of the CA (or the self-signed server
        certificate) -> TLS channel; empty = plaintext."""
        opts = [("grpc.max_receive_message_length", 4 << 20)]
        comp = grpc.Compression.Gzip if gzip else None
        if root_cert:
            with open(root_cert, "rb") as f:
                cred = grpc.ssl_channel_credentials(root_certificates=f.read())
            self.channel = grpc.secure_channel(target, cred, options=opts, compression=comp)
        else:
            self.channel = grpc.insecure_channel(target, options=opts, compression=comp)
        md = []
        if token:
            md.append(("authorization", f"Bearer {token}"))
        if api_key:
            md.append((api_key_header.lower(), api_key))
        self.metadata = tuple(md)
        for rpc, (req, resp, cs, ss, _) in RPCS.items():
            kind = {(False, False): self.channel.unary_unary, (False, True): self.channel.unary_stream,
                    (True, True): self.channel.stream_stream, (True, False): self.channel.stream_unary}[(cs, ss)]
            setattr(self, "_" + rpc, kind(f"/{PACKAGE}.{SERVICE}/{rpc}", request_serializer=pb[req].SerializeToString,
                                          response_deserializer=pb[resp].FromString))

    @staticmethod
    def request(content: str = "", **kw) -> Any:
        return pb["SubmitRequest"](content=content, **kw)

    def submit(self, content: str = "", timeout: float = 30.0, **kw):
        return self._Submit(self.request(content, **kw), timeout=timeout, metadata=self.metadata)

    def submit_batch(self, requests, timeout: float = 60.0):
        return self._SubmitBatch(pb["SubmitBatchRequest"](items=list(requests)), timeout=timeout,
                                 metadata=self.metadata).items

    def submit_stream(self, requests, timeout: Optional[float] = None):
        return self._SubmitStream(iter(requests), timeout=timeout, metadata=self.metadata)

    def get_message(self, message_id: str, timeout: float = 10.0):
        return self._GetMessage(pb["MessageRef"](message_id=message_id), timeout=timeout, metadata=self.metadata)

    def watch(self, message_id: str, timeout_ms: int = 60_000):
        return self._WatchMessage(pb["MessageRef"](message_id=message_id, timeout_ms=timeout_ms),
                                  metadata=self.metadata)

    def queue_stats(self, timeout: float = 10.0):
        return self._QueueStats(pb["Empty"](), timeout=timeout, metadata=self.metadata)

    def health(self, timeout: float = 10.0):
        return self._Health(pb["Empty"](), timeout=timeout, metadata=self.metadata)

    def close(self) -> None:
        self.channel.close()
