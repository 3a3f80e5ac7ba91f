"""REST API (component C17): the reference's 21 routes with the same
payloads (`api/handlers.go:75-118`), plus ``/metrics`` (D6) and the doc-only
extras of `docs/api.md` that the gateway can actually serve
(``GET /api/v1/queues/status``, ``GET /api/v1/config``,
``PUT /api/v1/messages/:id/status``, ``DELETE /api/v1/messages/:id``,
``GET /api/v1/conversations``, ``PUT /api/v1/conversations/:id``).

Behaviour notes vs the reference:
  * ``priority`` accepts ints or level names (D4); timeouts default to 30 s (D16);
  * stub routes are implemented (D24): get/list messages, preprocessor rule
    admin, remove message, dead-letter requeue by id / all;
  * ``GET /conversations/:id`` returns 404 for unknown ids (D19, the docs'
    contract); POST paths keep get-or-create;
  * ``setUserPriority`` accepts ``realtime`` (D18);
  * ``estimated_wait`` comes from live queue depth / dispatch rate;
  * CORS: echo an allowed Origin (or any, with "*"), allow credentials,
    OPTIONS -> 204 (`:121-148`);
  * doc-only features of the reference, off by default: API-key / JWT
    authentication, RBAC and token-bucket rate limits (``api/security.py``,
    401 / 403 / 429 + Retry-After), and the ``{"code","message","data",
    "timestamp"}`` response envelope (`docs/api.md:12-20`,
    ``server.response_envelope``).
"""
from __future__ import annotations

import asyncio
import dataclasses
import json
import math
import time
import uuid
from typing import Any, Dict, List, Optional, Sequence

from fastapi import FastAPI, Request
from fastapi.responses import JSONResponse, Response

from ..balancer.load_balancer import Endpoint, LoadBalancerError
from ..models.message import (ConversationNotFound, Message, MessageStatus,
                              PriorityParseError, format_time, level_priority_from_name, parse_priority,
                              priority_name)
from ..scheduler.resource_scheduler import Resource, ResourceError
from ..utils.metrics import CONTENT_TYPE_LATEST
from .security import guard_from_config, redact_config

VERSION = "1.0.0"
MAX_BODY = 4 << 20


def business_error_code(status: int, path: str, msg: str) -> Optional[int]:
    """The documented business / system error codes (`docs/api.md:745-771`
    of the reference: 1001-1010, 2001-2008) for an error response; reported
    as ``error_code`` in the envelope format."""
    m = (msg or "").lower()
    if status == 429:
        return 1009                                   # request rate too high
    if status == 408 or "timeout" in m or "deadline" in m:
        return 1010                                   # message processing timed out
    if status == 404:
        if "/conversations" in path:
            return 1005                               # conversation does not exist
        if "/messages" in path:
            return 1004                               # message does not exist
        return None
    if "full" in m:
        return 1007                                   # queue full
    if status == 400:
        if "priority" in m:
            return 1003                               # invalid priority
        if "user_id" in m:
            return 1006                               # invalid user id
        if "too long" in m:
            return 1002                               # content too long
        if "content" in m or "empty" in m or "eof" in m:
            return 1001                               # content empty
        return None
    if status == 503:
        return 2003                                   # queue service unavailable
    if status >= 500:
        if "redis" in m:
            return 2002
        if "database" in m or "postgres" in m or "sqlite" in m:
            return 2001
        if "queue" in m:
            return 2003
        return None
    return None


def _err(code: int, msg: str) -> JSONResponse:
    return JSONResponse({"error": msg}, status_code=code)


async def _json(request: Request) -> Any:
    raw = await request.body()
    if not raw:
        raise ValueError("EOF")
    return json.loads(raw)


def create_app(gw_app, allowed_origins: Optional[List[str]] = None,
               trusted_proxies: Sequence[str] = ()) -> FastAPI:
    """``gw_app`` is a ``gateway.app.GatewayApp``.

    ``trusted_proxies``: peer addresses whose ``X-Forwarded-For`` names the
    real client (the C++ front door on loopback, which drops any
    client-sent XFF and appends the connection's own address,
    `csrc/ingress/http_ingress.cpp` start_proxy).  Behind it every request's
    peer is 127.0.0.1, so without this the per-IP rate limit would put every
    proxied client into one bucket."""
    app = FastAPI(title="llm_message_queue_amd", version=VERSION)
    origins = allowed_origins if allowed_origins is not None else ["*"]
    G = gw_app

    # ------------------------------------------------------------------ guard
    # authentication / RBAC / rate limits (api/security.py; native checks).
    # Middleware order, outermost first: CORS -> envelope -> guard -> route.
    guard = guard_from_config(G.cfg)
    app.state.guard = guard
    trusted = frozenset(trusted_proxies)
    if guard is not None:
        @app.middleware("http")
        async def guard_mw(request: Request, call_next):
            if request.method == "OPTIONS":
                return await call_next(request)
            path = request.url.path
            user = request.headers.get("x-user-id", "") or request.query_params.get("user_id", "")
            if not user and request.method == "POST" and path.rstrip("/") == "/api/v1/messages":
                try:  # per-user limits key on the body's user_id (cached for the route)
                    body = json.loads(await request.body() or b"{}")
                    user = str(body.get("user_id", "") or "") if isinstance(body, dict) else ""
                except ValueError:
                    user = ""
            ip = request.client.host if request.client else ""
            if ip in trusted:
                fwd = request.headers.get("x-forwarded-for", "")
                if fwd:
                    ip = fwd.rsplit(",", 1)[-1].strip() or ip
            code, subject, role, reason, retry = guard.check(
                request.method, path, ip,
                request.headers.get(guard.key_header, ""), request.headers.get("authorization", ""), user)
            if code == 401:
                return JSONResponse({"error": reason}, status_code=401, headers={"WWW-Authenticate": "Bearer"})
            if code in (403, 429):
                hdrs = {"Retry-After": str(max(1, math.ceil(retry)))} if code == 429 else None
                return JSONResponse({"error": reason}, status_code=code, headers=hdrs)
            request.state.subject, request.state.role = subject, role
            return await call_next(request)

    # ------------------------------------------------------------------ envelope
    if G.cfg.server.response_envelope:
        @app.middleware("http")
        async def envelope(request: Request, call_next):
            resp = await call_next(request)
            if not resp.headers.get("content-type", "").startswith("application/json"):
                return resp
            raw = b"".join([chunk async for chunk in resp.body_iterator])
            try:
                payload = json.loads(raw) if raw else None
            except ValueError:
                return Response(raw, status_code=resp.status_code, headers=dict(resp.headers))
            code = resp.status_code
            env: Dict[str, Any] = {"code": code}
            if code >= 400:
                msg = payload.get("error", "") if isinstance(payload, dict) else ""
                env.update(message=msg or "error", error=msg or "error")
                biz = business_error_code(code, request.url.path, msg)
                if biz:
                    env["error_code"] = biz
            else:
                env.update(message="success", data=payload)
            env["timestamp"] = format_time(time.time_ns())
            hdrs = {k: v for k, v in resp.headers.items() if k.lower() not in ("content-length", "content-type")}
            return JSONResponse(env, status_code=code, headers=hdrs)

    # ------------------------------------------------------------------ body cap
    # same 4 MiB cap as the native ingress: a declared oversize body is
    # refused before it is read (413), not buffered into memory
    @app.middleware("http")
    async def body_cap(request: Request, call_next):
        cl = request.headers.get("content-length")
        if cl is not None:
            if not cl.isdigit():
                return JSONResponse({"error": "bad Content-Length"}, status_code=400)
            if int(cl) > MAX_BODY:
                return JSONResponse({"error": "body exceeds 4 MiB"}, status_code=413)
        return await call_next(request)       # chunked bodies: ChunkedBodyCap (raw ASGI, below)

    # ------------------------------------------------------------------ CORS
    @app.middleware("http")
    async def cors(request: Request, call_next):
        origin = request.headers.get("origin", "")
        if request.method == "OPTIONS":
            resp: Response = Response(status_code=204)
        else:
            resp = await call_next(request)
        if origin and ("*" in origins or origin in origins):
            resp.headers["Access-Control-Allow-Origin"] = origin
            resp.headers["Access-Control-Allow-Credentials"] = "true"
            resp.headers["Access-Control-Allow-Headers"] = \
                "Content-Type, Content-Length, Accept-Encoding, X-CSRF-Token, Authorization, accept, origin, Cache-Control, X-Requested-With"
            resp.headers["Access-Control-Allow-Methods"] = "POST, OPTIONS, GET, PUT, DELETE"
        return resp

    # ------------------------------------------------------------------ health / metrics
    @app.get("/health")
    @app.get("/api/v1/health")            # the path the reference's API docs use (docs/api.md:796)
    def health():
        # a stalled or failing serve loop is NOT healthy: probes (k8s,
        # the load balancer's URL checks) must see it and replace the process
        ok, reason = G.health() if hasattr(G, "health") else (True, "")
        if not ok:
            return JSONResponse({"status": "unhealthy", "reason": reason, "version": VERSION,
                                 "time": format_time(time.time_ns())}, status_code=503)
        return {"status": "ok", "version": VERSION, "time": format_time(time.time_ns())}

    @app.get("/metrics")
    def metrics():
        render = getattr(G, "metrics_exposition", None) or G.metrics.render
        return Response(render(), media_type=CONTENT_TYPE_LATEST)

    # ------------------------------------------------------------------ messages
    # `cli api-gateway` (role "ingress"): replies also carry the reference
    # api-gateway's fields (cmd/api-gateway/main.go:113, 177) so clients of
    # either reference binary read them
    gateway_compat = getattr(G, "role", "") == "ingress"

    def _bind_message(body: Any) -> Message:
        m = Message.from_dict(body)
        if not m.id:
            m.id = str(uuid.uuid4())
        now = time.time_ns()
        m.created_at = m.updated_at = now
        return m

    async def _enqueue(m: Message) -> Optional[JSONResponse]:
        if G.cfg.queue.enable_metrics:
            a = G.preprocessor.analyze_message_content(m.content)
            m.metadata["analysis"] = G.preprocessor.analysis_json(a["word_count"], a["sentiment"], a["is_question"])
        try:
            # await the micro-batch (GPU preprocess + queue push) without
            # blocking the event loop: concurrent requests share one batch
            err = await asyncio.wait_for(asyncio.wrap_future(G.submit_future(m)), timeout=30.0)
        except Exception as e:
            return _err(500, f"Failed to queue message: {e}")
        if err is not None:
            return _err(500, "Failed to queue message")
        return None

    @app.post("/api/v1/messages")
    async def submit_message(request: Request):
        try:
            m = _bind_message(await _json(request))
        except (ValueError, PriorityParseError, TypeError) as e:
            return _err(400, f"Invalid message format: {e}")
        bad = await _enqueue(m)
        if bad is not None:
            return bad
        if m.conversation_id:
            G.state.get_conversation(m.conversation_id, m.user_id)
            try:
                G.state.add_message(m.conversation_id, m)
            except ConversationNotFound:
                pass
        out = {"message_id": m.id, "priority": int(m.priority), "queue_time": format_time(time.time_ns()),
               "estimated_wait": G.estimated_wait_ns(m)}
        if gateway_compat:
            out.update(message="Message accepted", id=m.id)
        return JSONResponse(out, status_code=202)

    @app.get("/api/v1/messages/{mid}")
    def get_message(mid: str):
        # this process's store, else the GPU rank that popped it (multi-GPU front door)
        d = G.find_message(mid)
        if d is None:
            return _err(404, "Message not found")
        return d

    @app.get("/api/v1/messages")
    def list_messages(user_id: str = "", conversation_id: str = "", status: str = "", limit: int = 10,
                      offset: int = 0):
        total, msgs = G.query_messages(user_id, conversation_id, status, max(0, limit), max(0, offset))
        return {"messages": msgs, "total": total, "limit": limit, "offset": offset}

    @app.put("/api/v1/messages/{mid}/status")
    async def update_message_status(mid: str, request: Request):
        try:
            body = await _json(request)
            status = str(body["status"])
        except Exception as e:
            return _err(400, f"Invalid request format: {e}")
        if status not in MessageStatus.ALL:
            return _err(400, f"invalid status {status!r}")
        m = G.messages.get(mid)
        if m is None:
            if G.peers is not None and G.peers.first("set_status", [mid, status]):
                return {"status": "updated", "message_id": mid}
            return _err(404, "Message not found")
        m.status = status
        m.updated_at = time.time_ns()
        return {"status": "updated", "message_id": mid}

    @app.delete("/api/v1/messages/{mid}")
    def delete_message(mid: str):
        # queued: removed from its queue; running on a GPU: aborted there
        # (its batch slot freed), on whichever rank popped it
        m = G.messages.get(mid)
        if m is None:
            res = G.peers.first("remove", [mid]) if G.peers is not None else None
            if isinstance(res, dict):
                return {"status": "deleted", "message_id": mid, "dequeued": bool(res.get("dequeued")),
                        "cancelled": bool(res.get("cancelled"))}
            return _err(404, "Message not found")
        # everywhere else in its lifecycle (inbox, preprocess, retry backoff,
        # held for its KV, a GPU slot here or on another rank): cancelled
        # through the gateway's request table -- after this 200 it is never
        # dispatched or completed again
        removed = m.queue_name and G.standard.has_queue(m.queue_name) and G.standard.remove_message(m.queue_name, m)
        res = "" if removed else (G.cancel_inflight(m) if hasattr(G, "cancel_inflight") else "")
        G.messages.remove(mid)
        return {"status": "deleted", "message_id": mid, "dequeued": bool(removed) or res == "dequeued",
                "cancelled": res in ("cancelled", "forwarded", "pending")}

    # ------------------------------------------------------------------ conversations
    @app.post("/api/v1/conversations")
    async def create_conversation(request: Request):
        try:
            body = await _json(request)
            user_id = body.get("user_id")
            if not user_id:
                raise ValueError("Key: 'user_id' Error:Field validation for 'user_id' failed on the 'required' tag")
            md = body.get("metadata") or {}
            if not isinstance(md, dict):
                raise ValueError("metadata must be an object")
        except Exception as e:
            return _err(400, f"Invalid request format: {e}")
        conv = G.state.create_conversation(str(user_id), md)
        return JSONResponse({"conversation_id": conv.id, "user_id": conv.user_id,
                             "created_at": format_time(conv.created_at), "state": conv.state}, status_code=201)

    @app.get("/api/v1/conversations")
    def list_conversations(user_id: str = "", state: str = "", limit: int = 20, offset: int = 0):
        if user_id:
            convs = G.state.get_user_conversations(user_id)
        else:
            convs = G.state.all_conversations()
        if state:
            convs = [c for c in convs if c.state == state]
        return {"conversations": [c.to_dict(False) for c in convs[offset:offset + limit]], "total": len(convs)}

    @app.get("/api/v1/conversations/{cid}")
    def get_conversation(cid: str):
        conv = G.state.find_conversation(cid)
        if conv is None:
            return _err(404, "Conversation not found")
        return conv.to_dict()

    @app.put("/api/v1/conversations/{cid}")
    async def update_conversation(cid: str, request: Request):
        try:
            body = await _json(request)
        except Exception as e:
            return _err(400, f"Invalid request format: {e}")
        conv = G.state.find_conversation(cid)
        if conv is None:
            return _err(404, "Conversation not found")
        if "metadata" in body:
            G.state.update_conversation_metadata(cid, body.get("metadata") or {})
        if "state" in body:
            G.state.update_conversation_state(cid, str(body["state"]))
        if "title" in body:
            conv.title = str(body["title"])
        return conv.to_dict(False)

    @app.post("/api/v1/conversations/{cid}/messages")
    async def add_message_to_conversation(cid: str, request: Request):
        try:
            m = _bind_message(await _json(request))
        except (ValueError, PriorityParseError, TypeError) as e:
            return _err(400, f"Invalid message format: {e}")
        m.conversation_id = cid
        # route sticky to the GPU holding this conversation's KV (residency hint)
        home = G.state.home_gpu(cid)
        if home >= 0:
            m.metadata.setdefault("home_gpu", home)
        try:
            G.state.add_message(cid, m)
        except ConversationNotFound:
            return _err(500, "Failed to add message to conversation")
        bad = await _enqueue(m)
        if bad is not None:
            return bad
        out = {"message_id": m.id, "conversation_id": cid, "priority": int(m.priority),
               "queue_time": format_time(time.time_ns()), "estimated_wait": G.estimated_wait_ns(m)}
        if gateway_compat:
            out["message"] = "Message added successfully"
        return JSONResponse(out, status_code=202)

    @app.put("/api/v1/conversations/{cid}/state")
    async def update_conversation_state(cid: str, request: Request):
        try:
            body = await _json(request)
            state = body.get("state")
            if not state:
                raise ValueError("Key: 'state' Error:Field validation for 'state' failed on the 'required' tag")
        except Exception as e:
            return _err(400, f"Invalid request format: {e}")
        try:
            G.state.update_conversation_state(cid, str(state))
        except ConversationNotFound:
            return _err(500, "Failed to update conversation state")
        if isinstance(body.get("metadata"), dict):
            G.state.update_conversation_metadata(cid, body["metadata"])
        return {"status": "updated"}

    @app.get("/api/v1/users/{user_id}/conversations")
    def list_user_conversations(user_id: str):
        return {"conversations": [c.to_dict() for c in G.state.get_user_conversations(user_id)]}

    # ------------------------------------------------------------------ queues
    @app.get("/api/v1/queues/stats")
    def queue_stats():
        return G.queue_stats()

    @app.get("/api/v1/queues/status")
    def queue_status():
        tiers = []
        for t, name in enumerate(G.gateway.tiers):
            st = G.standard.get_queue_stats(name)
            tiers.append({"name": name, "priority": G.gateway.tier_prio[t], "pending": st.pending_count,
                          "processing": st.processing_count, "completed": st.completed_count,
                          "failed": st.failed_count,
                          "avg_wait_ms": (st.total_wait_time / max(1, st.completed_count + st.processing_count
                                                                   + st.failed_count)) / 1e6})
        lat = G.gateway.rec.summary()
        out = {"queues": tiers, "total_pending": G.standard.total_pending(), "latency": lat,
               "dead_letter": G.factory.dead_letter_queue.size(), "delayed": G.factory.delayed_queue.size()}
        if G.peers is not None:
            out["job"] = G.job_stats()            # every GPU rank (the fields above are rank 0's)
        return out

    @app.get("/api/v1/metrics")
    def metrics_json():
        """JSON metrics summary (doc-only in the reference, docs/api.md:647-698:
        requests/s, average response time, error rate, queue lengths)."""
        c = G.gateway.counters
        done = G.gateway.rec_done.summary()
        failed = sum(G.standard.get_queue_stats(n).failed_count for n in G.gateway.tiers)
        completed = sum(G.standard.get_queue_stats(n).completed_count for n in G.gateway.tiers)
        return {"requests_total": G.messages_seen() + c["submitted"], "dispatched_total": c["dispatched"],
                "completed_total": completed, "failed_total": failed,
                "requests_per_second": round(G._dispatch_rate(), 2),
                "error_rate": round(failed / max(1, completed + failed), 6),
                "latency": {"dispatch": G.gateway.rec.summary(), "end_to_end": done},
                "queue_lengths": {n: G.standard.size(n) for n in G.gateway.tiers},
                "dead_letter": G.factory.dead_letter_queue.size(), "delayed": G.factory.delayed_queue.size(),
                "gpu": {"healthy": G.gateway.healthy, "reason": G.gateway.health_reason,
                        "inflight_slots": G.engine.inflight() if G.engine is not None else 0},
                **({"job": G.job_stats()} if G.peers is not None else {})}

    # ------------------------------------------------------------------ resources
    @app.post("/api/v1/resources")
    async def register_resource(request: Request):
        try:
            r = Resource.from_dict(await _json(request))
        except Exception as e:
            return _err(400, f"Invalid resource format: {e}")
        try:
            G.resources.register_resource(r)
        except ResourceError as e:
            return _err(500, f"Failed to register resource: {e}")
        return JSONResponse({"resource_id": r.id, "status": "registered"}, status_code=201)

    @app.get("/api/v1/resources")
    def list_resources():
        return {"resources": [r.to_dict() for r in G.resources.get_all_resources()]}

    @app.get("/api/v1/resources/stats")
    def resource_stats():
        return G.resources.get_resource_stats()

    # ------------------------------------------------------------------ endpoints
    @app.post("/api/v1/endpoints")
    async def register_endpoint(request: Request):
        try:
            ep = Endpoint.from_dict(await _json(request))
        except Exception as e:
            return _err(400, f"Invalid endpoint format: {e}")
        try:
            G.lb.add_endpoint(ep)
        except LoadBalancerError as e:
            return _err(500, f"Failed to register endpoint: {e}")
        return JSONResponse({"endpoint_id": ep.id, "status": "registered"}, status_code=201)

    @app.delete("/api/v1/endpoints/{eid}")
    def remove_endpoint(eid: str):
        try:
            G.lb.remove_endpoint(eid)
        except LoadBalancerError:
            return _err(404, "endpoint not found")
        return {"endpoint_id": eid, "status": "removed"}

    @app.put("/api/v1/endpoints/{eid}/status")
    async def update_endpoint_status(eid: str, request: Request):
        try:
            status = str((await _json(request))["status"])
            G.set_endpoint_status(eid, status)
        except LoadBalancerError:
            return _err(404, "endpoint not found")
        except Exception as e:
            return _err(400, f"Invalid request format: {e}")
        return {"endpoint_id": eid, "status": status}

    @app.get("/api/v1/endpoints")
    def list_endpoints():
        return {"endpoints": [e.to_dict() for e in G.lb.get_all_endpoints()]}

    @app.get("/api/v1/endpoints/stats")
    def endpoint_stats():
        return G.lb.get_endpoint_stats()

    # ------------------------------------------------------------------ admin
    async def _sync_preprocessor() -> Optional[JSONResponse]:
        """Multi-GPU front door: every rank preprocesses the requests it
        pops, so an admin change on this rank is copied to all of them
        before the reply (a 500 names ranks that did not confirm; the next
        change, which carries the whole state, repairs them)."""
        sync = getattr(G, "sync_preprocessor", None)
        missing = await asyncio.get_running_loop().run_in_executor(None, sync) if sync is not None else None
        if missing:
            return _err(500, f"preprocessor change not confirmed by GPU ranks {missing}")
        return None

    @app.post("/api/v1/admin/preprocessor/rules")
    async def add_priority_rule(request: Request):
        try:
            body = await _json(request)
            pattern = str(body.get("pattern") or body.get("rule") or "")
            if not pattern:
                raise ValueError("pattern is required")
            prio = parse_priority(body.get("priority"), 0)
            if prio <= 0:
                raise ValueError("priority is required")
        except Exception as e:
            return _err(400, f"Invalid rule format: {e}")
        try:
            G.preprocessor.add_keyword_pattern(prio, pattern)
        except Exception as e:
            return _err(400, f"Invalid pattern: {e}")
        bad = await _sync_preprocessor()
        if bad is not None:
            return bad
        return JSONResponse({"status": "rule added"}, status_code=201)

    @app.get("/api/v1/admin/preprocessor/rules")
    def list_priority_rules():
        rules = [{"priority": p, "priority_name": priority_name(p), "pattern": s}
                 for p, pats in G.preprocessor.all_patterns().items() for s in pats]
        return {"rules": rules}

    @app.delete("/api/v1/admin/preprocessor/rules")
    async def remove_priority_rule(request: Request):
        try:
            body = await _json(request)
            ok = G.preprocessor.remove_keyword_pattern(parse_priority(body.get("priority")), str(body["pattern"]))
        except Exception as e:
            return _err(400, f"Invalid rule format: {e}")
        if not ok:
            return _err(404, "rule not found")
        bad = await _sync_preprocessor()
        return bad if bad is not None else {"status": "rule removed"}

    @app.post("/api/v1/admin/preprocessor/user-priorities")
    async def set_user_priority(request: Request):
        try:
            body = await _json(request)
            user_id = body.get("user_id")
            pstr = body.get("priority")
            if not user_id or pstr in (None, ""):
                raise ValueError("user_id and priority are required")
        except Exception as e:
            return _err(400, f"Invalid request format: {e}")
        p = level_priority_from_name(pstr) if isinstance(pstr, str) else None
        if p is None:
            try:
                p = parse_priority(pstr)
            except PriorityParseError:
                p = 3
        if p not in (1, 2, 3, 4):
            p = 3
        G.preprocessor.set_user_priority(str(user_id), p)
        bad = await _sync_preprocessor()
        return bad if bad is not None else {"status": "user priority set"}

    @app.delete("/api/v1/admin/queues/{queue_type}/{mid}")
    def remove_message(queue_type: str, mid: str):
        if queue_type not in ("standard", "delayed", "dead_letter", "priority"):
            return _err(400, "Invalid queue type")
        # (multi-GPU: on whichever rank holds the message)
        if queue_type == "dead_letter":
            if G.dead_letters("remove", mid) is not True:
                return _err(404, "Message not found")
            return {"status": "removed", "message_id": mid}
        if not G.dequeue(queue_type, mid):
            return _err(404, "Message not found")
        return {"status": "removed", "message_id": mid}

    @app.post("/api/v1/admin/dead-letter/requeue/{mid}")
    def requeue_dead_letter(mid: str):
        res = G.dead_letters("requeue", mid)
        if isinstance(res, dict):
            return _err(500, str(res.get("error")))
        if res is not True:
            return _err(404, f"message {mid} not in dead letter queue")
        return {"status": "requeued", "message_id": mid}

    @app.post("/api/v1/admin/dead-letter/requeue-all")
    def requeue_all_dead_letter():
        return {"status": "requeued", "count": G.dead_letters("requeue_all")}

    @app.post("/api/v1/admin/stats/reset")
    def reset_stats():
        """Open a new latency window (arrival->dispatch and ->completion
        histograms); counters are cumulative and stay."""
        gw_app.reset_latency_all()                  # (every GPU rank behind the front door)
        return {"status": "reset"}

    @app.get("/api/v1/admin/dead-letter")
    def list_dead_letter(limit: int = 1000):
        """The oldest ``limit`` dead letters of each GPU rank (``rank`` field)."""
        return {"items": G.dead_letters("list", str(max(1, min(int(limit), 5000))))}

    @app.post("/api/v1/admin/faults")
    async def inject_fault(request: Request):
        """Failure drills (SURVEY.md §5 failure injection): inject faults
        into this process's GPU backend -- ``{"fail_launch": n}`` (the next
        n launches raise a HIP error), ``{"slow_ms": x}`` (every launch
        stalls x ms; longer than ``server.stall_fatal_after`` drives the
        stall watchdog to a fatal exit), ``{"drop_heartbeat": true}``; 0 /
        false clears one.  403 unless ``server.fault_injection``."""
        if not G.cfg.server.fault_injection:
            return _err(403, "fault injection is disabled (server.fault_injection)")
        eng = getattr(G, "engine", None)
        if eng is None or not hasattr(eng, "inject"):
            return _err(409, "no GPU backend in this process")
        try:
            body = await _json(request)
            eng.inject(**dict(body))
        except (ValueError, TypeError) as e:
            return _err(400, f"bad fault: {e}")
        return {"status": "injected", "faults": dict(eng.fault)}

    @app.get("/api/v1/config")
    def get_config():
        return redact_config(dataclasses.asdict(G.cfg))

    app.add_middleware(ChunkedBodyCap)
    return app


class ChunkedBodyCap:
    """Raw-ASGI cap for bodies without a Content-Length (chunked transfer
    encoding): the stream is read incrementally and refused with 413 as soon
    as the running total passes ``MAX_BODY`` -- at most 4 MiB plus one chunk
    is ever buffered (``await request.body()`` buffered the whole
    stream first).  An accepted body is replayed to the app unchanged."""

    def __init__(self, app):
        self.app = app

    async def __call__(self, scope, receive, send):
        if scope.get("type") != "http":
            return await self.app(scope, receive, send)
        hdrs = {k.lower(): v for k, v in scope.get("headers") or []}
        if b"content-length" in hdrs or hdrs.get(b"transfer-encoding", b"").lower() != b"chunked":
            return await self.app(scope, receive, send)
        chunks, total = [], 0
        while True:
            msg = await receive()
            if msg["type"] == "http.disconnect":
                return
            body = msg.get("body", b"")
            total += len(body)
            if total > MAX_BODY:
                resp = JSONResponse({"error": "body exceeds 4 MiB"}, status_code=413)
                return await resp(scope, receive, send)
            chunks.append(body)
            if not msg.get("more_body", False):
                break
        replay = [{"type": "http.request", "body": b"".join(chunks), "more_body": False}]

        async def again():
            return replay.pop() if replay else await receive()
        return await self.app(scope, again, send)
