"""LoadBalancer (component C11), GPU-aware.

Reference `internal/loadbalancer/load_balancer.go`:
  * strategies round_robin / least_connections / weighted_random /
    adaptive_load; unknown names fall back to round robin (`:272-275`);
  * endpoints grouped by ``type``; a message picks the group from
    ``metadata["model_type"]`` (default ``"llm"``, `:654-669`);
  * only healthy/degraded endpoints are eligible (`:672-682`);
  * ``get_endpoint`` honours session affinity, selects, ``connections++``,
    saves the session (`:234-294`); ``release_endpoint`` decrements and keeps
    EWMA(alpha=0.1) response time and error rate (`:297-330`);
  * adaptive score = 0.4*load + 0.4*min(rt_s, 10) + 0.2*(10*err), best
    ascending, 10 % chance of the runner-up (`:458-498`).

Fixes: the lock is never leaked on error paths (D7); affinity and session
timeout come from config (D8); health checks are real -- a probe per
endpoint, ``max_failures`` consecutive failures -> unhealthy,
``healthy_threshold`` successes -> healthy, unhealthy -> degraded on the
first success (D9); the RR cursor walks the FULL list and skips ineligible
entries, so a health change does not shift everybody's turn.

MI355X additions: an endpoint may be bound to a GPU backend's load page
(N9) and telemetry (N8).  Then ``connections`` = live in-flight slots read
zero-copy from the page (+ dispatched-but-not-yet-admitted), ``max_connections``
= batch slots, and the strategies add HBM occupancy: least-connections breaks
ties on free HBM, weighted-random scales weights by free-slot and free-HBM
fractions, adaptive adds an HBM-pressure term.
"""
from __future__ import annotations

import random
import threading
import time
import urllib.request
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..utils.logging import get_logger


class Strategy:
    ROUND_ROBIN = "round_robin"
    LEAST_CONNECTIONS = "least_connections"
    WEIGHTED_RANDOM = "weighted_random"
    ADAPTIVE_LOAD = "adaptive_load"
    ALL = ("round_robin", "least_connections", "weighted_random", "adaptive_load")


class EndpointStatus:
    HEALTHY = "healthy"
    DEGRADED = "degraded"
    UNHEALTHY = "unhealthy"


class LoadBalancerError(Exception):
    pass


@dataclass
class Endpoint:
    """`load_balancer.go:35-49` plus GPU binding."""
    id: str
    url: str = ""
    name: str = ""
    type: str = "llm"
    capabilities: List[str] = field(default_factory=list)
    weight: int = 1
    status: str = ""
    connections: int = 0
    max_connections: int = 0
    response_time: int = 0         # ns (EWMA)
    error_rate: float = 0.0        # EWMA
    last_check: int = 0
    metadata: Dict[str, Any] = field(default_factory=dict)
    # ---- MI355X binding (not part of the reference JSON)
    gpu_index: int = -1
    page: Any = None               # backend.slot_page.SlotPage
    pending: int = 0               # dispatched, not yet visible on the page
    consecutive_failures: int = 0
    consecutive_successes: int = 0
    probe: Optional[Callable[["Endpoint"], bool]] = None

    def live_connections(self) -> int:
        if self.page is not None:
            return self.page.active() + self.pending
        return self.connections

    def capacity(self) -> int:
        if self.page is not None and self.max_connections <= 0:
            try:
                r = self.page.read()
                return r["active"] + r["free"]
            except Exception:
                return 0
        return self.max_connections

    def hbm_free_frac(self) -> Optional[float]:
        if self.page is None:
            return None
        w = self.page.words
        tot = int(w[6])
        if tot <= 0:
            return None
        return max(0.0, 1.0 - int(w[5]) / tot)

    def to_dict(self) -> Dict[str, Any]:
        from ..models.message import format_time
        d = {"id": self.id, "url": self.url, "name": self.name, "type": self.type,
             "capabilities": list(self.capabilities), "weight": self.weight, "status": self.status,
             "connections": self.live_connections(), "max_connections": self.max_connections,
             "response_time": self.response_time, "error_rate": self.error_rate,
             "last_check": format_time(self.last_check), "metadata": self.metadata}
        if self.gpu_index >= 0:
            d["gpu_index"] = self.gpu_index
            if self.page is not None:
                d["load"] = self.page.read()
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Endpoint":
        if not isinstance(d, dict) or not d.get("id"):
            raise ValueError("endpoint id is required")
        from ..utils.duration import parse_duration_ns
        rt = d.get("response_time", 0)
        return cls(id=str(d["id"]), url=str(d.get("url", "")), name=str(d.get("name", "")),
                   type=str(d.get("type") or "llm"), capabilities=list(d.get("capabilities") or []),
                   weight=int(d.get("weight") or 0), status=str(d.get("status") or ""),
                   connections=int(d.get("connections") or 0),
                   max_connections=int(d.get("max_connections") or 0),
                   response_time=parse_duration_ns(rt) if rt else 0,
                   error_rate=float(d.get("error_rate") or 0.0),
                   metadata=dict(d.get("metadata") or {}),
                   gpu_index=int(d.get("gpu_index", -1)))


@dataclass
class SessionInfo:
    session_id: str
    endpoint_id: str
    created_at: float
    last_used: float


def http_probe(timeout_s: float = 2.0) -> Callable[[Endpoint], bool]:
    """GET <url>/health -> 2xx."""
    def probe(ep: Endpoint) -> bool:
        if not ep.url:
            return True
        try:
            with urllib.request.urlopen(ep.url.rstrip("/") + "/health", timeout=timeout_s) as r:
                return 200 <= r.status < 300
        except Exception:
            return False
    return probe


def page_probe(stale_after_s: float = 10.0) -> Callable[[Endpoint], bool]:
    """GPU backend is healthy if its page says so and its step counter moved
    (or it is idle with free slots)."""
    state: Dict[str, tuple] = {}

    def probe(ep: Endpoint) -> bool:
        if ep.page is None:
            return True
        r = ep.page.read()
        if not r["healthy"]:
            return False
        now = time.monotonic()
        prev = state.get(ep.id)
        if prev is None or prev[0] != r["seq"] or r["active"] == 0:
            state[ep.id] = (r["seq"], now)
            return True
        return now - prev[1] < stale_after_s
    return probe


class LoadBalancer:
    def __init__(self, cfg=None, logger=None, seed: Optional[int] = None,
                 default_probe: Optional[Callable[[Endpoint], bool]] = None):
        from ..utils.config import LoadBalancerConfig
        cfg = cfg or LoadBalancerConfig()
        self.cfg = cfg
        self.strategy = cfg.algorithm if cfg.algorithm in Strategy.ALL else Strategy.ROUND_ROBIN
        self.enable_session_affinity = cfg.enable_session_affinity
        self.session_timeout_s = cfg.session_timeout / 1e9
        self.unhealthy_threshold = max(1, cfg.max_failures)
        self.healthy_threshold = max(1, cfg.healthy_threshold)
        self.logger = logger or get_logger("load_balancer")
        self._lock = threading.RLock()
        self._groups: Dict[str, List[Endpoint]] = {}
        self._sessions: Dict[str, SessionInfo] = {}
        self._cursor: Dict[str, int] = {}
        self._rand = random.Random(seed)
        self._default_probe = default_probe
        # URL endpoints without a probe of their own: a real HTTP health check (D9)
        self._http_probe = http_probe() if getattr(cfg, "http_health_probe", True) else None
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        if cfg.health_check_interval > 0:
            self._spawn(self._health_loop, cfg.health_check_interval / 1e9)
        if self.enable_session_affinity and cfg.session_timeout > 0:
            self._spawn(self._session_loop, max(cfg.session_timeout / 2e9, 0.01))

    def _spawn(self, fn, interval_s: float) -> None:
        t = threading.Thread(target=fn, args=(interval_s,), daemon=True)
        t.start()
        self._threads.append(t)

    def stop(self) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=2)

    # ------------------------------------------------------------------ registry
    def add_endpoint(self, ep: Endpoint) -> None:
        with self._lock:
            for g in self._groups.values():
                if any(e.id == ep.id for e in g):
                    raise LoadBalancerError("endpoint with this ID already exists")
            if not ep.status:
                ep.status = EndpointStatus.HEALTHY
            ep.last_check = time.time_ns()
            self._groups.setdefault(ep.type or "llm", []).append(ep)
        self.logger.info("Added endpoint", id=ep.id, type=ep.type, gpu=ep.gpu_index)

    def remove_endpoint(self, endpoint_id: str) -> None:
        with self._lock:
            for t, g in list(self._groups.items()):
                for i, e in enumerate(g):
                    if e.id == endpoint_id:
                        del g[i]
                        if not g:
                            del self._groups[t]
                        for sid in [s for s, info in self._sessions.items() if info.endpoint_id == endpoint_id]:
                            del self._sessions[sid]
                        return
        raise LoadBalancerError("endpoint not found")

    def update_endpoint_status(self, endpoint_id: str, status: str) -> None:
        with self._lock:
            ep = self._find(endpoint_id)
            if ep is None:
                raise LoadBalancerError("endpoint not found")
            ep.status = status
            ep.consecutive_failures = ep.consecutive_successes = 0

    def _find(self, endpoint_id: str) -> Optional[Endpoint]:
        for g in self._groups.values():
            for e in g:
                if e.id == endpoint_id:
                    return e
        return None

    # ------------------------------------------------------------------ selection
    @staticmethod
    def endpoint_type(msg) -> str:
        if msg is not None and getattr(msg, "metadata", None):
            mt = msg.metadata.get("model_type")
            if isinstance(mt, str) and mt:
                return mt
        return "llm"

    @staticmethod
    def _eligible(ep: Endpoint) -> bool:
        return ep.status in (EndpointStatus.HEALTHY, EndpointStatus.DEGRADED)

    def get_endpoint(self, msg=None, session_id: str = "") -> Endpoint:
        if self.enable_session_affinity and session_id:
            ep = self._session_endpoint(session_id)
            if ep is not None:
                with self._lock:
                    self._acquire(ep)
                return ep
        etype = self.endpoint_type(msg)
        with self._lock:
            group = self._groups.get(etype)
            if not group:
                raise LoadBalancerError("no endpoints available for the requested type")
            healthy = [e for e in group if self._eligible(e)]
            if not healthy:
                raise LoadBalancerError("no healthy endpoints available")
            s = self.strategy
            if s == Strategy.LEAST_CONNECTIONS:
                ep = self._least_connections(healthy)
            elif s == Strategy.WEIGHTED_RANDOM:
                ep = self._weighted_random(healthy)
            elif s == Strategy.ADAPTIVE_LOAD:
                ep = self._adaptive(healthy)
            else:
                ep = self._round_robin(etype, group)
            if ep is None:
                raise LoadBalancerError("failed to select an endpoint")
            self._acquire(ep)
        if self.enable_session_affinity and session_id:
            self._save_session(session_id, ep.id)
        return ep

    def _acquire(self, ep: Endpoint) -> None:
        if ep.page is not None:
            ep.pending += 1
        else:
            ep.connections += 1

    def _round_robin(self, etype: str, group: List[Endpoint]) -> Optional[Endpoint]:
        n = len(group)
        start = self._cursor.get(etype, 0)
        for k in range(n):
            i = (start + k) % n
            if self._eligible(group[i]):
                self._cursor[etype] = (i + 1) % n
                return group[i]
        return None

    def _least_connections(self, eps: List[Endpoint]) -> Endpoint:
        def key(e: Endpoint):
            cap = e.capacity()
            load = e.live_connections()
            util = load / cap if cap > 0 else float(load)
            hf = e.hbm_free_frac()
            # GPU endpoints compare utilisation; plain ones raw connections (reference)
            primary = util if e.page is not None else load
            return (primary, -(hf if hf is not None else 0.0))
        best, best_k = None, None
        for e in eps:                 # first minimum wins, as in the reference
            k = key(e)
            if best_k is None or k < best_k:
                best, best_k = e, k
        return best

    def _weighted_random(self, eps: List[Endpoint]) -> Endpoint:
        ws = []
        for e in eps:
            w = float(e.weight if e.weight > 0 else 1)
            if e.page is not None:
                cap = e.capacity()
                free = max(0, cap - e.live_connections())
                hf = e.hbm_free_frac()
                w *= (free / cap if cap > 0 else 1.0) * (hf if hf is not None else 1.0)
            ws.append(w)
        tot = sum(ws)
        if tot <= 0:
            return eps[0]
        r = self._rand.random() * tot
        acc = 0.0
        for e, w in zip(eps, ws):
            acc += w
            if r < acc:
                return e
        return eps[-1]

    def _adaptive(self, eps: List[Endpoint]) -> Endpoint:
        scored = []
        for e in eps:
            cap = e.capacity()
            conn = e.live_connections()
            load = conn / cap if cap > 0 else conn / 100.0
            ts = min(e.response_time / 1e9, 10.0)
            score = load * 0.4 + ts * 0.4 + e.error_rate * 10 * 0.2
            hf = e.hbm_free_frac()
            if hf is not None:
                score += 0.2 * (1.0 - hf)
            scored.append((score, e))
        scored.sort(key=lambda x: x[0])   # stable: ties keep list order
        if len(scored) > 1 and self._rand.random() < 0.1:
            return scored[1][1]
        return scored[0][1]

    def release_endpoint(self, endpoint_id: str, response_time_ns: int = 0, is_error: bool = False,
                         admitted: bool = True) -> None:
        with self._lock:
            ep = self._find(endpoint_id)
            if ep is None:
                return
            if ep.page is not None:
                if not admitted and ep.pending > 0:
                    ep.pending -= 1
            elif ep.connections > 0:
                ep.connections -= 1
            if response_time_ns > 0:
                ep.response_time = response_time_ns if ep.response_time == 0 else \
                    (ep.response_time * 9 + response_time_ns) // 10
            ep.error_rate = (ep.error_rate * 9 + 1) / 10 if is_error else ep.error_rate * 0.9

    def note_dispatch(self, endpoint_id: str, n: int = 1) -> None:
        """``n`` requests were placed on this endpoint by the multi-GPU
        planner (the batch equivalent of ``n`` GetEndpoint picks): count them
        as connections until their completions ``release_endpoint``."""
        with self._lock:
            ep = self._find(endpoint_id)
            if ep is None:
                return
            if ep.page is not None:
                ep.pending += n
            else:
                ep.connections += n

    def mark_admitted(self, endpoint_id: str, n: int = 1) -> None:
        """GPU endpoints: ``n`` dispatched requests are now counted by the page."""
        with self._lock:
            ep = self._find(endpoint_id)
            if ep is not None:
                ep.pending = max(0, ep.pending - n)

    # ------------------------------------------------------------------ sessions
    def _session_endpoint(self, session_id: str) -> Optional[Endpoint]:
        with self._lock:
            s = self._sessions.get(session_id)
            if s is None:
                return None
            if self.session_timeout_s > 0 and time.monotonic() - s.last_used > self.session_timeout_s:
                del self._sessions[session_id]
                return None
            ep = self._find(s.endpoint_id)
            if ep is None or not self._eligible(ep):
                del self._sessions[session_id]
                return None
            s.last_used = time.monotonic()
            return ep

    def _save_session(self, session_id: str, endpoint_id: str) -> None:
        with self._lock:
            now = time.monotonic()
            s = self._sessions.get(session_id)
            if s is None:
                self._sessions[session_id] = SessionInfo(session_id, endpoint_id, now, now)
            else:
                s.endpoint_id = endpoint_id
                s.last_used = now

    def session_endpoint_id(self, session_id: str) -> Optional[str]:
        with self._lock:
            s = self._sessions.get(session_id)
            return s.endpoint_id if s else None

    def bind_session(self, session_id: str, endpoint_id: str) -> None:
        self._save_session(session_id, endpoint_id)

    def get_session_count(self) -> int:
        with self._lock:
            return len(self._sessions)

    def clear_sessions(self) -> None:
        with self._lock:
            self._sessions = {}

    def cleanup_expired_sessions(self) -> int:
        if self.session_timeout_s <= 0:
            return 0
        now = time.monotonic()
        with self._lock:
            dead = [k for k, s in self._sessions.items() if now - s.last_used > self.session_timeout_s]
            for k in dead:
                del self._sessions[k]
        return len(dead)

    def _session_loop(self, interval_s: float) -> None:
        while not self._stop.wait(interval_s):
            self.cleanup_expired_sessions()

    # ------------------------------------------------------------------ health
    def check_endpoint_health(self, ep: Endpoint) -> bool:
        probe = ep.probe or self._default_probe or (
            page_probe() if ep.page is not None else (self._http_probe if ep.url else None))
        ok = True if probe is None else bool(probe(ep))
        with self._lock:
            ep.last_check = time.time_ns()
            if ok:
                ep.consecutive_failures = 0
                ep.consecutive_successes += 1
                if ep.status == EndpointStatus.UNHEALTHY:
                    ep.status = EndpointStatus.DEGRADED
                    ep.consecutive_successes = 1
                elif ep.status == EndpointStatus.DEGRADED and \
                        ep.consecutive_successes >= self.healthy_threshold:
                    ep.status = EndpointStatus.HEALTHY
            else:
                ep.consecutive_successes = 0
                ep.consecutive_failures += 1
                if ep.consecutive_failures >= self.unhealthy_threshold:
                    if ep.status != EndpointStatus.UNHEALTHY:
                        self.logger.warning("Endpoint unhealthy", id=ep.id)
                    ep.status = EndpointStatus.UNHEALTHY
                elif ep.status == EndpointStatus.HEALTHY:
                    ep.status = EndpointStatus.DEGRADED
        return ok

    def perform_health_checks(self) -> None:
        for ep in self.get_all_endpoints():
            try:
                self.check_endpoint_health(ep)
            except Exception as e:  # a broken probe is a failed probe
                self.logger.error("health probe raised", id=ep.id, error=str(e))

    def _health_loop(self, interval_s: float) -> None:
        while not self._stop.wait(interval_s):
            self.perform_health_checks()

    # ------------------------------------------------------------------ stats
    def get_endpoint_stats(self) -> Dict[str, Any]:
        with self._lock:
            st = {"total": 0, "healthy": 0, "degraded": 0, "unhealthy": 0}
            by_type, conns = {}, 0
            for t, g in self._groups.items():
                by_type[t] = len(g)
                st["total"] += len(g)
                for e in g:
                    if e.status in st:
                        st[e.status] += 1
                    conns += e.live_connections()
            return {"endpoints": st, "endpoints_by_type": by_type, "total_connections": conns,
                    "sessions": len(self._sessions)}

    def get_all_endpoints(self) -> List[Endpoint]:
        with self._lock:
            return [e for g in self._groups.values() for e in g]

    def get_endpoints_by_type(self, etype: str) -> List[Endpoint]:
        with self._lock:
            return list(self._groups.get(etype, []))

    def get_endpoint_by_id(self, endpoint_id: str) -> Endpoint:
        with self._lock:
            ep = self._find(endpoint_id)
        if ep is None:
            raise LoadBalancerError("endpoint not found")
        return ep
