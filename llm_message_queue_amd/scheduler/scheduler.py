"""Endpoint autoscaler (component C12).

Reference `internal/scheduler/scheduler.go`: a ticker reads queue depth and
adds/removes load-balancer endpoints:
  * dynamic (also the default for unknown names such as the shipped
    ``priority_weighted``): pending > scale_up && n < max -> add
    ``endpoint-<n+1>``; pending < scale_down && n > min -> remove the last
    (`:119-156`), then *recommend* an LB strategy (`:158-180`);
  * adaptive: business hours (Mon-Fri 09-17) target max-1 (max if above
    scale_up), else min+1 (min if below scale_down) (`:184-254`);
  * hybrid: dynamic + per-endpoint weight clamp(100ms/avgRT, 1, 10) -- only
    logged in the reference (`:257-296`), APPLIED here;
  * static: no-op.

MI355X mapping: an endpoint is a GPU backend.  On one node the GPUs are a
fixed pool, so "scale up" re-activates a parked GPU backend from
``EndpointPool`` (and "scale down" parks one, draining its slots) instead of
inventing ``http://llm-processor-<n>:8080`` URLs; without a pool the
reference's URL endpoints are generated.  Fixes D13 (missing level stats no
longer nil-deref) and the unguarded ``isRunning`` flag.
"""
from __future__ import annotations

import datetime as _dt
import threading
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..balancer.load_balancer import Endpoint, LoadBalancer
from ..utils.logging import get_logger


class Strategy:
    STATIC = "static"
    DYNAMIC = "dynamic"
    ADAPTIVE = "adaptive"
    HYBRID = "hybrid"


@dataclass
class SchedulerConfig:
    strategy: str = Strategy.DYNAMIC
    monitor_interval: int = 100_000_000
    scaling_thresholds: Dict[str, int] = field(default_factory=lambda: {
        "scale_up_queue_length": 100, "scale_down_queue_length": 10})
    resource_limits: Dict[str, int] = field(default_factory=lambda: {"min_endpoints": 1, "max_endpoints": 10})
    adaptive_parameters: Dict[str, float] = field(default_factory=dict)
    apply_weights: bool = True


class EndpointPool:
    """Parked GPU backends that can be (re)activated, most preferred first."""

    def __init__(self, endpoints: Optional[List[Endpoint]] = None):
        self._parked: List[Endpoint] = list(endpoints or [])
        self._lock = threading.Lock()

    def take(self) -> Optional[Endpoint]:
        with self._lock:
            return self._parked.pop(0) if self._parked else None

    def give(self, ep: Endpoint) -> None:
        with self._lock:
            self._parked.insert(0, ep)

    def size(self) -> int:
        with self._lock:
            return len(self._parked)


def _always_healthy(ep) -> bool:
    return True


def generate_endpoint_url(index: int) -> str:
    return f"http://llm-processor-{index}:8080"


class Scheduler:
    def __init__(self, cfg: SchedulerConfig, queue_stats: Callable[[], Dict[str, int]], lb: LoadBalancer,
                 pool: Optional[EndpointPool] = None, clock: Callable[[], _dt.datetime] = _dt.datetime.now,
                 logger=None):
        """``queue_stats()`` returns {queue name: pending count}."""
        self.cfg = cfg
        self.queue_stats = queue_stats
        self.lb = lb
        self.pool = pool
        self.clock = clock
        self.logger = logger or get_logger("scheduler")
        self._lock = threading.Lock()
        self._running = False
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.recommendation = ""
        self.events: List[dict] = []

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        with self._lock:
            if self._running:
                self.logger.info("Scheduler is already running")
                return
            self._running = True
            self._stop.clear()
        self._thread = threading.Thread(target=self._loop, name="scheduler", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=5)
        with self._lock:
            self._running = False

    def is_running(self) -> bool:
        with self._lock:
            return self._running

    def _loop(self) -> None:
        iv = max(self.cfg.monitor_interval, 1_000_000) / 1e9
        while not self._stop.wait(iv):
            try:
                self.schedule_resources()
            except Exception as e:   # keep ticking
                self.logger.error("scheduling failed", error=str(e))

    # ------------------------------------------------------------------ policy
    def schedule_resources(self) -> str:
        stats = self.queue_stats() or {}
        s = self.cfg.strategy
        if s == Strategy.STATIC:
            return "static"
        if s == Strategy.ADAPTIVE:
            return self.apply_adaptive(stats)
        if s == Strategy.HYBRID:
            return self.apply_hybrid(stats)
        return self.apply_dynamic(stats)

    def _limits(self):
        rl, th = self.cfg.resource_limits, self.cfg.scaling_thresholds
        return (rl.get("min_endpoints", 1), rl.get("max_endpoints", 10),
                th.get("scale_up_queue_length", 100), th.get("scale_down_queue_length", 10))

    def _add(self, n_now: int, prefix: str = "endpoint") -> Optional[Endpoint]:
        ep = self.pool.take() if self.pool is not None else None
        if ep is None:
            if self.pool is not None:
                return None           # every GPU already active
            i = n_now + 1
            ep = Endpoint(id=f"{prefix}-{i}", url=generate_endpoint_url(i), name=f"Endpoint {i}", type="llm",
                          weight=1, max_connections=100)
            # a placeholder replica (the reference's generated URL is never
            # called, scheduler.go:299-301): nothing to probe over HTTP
            ep.probe = _always_healthy
        self.lb.add_endpoint(ep)
        self.events.append({"action": "add", "endpoint": ep.id})
        return ep

    def _remove(self, ep: Endpoint) -> None:
        self.lb.remove_endpoint(ep.id)
        if self.pool is not None:
            ep.pending = 0
            self.pool.give(ep)
        self.events.append({"action": "remove", "endpoint": ep.id})

    def apply_dynamic(self, stats: Dict[str, int]) -> str:
        eps = self.lb.get_all_endpoints()
        n = len(eps)
        total = sum(int(v) for v in stats.values())
        mn, mx, up, down = self._limits()
        action = "none"
        if total > up and n < mx:
            if self._add(n):
                action = "scale_up"
        elif total < down and n > mn:
            self._remove(eps[-1])
            action = "scale_down"
        rt, hi = int(stats.get("realtime", 0)), int(stats.get("high", 0))
        if rt > hi * 2:
            self.recommendation = "least_connections"
        elif total > up:
            self.recommendation = "adaptive_load"
        else:
            self.recommendation = "weighted_random"
        return action

    def apply_adaptive(self, stats: Dict[str, int]) -> str:
        now = self.clock()
        business = 9 <= now.hour < 17 and now.weekday() < 5
        eps = self.lb.get_all_endpoints()
        n = len(eps)
        total = sum(int(v) for v in stats.values())
        mn, mx, up, down = self._limits()
        if business:
            target = mx if total > up else mx - 1
        else:
            target = mn if total < down else mn + 1
        if target > n:
            for i in range(n, target):
                if self._add(i, prefix="adaptive-endpoint") is None:
                    break
            return "scale_up"
        if target < n:
            for i in range(n - 1, target - 1, -1):
                self._remove(eps[i])
            return "scale_down"
        return "none"

    def apply_hybrid(self, stats: Dict[str, int]) -> str:
        action = self.apply_dynamic(stats)
        for ep in self.lb.get_all_endpoints():
            if ep.response_time > 0:
                w = int(100_000_000 / ep.response_time)
                w = max(1, min(10, w))
                if self.cfg.apply_weights:
                    ep.weight = w
        return action
