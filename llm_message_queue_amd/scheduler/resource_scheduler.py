"""ResourceScheduler (component C13): capacity-aware allocation of typed LLM
resources -- on this node, the MI355X GPUs (HBM bytes, batch slots, KV-token
budget).

Reference `internal/scheduler/resource_scheduler.go`:
  * register forces available / load 0 / heartbeat now (`:138-162`);
  * allocate: candidates available|busy, type == request model type,
    capabilities superset, capacity - used >= required for every type;
    lowest load wins; used += req; load = mean(used/capacity); busy if > 0.9
    (`:336-398`, `:598-688`); token = "<req>-<res>-<RFC3339>" (`:698-702`);
  * otherwise the request waits in a pending queue retried every second
    (`:213-234`, `:418-474`); monitor: heartbeat timeout -> offline,
    expired allocations released, autoscale check (`:401-571`).

Fixes: D10 (``queued_at`` is always set, no type-assert panic), D11 (release
subtracts exactly what was allocated; the reference halves ``Load`` and
never decrements ``Used``), D12 (pending queue ordered MORE urgent first:
lower priority int, then FIFO).  Autoscale decisions are returned/recorded and
drive ``on_scale``: on a GPU node the gateway wires it to park / unpark GPU
endpoints (``Gateway.attach_resource_scheduler``), which takes the GPU out of
(or back into) multi-GPU placement through the balancer's ``L_EXCLUDE`` view
-- the reference's `checkAutoScaling` (`:525-571`) only logs.
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

from ..models.message import format_time
from ..utils.logging import get_logger


class ResourceType:
    CPU = "cpu"
    GPU = "gpu"
    MEMORY = "memory"
    TOKENS = "tokens"


class ResourceStatus:
    AVAILABLE = "available"
    BUSY = "busy"
    OFFLINE = "offline"
    ERROR = "error"


class ResourceError(Exception):
    pass


class RequestQueued(ResourceError):
    def __init__(self):
        super().__init__("no resources available, request queued")


@dataclass
class Resource:
    id: str
    name: str = ""
    type: str = ""                       # model type
    capabilities: List[str] = field(default_factory=list)
    status: str = ResourceStatus.AVAILABLE
    load: float = 0.0
    capacity: Dict[str, int] = field(default_factory=dict)
    used: Dict[str, int] = field(default_factory=dict)
    endpoint: str = ""
    last_heartbeat: int = 0              # wall ns
    metadata: Dict[str, object] = field(default_factory=dict)

    def to_dict(self) -> dict:
        return {"id": self.id, "name": self.name, "type": self.type, "capabilities": list(self.capabilities),
                "status": self.status, "load": self.load, "capacity": dict(self.capacity),
                "used": dict(self.used), "endpoint": self.endpoint,
                "last_heartbeat": format_time(self.last_heartbeat), "metadata": self.metadata}

    @classmethod
    def from_dict(cls, d: dict) -> "Resource":
        if not isinstance(d, dict) or not d.get("id"):
            raise ValueError("resource id is required")
        return cls(id=str(d["id"]), name=str(d.get("name", "")), type=str(d.get("type", "")),
                   capabilities=list(d.get("capabilities") or []),
                   capacity={str(k): int(v) for k, v in (d.get("capacity") or {}).items()},
                   used={str(k): int(v) for k, v in (d.get("used") or {}).items()},
                   endpoint=str(d.get("endpoint", "")), metadata=dict(d.get("metadata") or {}))


@dataclass
class ResourceRequest:
    request_id: str
    model_type: str
    requirements: Dict[str, int] = field(default_factory=dict)
    priority: int = 3
    timeout: int = 0                     # ns; allocation lifetime and max queue wait
    capabilities: List[str] = field(default_factory=list)
    metadata: Dict[str, object] = field(default_factory=dict)
    queued_at: int = 0                   # monotonic ns (D10)
    seq: int = 0


@dataclass
class ResourceAllocation:
    request_id: str
    resource_id: str
    endpoint: str
    allocated: int
    expires: int                         # wall ns (0 = never)
    token: str
    requirements: Dict[str, int] = field(default_factory=dict)

    def to_dict(self) -> dict:
        return {"request_id": self.request_id, "resource_id": self.resource_id, "endpoint": self.endpoint,
                "allocated": format_time(self.allocated), "expires": format_time(self.expires) if self.expires else None,
                "token": self.token}


@dataclass
class ResourceSchedulerConfig:
    heartbeat_timeout: int = 30_000_000_000
    allocation_timeout: int = 30_000_000_000
    resource_check_period: int = 100_000_000
    pending_retry_period: int = 1_000_000_000
    enable_auto_scaling: bool = False
    min_resources: int = 1
    max_resources: int = 10
    scale_up_threshold: float = 0.8
    scale_down_threshold: float = 0.2
    scale_cooldown: int = 300_000_000_000


def _load(r: Resource) -> float:
    fr = [r.used.get(k, 0) / c for k, c in r.capacity.items() if c > 0]
    return sum(fr) / len(fr) if fr else 0.0


class ResourceScheduler:
    def __init__(self, cfg: Optional[ResourceSchedulerConfig] = None, logger=None, start: bool = True,
                 on_scale: Optional[Callable[[str, float], None]] = None):
        self.cfg = cfg or ResourceSchedulerConfig()
        self.logger = logger or get_logger("resource_scheduler")
        self._lock = threading.RLock()
        self.resources: Dict[str, Resource] = {}
        self.allocations: Dict[str, ResourceAllocation] = {}
        self.pending: List[ResourceRequest] = []
        self._seq = 0
        self._last_scale = 0.0
        self.on_scale = on_scale
        self.scale_events: List[dict] = []
        # resources taken out of service by a scale-down (GPU endpoints parked
        # in the balancer): not counted as active capacity, first to return
        self.parked: List[str] = []
        # demand waiting outside this scheduler's own pending queue: a gateway
        # reports its queued requests that no active GPU has a free slot for
        # (``note_backlog``).  They are pending resource requests in all but
        # name, so they count where the reference counts its pending queue
        # (`resource_scheduler.go:525-571`: scale up while it is non-empty).
        self.external_pending = 0
        self._stop = threading.Event()
        self._threads: List[threading.Thread] = []
        if start:
            self.start()

    @classmethod
    def from_config(cls, sched_cfg, **kw) -> "ResourceScheduler":
        return cls(ResourceSchedulerConfig(
            heartbeat_timeout=sched_cfg.heartbeat_timeout, allocation_timeout=sched_cfg.timeout,
            resource_check_period=sched_cfg.check_interval, enable_auto_scaling=sched_cfg.enable_auto_scaling,
            min_resources=sched_cfg.min_endpoints, max_resources=sched_cfg.max_endpoints,
            scale_cooldown=sched_cfg.autoscale_cooldown), **kw)

    def start(self) -> None:
        if self._threads:
            return
        for fn, period in ((self._monitor_tick, self.cfg.resource_check_period),
                           (self.process_pending_requests, self.cfg.pending_retry_period)):
            t = threading.Thread(target=self._loop, args=(fn, period), daemon=True)
            t.start()
            self._threads.append(t)

    def stop(self) -> None:
        self._stop.set()
        for t in self._threads:
            t.join(timeout=5)
        self._threads = []

    def _loop(self, fn, period_ns: int) -> None:
        while not self._stop.wait(max(period_ns, 1_000_000) / 1e9):
            try:
                fn()
            except Exception as e:
                self.logger.error("resource scheduler task failed", error=str(e))

    # ------------------------------------------------------------------ registry
    def register_resource(self, r: Resource) -> None:
        with self._lock:
            if r.id in self.resources:
                raise ResourceError("resource with this ID already exists")
            r.status = ResourceStatus.AVAILABLE
            r.load = _load(r)
            r.last_heartbeat = time.time_ns()
            self.resources[r.id] = r
        self.process_pending_requests()

    def update_resource_status(self, resource_id: str, status: str, load: float) -> None:
        with self._lock:
            r = self.resources.get(resource_id)
            if r is None:
                raise ResourceError("resource not found")
            r.status, r.load, r.last_heartbeat = status, float(load), time.time_ns()

    def heartbeat(self, resource_id: str, load: Optional[float] = None,
                  used: Optional[Dict[str, int]] = None, capacity: Optional[Dict[str, int]] = None) -> None:
        with self._lock:
            r = self.resources.get(resource_id)
            if r is None:
                raise ResourceError("resource not found")
            r.last_heartbeat = time.time_ns()
            if capacity:
                r.capacity.update({k: int(v) for k, v in capacity.items()})
            if used is not None:
                r.used = {k: int(v) for k, v in used.items()}
            r.load = float(load) if load is not None else _load(r)
            if r.status == ResourceStatus.OFFLINE:
                r.status = ResourceStatus.AVAILABLE

    # ------------------------------------------------------------------ allocation
    @staticmethod
    def _fits(r: Resource, req: ResourceRequest) -> bool:
        if r.status not in (ResourceStatus.AVAILABLE, ResourceStatus.BUSY) or r.type != req.model_type:
            return False
        if any(c not in r.capabilities for c in req.capabilities):
            return False
        for k, need in req.requirements.items():
            if k not in r.capacity or r.capacity[k] - r.used.get(k, 0) < need:
                return False
        return True

    def try_allocate(self, req: ResourceRequest) -> Optional[ResourceAllocation]:
        with self._lock:
            best = None
            for r in self.resources.values():
                if self._fits(r, req) and (best is None or r.load < best.load):
                    best = r
            if best is None:
                return None
            now = time.time_ns()
            lifetime = req.timeout or self.cfg.allocation_timeout
            alloc = ResourceAllocation(req.request_id, best.id, best.endpoint, now,
                                       now + lifetime if lifetime > 0 else 0,
                                       f"{req.request_id}-{best.id}-{format_time(now)}", dict(req.requirements))
            for k, need in req.requirements.items():
                best.used[k] = best.used.get(k, 0) + int(need)
            best.load = _load(best)
            if best.load > 0.9:
                best.status = ResourceStatus.BUSY
            self.allocations[req.request_id] = alloc
            return alloc

    def request_resource(self, req: ResourceRequest) -> ResourceAllocation:
        alloc = self.try_allocate(req)
        if alloc is not None:
            return alloc
        with self._lock:
            req.queued_at = time.monotonic_ns()
            self._seq += 1
            req.seq = self._seq
            self.pending.append(req)
            self.pending.sort(key=lambda q: (q.priority, q.seq))   # D12: urgent first, FIFO within
        raise RequestQueued()

    def _free(self, alloc: ResourceAllocation) -> None:
        r = self.resources.get(alloc.resource_id)
        if r is None:
            return
        for k, need in alloc.requirements.items():
            r.used[k] = max(0, r.used.get(k, 0) - int(need))
        r.load = _load(r)
        if r.status == ResourceStatus.BUSY and r.load <= 0.9:
            r.status = ResourceStatus.AVAILABLE

    def release_resource(self, request_id: str) -> None:
        with self._lock:
            alloc = self.allocations.pop(request_id, None)
            if alloc is None:
                raise ResourceError("allocation not found")
            self._free(alloc)
        self.process_pending_requests()

    def process_pending_requests(self) -> int:
        with self._lock:
            todo, self.pending = self.pending, []
        now = time.monotonic_ns()
        keep, granted = [], 0
        for req in todo:
            if req.timeout > 0 and now - req.queued_at > req.timeout:
                continue                      # waited too long: dropped
            if self.try_allocate(req) is not None:
                granted += 1
            else:
                keep.append(req)
        with self._lock:
            self.pending = sorted(keep + self.pending, key=lambda q: (q.priority, q.seq))
        return granted

    # ------------------------------------------------------------------ monitor
    def _monitor_tick(self) -> None:
        self.check_resource_status()
        self.check_allocations()
        self.check_auto_scaling()

    def check_resource_status(self) -> List[str]:
        now = time.time_ns()
        off = []
        with self._lock:
            for r in self.resources.values():
                if r.status != ResourceStatus.OFFLINE and now - r.last_heartbeat > self.cfg.heartbeat_timeout:
                    r.status = ResourceStatus.OFFLINE
                    off.append(r.id)
        for rid in off:
            self.logger.warning("Resource went offline", resource_id=rid)
        return off

    def check_allocations(self) -> int:
        now = time.time_ns()
        with self._lock:
            dead = [a for a in self.allocations.values() if a.expires and now > a.expires]
            for a in dead:
                del self.allocations[a.request_id]
                self._free(a)
        if dead:
            self.process_pending_requests()
        return len(dead)

    def average_load(self) -> float:
        with self._lock:
            act = [r.load for r in self.resources.values()
                   if r.status not in (ResourceStatus.OFFLINE, ResourceStatus.ERROR) and r.id not in self.parked]
        return sum(act) / len(act) if act else 0.0

    # ------------------------------------------------------------------ scale actions
    def scale_target(self, action: str) -> Optional[str]:
        """Which resource a scale action applies to: ``scale_down`` parks
        the least-loaded active one (ties: highest id, so GPU 0 -- which
        fronts HTTP -- goes last); ``scale_up`` returns the most recently
        parked one."""
        with self._lock:
            if action == "scale_up":
                return self.parked[-1] if self.parked else None
            act = [r for r in self.resources.values()
                   if r.status not in (ResourceStatus.OFFLINE, ResourceStatus.ERROR) and r.id not in self.parked]
            if len(act) <= max(1, self.cfg.min_resources):
                return None
            return min(act, key=lambda r: (r.load, [-ord(c) for c in r.id])).id

    def park(self, resource_id: str) -> None:
        with self._lock:
            if resource_id not in self.parked:
                self.parked.append(resource_id)
            r = self.resources.get(resource_id)
            if r is not None:
                r.metadata["parked"] = True

    def unpark(self, resource_id: str) -> None:
        with self._lock:
            if resource_id in self.parked:
                self.parked.remove(resource_id)
            r = self.resources.get(resource_id)
            if r is not None:
                r.metadata.pop("parked", None)

    def note_backlog(self, n: int) -> None:
        self.external_pending = max(0, int(n))

    def check_auto_scaling(self) -> Optional[str]:
        if not self.cfg.enable_auto_scaling:
            return None
        if time.monotonic() - self._last_scale < self.cfg.scale_cooldown / 1e9:
            return None
        with self._lock:
            active = sum(1 for r in self.resources.values()
                         if r.status not in (ResourceStatus.OFFLINE, ResourceStatus.ERROR)
                         and r.id not in self.parked)
            pend = len(self.pending) + self.external_pending
        avg = self.average_load()
        action = None
        if (avg > self.cfg.scale_up_threshold or pend > 0) and active < self.cfg.max_resources:
            action = "scale_up"
        elif avg < self.cfg.scale_down_threshold and pend == 0 and active > self.cfg.min_resources:
            action = "scale_down"
        if action:
            self._last_scale = time.monotonic()
            self.scale_events.append({"action": action, "average_load": avg, "pending": pend})
            if self.on_scale is not None:
                self.on_scale(action, avg)
        return action

    # ------------------------------------------------------------------ queries
    def get_resource_stats(self) -> dict:
        with self._lock:
            st = {"total": len(self.resources), "available": 0, "busy": 0, "offline": 0, "error": 0}
            by_type: Dict[str, int] = {}
            for r in self.resources.values():
                if r.status in st:
                    st[r.status] += 1
                by_type[r.type] = by_type.get(r.type, 0) + 1
            return {"resources": st, "resource_by_type": by_type, "average_load": self.average_load(),
                    "allocations": len(self.allocations), "pending_requests": len(self.pending)}

    def get_allocation(self, request_id: str) -> ResourceAllocation:
        with self._lock:
            a = self.allocations.get(request_id)
        if a is None:
            raise ResourceError("allocation not found")
        return a

    def get_resource(self, resource_id: str) -> Resource:
        with self._lock:
            r = self.resources.get(resource_id)
        if r is None:
            raise ResourceError("resource not found")
        return r

    def get_all_resources(self) -> List[Resource]:
        with self._lock:
            return list(self.resources.values())

    def get_all_allocations(self) -> List[ResourceAllocation]:
        with self._lock:
            return list(self.allocations.values())

    def get_pending_queue_length(self) -> int:
        with self._lock:
            return len(self.pending)

    # ------------------------------------------------------------------ MI355X
    def register_gpu(self, gpu: int, model_type: str, slots: int, hbm_total: int, kv_tokens: int,
                     endpoint: str = "") -> Resource:
        """A GPU backend as a typed resource: gpu = batch slots, memory = HBM
        bytes, tokens = KV-cache token budget."""
        r = Resource(id=f"gpu{gpu}", name=f"MI355X #{gpu}", type=model_type, capabilities=["mi355x", "bf16"],
                     capacity={ResourceType.GPU: slots, ResourceType.MEMORY: hbm_total,
                               ResourceType.TOKENS: kv_tokens},
                     endpoint=endpoint or f"gpu://{gpu}", metadata={"gpu_index": gpu})
        self.register_resource(r)
        return r
