"""Telemetry service (N8 + failure detection): publishes the native amd-smi
poller's snapshot to the node-shared load pages (HBM used/total, busy %), the
Prometheus gauges, and the ResourceScheduler (``Heartbeat`` with used HBM),
and flags GPUs as unhealthy when amd-smi stops answering or the uncorrectable
ECC count rises -- the reference's health check is a stub that always
succeeds (`internal/loadbalancer/load_balancer.go:588-616`, D9).

GPU index mapping: amd-smi enumerates every GPU of the node in PCI order,
which is also HIP's default order; a process restricted with
``HIP_VISIBLE_DEVICES`` passes an explicit ``gpu_map``.
"""
from __future__ import annotations

import threading
from typing import Callable, Dict, List, Optional

from .. import _native
from ..utils.logging import get_logger


def hip_gpu_map(pci_addresses) -> Dict[int, Optional[int]]:
    """amd-smi index -> visible HIP device index, matched on PCI domain/bus/
    device (function ignored).  Unmatched (other containers' GPUs) -> None."""
    import torch
    if not torch.cuda.is_available():
        return {}
    hip = {}
    for i in range(torch.cuda.device_count()):
        p = torch.cuda.get_device_properties(i)
        hip[(int(p.pci_domain_id) << 16) | (int(p.pci_bus_id) << 8) | (int(p.pci_device_id) << 3)] = i
    out: Dict[int, Optional[int]] = {}
    for k, addr in enumerate(pci_addresses):
        out[k] = hip.get(int(addr) & ~0x7) if addr >= 0 else None
    if not any(v is not None for v in out.values()):
        return {}                            # no PCI info: fall back to index order
    return out


class TelemetryService:
    def __init__(self, period_ms: int = 20, pages: Optional[Dict[int, object]] = None, metrics=None,
                 resource_scheduler=None, on_unhealthy: Optional[Callable[[int, str], None]] = None,
                 synthetic: int = 0, gpu_map: Optional[Dict[int, int]] = None):
        self.native = _native.telemetry().Telemetry(int(period_ms))
        if gpu_map is None and self.native.available():
            gpu_map = hip_gpu_map(self.native.pci_addresses())
        self.period_s = period_ms / 1e3
        self.pages = pages or {}
        self.metrics = metrics
        self.rs = resource_scheduler
        self.on_unhealthy = on_unhealthy
        self.synthetic = synthetic
        # amd-smi index -> HIP device index (by PCI address); GPUs of the node
        # that this process cannot see map to None and are ignored
        self.gpu_map = gpu_map if gpu_map is not None else {}
        self.log = get_logger("telemetry")
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self._ecc0: Dict[int, int] = {}
        self.unhealthy: Dict[int, str] = {}
        self.last: List[dict] = []

    @property
    def available(self) -> bool:
        return self.native.available()

    def start(self) -> None:
        self.native.start()
        if self._thread is None:
            self._thread = threading.Thread(target=self._loop, name="telemetry", daemon=True)
            self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=2)
        self.native.stop()

    def _loop(self) -> None:
        while not self._stop.wait(self.period_s):
            self.publish()

    def inject(self, gpu: int, field: str, value: float) -> None:
        """Fault injection: override a telemetry field (e.g. valid=0, ecc_uncorrectable=5)."""
        self.native.inject(gpu, field, float(value))

    def publish(self) -> List[dict]:
        snap = self.native.snapshot(self.synthetic)
        self.last = snap
        for s in snap:
            g = self.gpu_map.get(s["gpu"], s["gpu"]) if self.gpu_map else s["gpu"]
            if g is None:
                continue
            if s.get("ts_ns", 1) == 0 and s["valid"] is False and not self.synthetic:
                continue                    # not polled yet
            page = self.pages.get(g)
            if page is not None:
                page.set_telemetry(int(s["hbm_used_mb"]), int(s["hbm_total_mb"]), int(s["gfx_pct"]))
            if self.metrics is not None:
                self.metrics.hbm_used.labels(str(g)).set(int(s["hbm_used_mb"]) << 20)
                if page is not None:
                    self.metrics.inflight.labels(str(g)).set(page.active())
            if self.rs is not None and s["valid"]:
                try:
                    # device-level HBM (amd-smi) rides in the metadata: the
                    # resource's "memory" dimension is the serving footprint
                    # (weights + live KV) the gateway heartbeats every tick
                    r = self.rs.get_resource(f"gpu{g}")
                    r.metadata["hbm_device_used"] = int(s["hbm_used_mb"]) << 20
                    r.metadata["hbm_device_total"] = int(s["hbm_total_mb"]) << 20
                    self.rs.heartbeat(f"gpu{g}", used=dict(r.used))
                except Exception:
                    pass
            self._health(g, s)
        return snap

    def _health(self, g: int, s: dict) -> None:
        reason = ""
        if not s["valid"] and (self.available or self.synthetic):
            reason = "telemetry unavailable"
        ecc = int(s["ecc_uncorrectable"])
        base = self._ecc0.setdefault(g, ecc)
        if ecc > base:
            reason = f"uncorrectable ECC errors: {ecc - base}"
        if reason and g not in self.unhealthy:
            self.unhealthy[g] = reason
            self.log.warning("GPU unhealthy", gpu=g, reason=reason)
            page = self.pages.get(g)
            if page is not None:
                page.set_health(False)
            if self.on_unhealthy is not None:
                self.on_unhealthy(g, reason)
        elif not reason and g in self.unhealthy:
            del self.unhealthy[g]
            page = self.pages.get(g)
            if page is not None:
                page.set_health(True)
