"""Prometheus metrics (reference `queue_manager.go:46-156`), fixed:

  * ONE shared registry with a ``manager`` label, so creating a second queue
    manager no longer panics on duplicate registration (defect D5);
  * ``/metrics`` is actually served by the API server (defect D6);
  * the wait-time histogram is observed per tier at dispatch (defect D23) and
    complete/fail carry the real priority label instead of ``"unknown"``.

New series for the MI355X gateway: ``llm_queue_enqueue_to_dispatch_seconds``
(the north-star latency), ``llm_gpu_hbm_used_bytes``, ``llm_gpu_inflight_slots``,
``llm_preprocess_kernel_seconds``.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional

try:  # prometheus_client is in the image; degrade to no-ops if absent
    from prometheus_client import (CollectorRegistry, Counter, Gauge, Histogram,
                                   generate_latest, CONTENT_TYPE_LATEST)
    HAVE_PROM = True
except Exception:  # pragma: no cover
    HAVE_PROM = False
    CONTENT_TYPE_LATEST = "text/plain; version=0.0.4; charset=utf-8"


def _exp_buckets(start: float, factor: float, count: int):
    return tuple(start * factor ** i for i in range(count))


class _Noop:
    def labels(self, *a, **k):
        return self

    def inc(self, *a, **k):
        pass

    def dec(self, *a, **k):
        pass

    def set(self, *a, **k):
        pass

    def observe(self, *a, **k):
        pass

    def set_function(self, *a, **k):
        pass


class QueueMetrics:
    """All gateway series, registered once per registry."""

    def __init__(self, registry=None):
        if not HAVE_PROM:
            self.registry = None
            n = _Noop()
            for name in ("pending", "processing", "completed", "failed", "wait_time",
                         "process_time", "operations", "dispatch_latency", "hbm_used",
                         "inflight", "preprocess_seconds", "dead_letter", "requests_rejected"):
                setattr(self, name, n)
            return
        self.registry = registry or CollectorRegistry()
        L = ["manager", "queue", "priority"]
        r = self.registry
        self.pending = Gauge("llm_queue_messages_pending_total",
                             "Number of pending messages in queue", L, registry=r)
        self.processing = Gauge("llm_queue_messages_processing_total",
                                "Number of processing messages in queue", L, registry=r)
        self.completed = Counter("llm_queue_messages_completed_total",
                                 "Total number of completed messages", L, registry=r)
        self.failed = Counter("llm_queue_messages_failed_total",
                              "Total number of failed messages", L, registry=r)
        self.wait_time = Histogram("llm_queue_messages_wait_time_seconds",
                                   "Time messages spend waiting in queue", L,
                                   buckets=_exp_buckets(0.01, 2, 15), registry=r)
        self.process_time = Histogram("llm_queue_messages_process_time_seconds",
                                      "Time spent processing messages", L,
                                      buckets=_exp_buckets(0.1, 2, 15), registry=r)
        self.operations = Counter("llm_queue_operations_total",
                                  "Total number of queue operations",
                                  ["manager", "queue", "operation"], registry=r)
        self.dispatch_latency = Histogram(
            "llm_queue_enqueue_to_dispatch_seconds",
            "Enqueue to dispatch latency per tier", ["tier"],
            buckets=_exp_buckets(0.0001, 2, 20), registry=r)
        self.hbm_used = Gauge("llm_gpu_hbm_used_bytes", "HBM bytes in use per GPU", ["gpu"],
                              registry=r)
        self.inflight = Gauge("llm_gpu_inflight_slots", "In-flight batch slots per GPU", ["gpu"],
                              registry=r)
        self.preprocess_seconds = Histogram(
            "llm_preprocess_kernel_seconds", "GPU preprocess batch time", ["stage"],
            buckets=_exp_buckets(0.00001, 2, 20), registry=r)
        self.dead_letter = Gauge("llm_queue_dead_letter_size", "Dead-letter queue size",
                                 ["manager"], registry=r)
        self.requests_rejected = Counter("llm_queue_requests_rejected_total",
                                         "Requests rejected at admission", ["reason"],
                                         registry=r)
        self.grpc_requests = Counter("llm_grpc_requests_total", "gRPC calls by method and final status",
                                     ["method", "code"], registry=r)

    def render(self) -> bytes:
        if not HAVE_PROM or self.registry is None:
            return b""
        return generate_latest(self.registry)


_DEFAULT: Optional[QueueMetrics] = None
_LOCK = threading.Lock()


def default_metrics() -> QueueMetrics:
    global _DEFAULT
    with _LOCK:
        if _DEFAULT is None:
            _DEFAULT = QueueMetrics()
        return _DEFAULT


def reset_default_metrics() -> QueueMetrics:
    """Fresh registry (tests)."""
    global _DEFAULT
    with _LOCK:
        _DEFAULT = QueueMetrics()
        return _DEFAULT


def _with_rank(line: str, rank: int) -> str:
    """One exposition sample line with a ``rank`` label added."""
    i = 0
    while i < len(line) and line[i] not in "{ ":
        i += 1
    if i < len(line) and line[i] == "{":
        sep = "" if line[i + 1:i + 2] == "}" else ","
        return f'{line[:i + 1]}rank="{rank}"{sep}{line[i + 1:]}'
    return f'{line[:i]}{{rank="{rank}"}}{line[i:]}'


def merge_expositions(parts: Dict[int, str]) -> bytes:
    """Prometheus text expositions of several ranks as one: every sample gets
    a ``rank`` label and each metric family stays one contiguous block under
    a single HELP / TYPE header (the multi-GPU front door's ``/metrics``: one
    scrape target for the whole job)."""
    blocks: Dict[str, List[List[str]]] = {}
    order: List[str] = []
    for rank, text in sorted(parts.items()):
        fam = ""
        for line in text.splitlines():
            if not line:
                continue
            if line.startswith("# HELP ") or line.startswith("# TYPE "):
                fam = line.split(" ", 3)[2]
                if fam not in blocks:
                    blocks[fam] = [[], []]
                    order.append(fam)
                if line not in blocks[fam][0]:
                    blocks[fam][0].append(line)
                continue
            if line.startswith("#"):
                continue
            if fam not in blocks:
                blocks[fam] = [[], []]
                order.append(fam)
            blocks[fam][1].append(_with_rank(line, rank))
    out: List[str] = []
    for fam in order:
        out.extend(blocks[fam][0])
        out.extend(blocks[fam][1])
    return ("\n".join(out) + "\n").encode() if out else b""
