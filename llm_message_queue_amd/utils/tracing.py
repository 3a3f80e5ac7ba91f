"""Per-request tracing (SURVEY.md §5 "tracing / profiling"; the reference's
pprof/Jaeger tracing is doc-only, `docs/performance.md:886-997`).

``RequestTracer`` samples requests and records their lifecycle timestamps
(arrival at ingress, enqueue into the C++ queue, dispatch to a GPU slot,
completion) plus backend step spans, and writes a Chrome trace
(``chrome://tracing`` / Perfetto JSON): one track per priority tier with a
"queued" and a "served" slice per sampled request, and one track for the
backend's forward steps.  Kernel-level timing comes from rocprofv3; this
covers the gateway-level view that joins them.
"""
from __future__ import annotations

import json
import threading
import time
from typing import List, Optional

TIER_NAMES = ("realtime", "high", "normal", "low")


class RequestTracer:
    def __init__(self, sample_every: int = 100, max_events: int = 200_000):
        self.sample_every = max(1, int(sample_every))
        self.max_events = max_events
        self._n = 0
        self._reqs: List[tuple] = []
        self._steps: List[tuple] = []
        self._lock = threading.Lock()
        self.t0_ns = time.monotonic_ns()

    def request(self, m, done_ns: Optional[int] = None) -> None:
        """Record a completed message (uses its monotonic timestamps)."""
        self._n += 1
        if self._n % self.sample_every:
            return
        with self._lock:
            if len(self._reqs) < self.max_events:
                self._reqs.append((m.id, int(getattr(m, "tier", -1)), int(m.arrival_ns or 0), int(m.enqueued_at or 0),
                                   int(m.dispatched_at or 0), int(done_ns or time.monotonic_ns()),
                                   str(getattr(m, "endpoint_id", ""))))

    def step(self, step_id: int, start_ns: int, end_ns: int, tokens: int) -> None:
        with self._lock:
            if len(self._steps) < self.max_events:
                self._steps.append((int(step_id), int(start_ns), int(end_ns), int(tokens)))

    def chrome_events(self) -> list:
        us = lambda ns: (ns - self.t0_ns) / 1e3      # noqa: E731
        ev = [{"ph": "M", "name": "process_name", "pid": 1, "args": {"name": "gateway"}}]
        for t, name in enumerate(TIER_NAMES):
            ev.append({"ph": "M", "name": "thread_name", "pid": 1, "tid": t + 1, "args": {"name": f"tier {name}"}})
        ev.append({"ph": "M", "name": "thread_name", "pid": 1, "tid": 10, "args": {"name": "backend steps"}})
        with self._lock:
            reqs, steps = list(self._reqs), list(self._steps)
        for mid, tier, arr, enq, disp, done, ep in reqs:
            tid = tier + 1 if 0 <= tier < 4 else 5
            start = arr or enq
            if start and disp:
                ev.append({"ph": "X", "name": "queued", "pid": 1, "tid": tid, "ts": us(start),
                           "dur": max(0.0, (disp - start) / 1e3), "args": {"id": mid, "enqueue_us": us(enq)}})
            if disp:
                ev.append({"ph": "X", "name": "served", "pid": 1, "tid": tid, "ts": us(disp),
                           "dur": max(0.0, (done - disp) / 1e3), "args": {"id": mid, "endpoint": ep}})
        for sid, a, b, tok in steps:
            ev.append({"ph": "X", "name": f"step {sid}", "pid": 1, "tid": 10, "ts": us(a),
                       "dur": max(0.0, (b - a) / 1e3), "args": {"tokens": tok}})
        return ev

    def dump(self, path: str) -> int:
        ev = self.chrome_events()
        with open(path, "w") as f:
            json.dump({"traceEvents": ev, "displayTimeUnit": "ms"}, f)
        return len(ev)
