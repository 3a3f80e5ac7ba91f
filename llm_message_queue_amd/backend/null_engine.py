"""Null backend: the BackendEngine interface with no model.  Every admitted
request completes at the next ``finish``.  Used to measure the gateway's own
capacity (GPU preprocess + native queue + dispatcher) in isolation -- the
quantity the reference's ">10,000 messages/s" target describes, since the
reference never calls a model."""
from __future__ import annotations

import time
from typing import List, Sequence

from .engine import Request, StepResult


class NullEngine:
    def __init__(self, slots: int = 4096):
        self.slots = slots
        self.active: List[Request] = []
        self.total_tokens = 0
        self.completed_total = 0
        self.completed_tokens = 0
        self.step_id = 0
        self._launched: List[Request] = []
        self.page = None

    def free_slots(self) -> int:
        return self.slots - len(self.active)

    def admit_capacity(self) -> int:
        return self.free_slots()

    def lane_capacity(self) -> int:
        return self.free_slots()

    def queued_steps(self) -> int:
        return 0

    def poll_one(self) -> bool:
        return False

    def warm_shapes(self, sizes=None) -> int:
        return 0

    def inflight(self) -> int:
        return len(self.active)

    def admit(self, reqs: Sequence[Request]) -> List[Request]:
        n = min(len(reqs), self.free_slots())
        now = time.monotonic_ns()
        out = list(reqs[:n])
        for r in out:
            r.admitted_ns = now
        self.active.extend(out)
        return out

    def launch(self, wait_cb=None) -> None:
        self._launched, self.active = self.active, []
        self.step_id += 1

    def sync(self) -> None:
        pass

    def finish(self, block: bool = False) -> StepResult:
        done, self._launched = self._launched, []
        now = time.monotonic_ns()
        for r in done:
            r.generated = r.gen_tokens
            r.done_ns = now
        self.completed_total += len(done)
        return StepResult(0, 0, 0, done, done, 0.0)

    def step(self) -> StepResult:
        self.launch()
        return self.finish()
