"""Ingress micro-batcher: concurrent HTTP handlers hand messages to one
thread that flushes them in batches (every ``window_us`` or ``max_batch``) so
the GPU preprocess pipeline runs one fused launch chain per batch instead of
one per request.  Each caller blocks on its own future.

Reference: `api/handlers.go:160-219` preprocesses and enqueues each request
inside its own handler; here the handlers only hand off.
"""
from __future__ import annotations

import threading
import time
from concurrent.futures import Future
from typing import Callable, List, Sequence, Tuple

from ..models.message import Message


class MicroBatcher:
    def __init__(self, flush_fn: Callable[[Sequence[Message]], Sequence[object]], window_us: int = 500,
                 max_batch: int = 4096):
        self.flush_fn = flush_fn
        self.window_s = window_us / 1e6
        self.max_batch = max_batch
        self._items: List[Tuple[Message, Future]] = []
        self._cv = threading.Condition()
        self._stop = False
        self.batches = 0
        self._t = threading.Thread(target=self._loop, name="ingress-batcher", daemon=True)
        self._t.start()

    def submit(self, msg: Message) -> Future:
        f: Future = Future()
        with self._cv:
            self._items.append((msg, f))
            if len(self._items) == 1 or len(self._items) >= self.max_batch:
                self._cv.notify()
        return f

    def _loop(self) -> None:
        while True:
            with self._cv:
                while not self._items and not self._stop:
                    self._cv.wait(0.1)
                if self._stop and not self._items:
                    return
                deadline = time.monotonic() + self.window_s
                while len(self._items) < self.max_batch and not self._stop:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        break
                    self._cv.wait(left)
                batch, self._items = self._items[:self.max_batch], self._items[self.max_batch:]
            msgs = [m for m, _ in batch]
            try:
                results = self.flush_fn(msgs)
                self.batches += 1
                for (_, f), r in zip(batch, results):
                    f.set_result(r)
            except Exception as e:   # every waiter sees the failure
                for _, f in batch:
                    if not f.done():
                        f.set_exception(e)

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        self._t.join(timeout=5)
