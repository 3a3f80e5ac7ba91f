"""DelayedQueue (component C8) over the native timer heap (N7).

Reference `internal/priorityqueue/delayed_queue.go`: ``schedule(msg, ready_at)``
delivers ``process_fn(msg)`` no earlier than ``ready_at`` (1 ms early-fire
tolerance), ordered by ``ready_at``; ``peek`` returns (msg, ready_at, ok).
The waker thread is C++; a Python thread drains due handles and calls
``process_fn`` serially (as `processReadyItems`, `:202-229`, does).
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Dict, Optional, Tuple

from .. import _native
from ..models.message import Message
from ..utils.logging import get_logger


class DelayedQueue:
    def __init__(self, process_fn: Optional[Callable[[Message], Optional[BaseException]]] = None,
                 logger=None):
        self._native = _native.mlq().DelayedQueue()
        # handle -> (msg, ready_at wall ns, per-item delivery target or None)
        self._items: Dict[int, Tuple[Message, int, Optional[Callable]]] = {}
        self._lock = threading.Lock()
        self.process_fn = process_fn
        self.logger = logger or get_logger("delayed_queue")
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.delivered = 0
        self.errors = 0

    def start(self) -> None:
        if self._thread is not None:
            return
        self._stop.clear()
        self._thread = threading.Thread(target=self._drain, name="delayed-queue", daemon=True)
        self._thread.start()
        # a queue nobody closed: stop its drain thread before interpreter
        # teardown destroys the native object it is blocked in
        import atexit
        import weakref
        ref = weakref.ref(self)
        atexit.register(lambda: (lambda q: q.stop() if q is not None else None)(ref()))

    def stop(self) -> None:
        self._stop.set()
        t = self._thread
        self._thread = None
        if t is not None:
            t.join(timeout=5)

    def close(self) -> None:
        self.stop()
        self._native.shutdown()

    # -------------------------------------------------------------- scheduling
    def schedule(self, message: Message, ready_at_ns: int,
                 target: Optional[Callable[[Message], Optional[BaseException]]] = None) -> None:
        """``ready_at_ns`` is wall-clock ns (``time.time_ns()`` domain).
        ``target`` (optional) receives this item instead of ``process_fn``
        (used by workers to route a retry back to its source queue)."""
        delay = int(ready_at_ns) - time.time_ns()
        with self._lock:
            self._items[message.handle] = (message, int(ready_at_ns), target)
        self._native.schedule(message.handle, time.monotonic_ns() + delay)

    def schedule_after(self, message: Message, delay_ns: int, target=None) -> None:
        self.schedule(message, time.time_ns() + int(delay_ns), target)

    def remove(self, message) -> bool:
        """Take a scheduled message out before it is delivered (``DELETE
        /api/v1/messages/{id}`` or ``DELETE /api/v1/admin/queues/delayed/{id}``
        on a request waiting out a retry backoff).  ``message``: a Message or
        its handle.  True if it was waiting (it will never be delivered);
        False if it is not here, including one the drain thread already took
        (the item map is the authority: delivery and removal both pop it
        under the same lock, so exactly one of them wins)."""
        h = message if isinstance(message, int) else message.handle
        with self._lock:
            item = self._items.pop(h, None)
        if item is None:
            return False
        self._native.remove(h)
        return True

    def find(self, message_id: str) -> Optional[Message]:
        """The scheduled message with this id (None: not waiting here)."""
        with self._lock:
            for msg, _ready, _t in self._items.values():
                if msg.id == message_id:
                    return msg
        return None

    # -------------------------------------------------------------- delivery
    def _drain(self) -> None:
        while not self._stop.is_set():
            handles = self._native.wait_ready(256, 0.05)
            for h in handles:
                with self._lock:
                    item = self._items.pop(h, None)
                if item is None:
                    continue
                msg, _ready, target = item
                self.delivered += 1
                fn = target or self.process_fn
                if fn is None:
                    continue
                try:
                    err = fn(msg)
                except Exception as e:  # processFn error is logged, not fatal
                    err = e
                if err:
                    self.errors += 1
                    self.logger.warning("Failed to process delayed message", message_id=msg.id,
                                        error=str(err))

    def poll_ready(self, max_n: int = 256, timeout_s: float = 0.0):
        """Synchronous drain (when no drain thread runs)."""
        out = []
        for h in self._native.wait_ready(max_n, timeout_s):
            with self._lock:
                item = self._items.pop(h, None)
            if item is not None:
                out.append(item[0])
        return out

    # -------------------------------------------------------------- inspection
    def size(self) -> int:
        return self._native.size()

    def peek(self) -> Tuple[Optional[Message], int, bool]:
        ok, h, _ready_mono = self._native.peek()
        if not ok:
            return None, 0, False
        with self._lock:
            item = self._items.get(h)
        if item is None:
            return None, 0, False
        return item[0], item[1], True

    def items(self):
        """[(msg, ready_at wall ns, target)] of every scheduled item (snapshot)."""
        with self._lock:
            return list(self._items.values())

    def clear(self) -> None:
        for h in self._native.clear():
            with self._lock:
                self._items.pop(h, None)
