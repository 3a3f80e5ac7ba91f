"""DeadLetterQueue (component C9).

Reference `internal/priorityqueue/dead_letter_queue.go`:
  * bounded list; ``push`` records reason/source/retry count, fires handlers
    asynchronously and notifies channels without blocking (`:62-119`);
  * ``requeue(i, qm)`` resets RetryCount and pushes to the source queue
    (`:187-215`); ``batch_requeue`` processes indices in descending order
    (`:218-258`).
Additions: lookup/requeue by message id (the API's requeue routes return 501
in the reference, `api/handlers.go:661-697`).
"""
from __future__ import annotations

import queue as _pyqueue
import threading
import time
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence

from ..models.message import Message, format_time
from ..utils.logging import get_logger
from .core import IndexOutOfRange, QueueFull


@dataclass
class DeadLetterItem:
    message: Message
    fail_reason: str
    failed_at: int          # wall ns
    source_queue: str
    retry_count: int

    def to_dict(self) -> dict:
        return {"message": self.message.to_dict(), "fail_reason": self.fail_reason,
                "failed_at": format_time(self.failed_at), "source_queue": self.source_queue,
                "retry_count": self.retry_count}


DeadLetterHandler = Callable[[DeadLetterItem], Optional[BaseException]]


class DeadLetterQueue:
    def __init__(self, max_size: int = 0, logger=None):
        self.max_size = int(max_size)
        self._items: List[DeadLetterItem] = []
        self._lock = threading.RLock()
        self._handlers: List[DeadLetterHandler] = []
        self._notify: List[_pyqueue.Queue] = []
        self.logger = logger or get_logger("dead_letter_queue")
        self.dropped_notifications = 0
        # handlers run asynchronously (the reference's `go handler(item)`) on
        # ONE worker thread fed by a queue -- a thread per item per handler
        # would spawn thousands of threads a second when overload shedding
        # moves whole batches here
        self._work: _pyqueue.SimpleQueue = _pyqueue.SimpleQueue()
        self._worker: Optional[threading.Thread] = None
        # bulk moves log at most once per LOG_EVERY_S with the count since the last line
        self._log_next = 0.0
        self._log_pending = 0

    def add_handler(self, handler: DeadLetterHandler) -> None:
        with self._lock:
            self._handlers.append(handler)

    def add_notification_channel(self, ch: _pyqueue.Queue) -> None:
        with self._lock:
            self._notify.append(ch)

    def push(self, message: Message, fail_reason: str, source_queue: str) -> None:
        with self._lock:
            if self.max_size > 0 and len(self._items) >= self.max_size:
                raise QueueFull()
            item = DeadLetterItem(message, str(fail_reason), time.time_ns(), source_queue,
                                  message.retry_count)
            self._items.append(item)
            handlers = list(self._handlers)
            chans = list(self._notify)
        self.logger.warning("Message moved to dead letter queue", message_id=message.id,
                            reason=str(fail_reason), source=source_queue)
        for h in handlers:
            self._submit(h, item)
        for ch in chans:
            try:
                ch.put_nowait(item)
            except _pyqueue.Full:
                self.dropped_notifications += 1

    def push_many(self, messages: Sequence[Message], fail_reason: str, source_queue: str) -> int:
        """Bulk ``push`` (one log line; overload shedding moves thousands at
        once).  Items beyond ``max_size`` are dropped; returns how many were
        kept."""
        now = time.time_ns()
        with self._lock:
            room = len(messages) if self.max_size <= 0 else max(0, self.max_size - len(self._items))
            items = [DeadLetterItem(m, str(fail_reason), now, source_queue, m.retry_count) for m in messages[:room]]
            self._items.extend(items)
            handlers = list(self._handlers)
            chans = list(self._notify)
        if items:
            self._log_pending += len(items)
            t = time.monotonic()
            if t >= self._log_next:
                self.logger.warning("Messages moved to dead letter queue", count=self._log_pending,
                                    reason=str(fail_reason), source=source_queue,
                                    dropped=len(messages) - len(items))
                self._log_pending = 0
                self._log_next = t + self.LOG_EVERY_S
        for item in items:
            for h in handlers:
                self._submit(h, item)
            for ch in chans:
                try:
                    ch.put_nowait(item)
                except _pyqueue.Full:
                    self.dropped_notifications += 1
        return len(items)

    def restore(self, item: DeadLetterItem) -> None:
        """Re-insert an item from a snapshot (no handlers/notifications fire)."""
        with self._lock:
            self._items.append(item)

    LOG_EVERY_S = 1.0

    def _submit(self, h: DeadLetterHandler, item: DeadLetterItem) -> None:
        self._work.put((h, item))
        if self._worker is None or not self._worker.is_alive():
            with self._lock:
                if self._worker is None or not self._worker.is_alive():
                    self._worker = threading.Thread(target=self._drain, name="dlq-handlers", daemon=True)
                    self._worker.start()

    def _drain(self) -> None:
        while True:
            h, item = self._work.get()
            self._run_handler(h, item)

    def _run_handler(self, h: DeadLetterHandler, item: DeadLetterItem) -> None:
        try:
            err = h(item)
        except Exception as e:
            err = e
        if err:
            self.logger.error("Dead letter handler failed", message_id=item.message.id, error=str(err))

    def get(self, index: int) -> DeadLetterItem:
        with self._lock:
            if index < 0 or index >= len(self._items):
                raise IndexOutOfRange()
            return self._items[index]

    def remove(self, index: int) -> None:
        with self._lock:
            if index < 0 or index >= len(self._items):
                raise IndexOutOfRange()
            del self._items[index]

    def size(self) -> int:
        with self._lock:
            return len(self._items)

    def get_all(self) -> List[DeadLetterItem]:
        with self._lock:
            return list(self._items)

    def clear(self) -> None:
        with self._lock:
            self._items = []

    def index_of(self, message_id: str) -> int:
        with self._lock:
            for i, it in enumerate(self._items):
                if it.message.id == message_id:
                    return i
        return -1

    def requeue(self, index: int, queue_manager) -> None:
        with self._lock:
            if index < 0 or index >= len(self._items):
                raise IndexOutOfRange()
            item = self._items[index]
            item.message.retry_count = 0
            item.message.status = "pending"
            queue_manager.push_message(item.source_queue, item.message)
            del self._items[index]

    def requeue_by_id(self, message_id: str, queue_manager) -> None:
        with self._lock:
            i = self.index_of(message_id)
            if i < 0:
                raise IndexOutOfRange(f"message {message_id} not in dead letter queue")
            self.requeue(i, queue_manager)

    def batch_requeue(self, indices: List[int], queue_manager) -> int:
        if not indices:
            return 0
        ok = 0
        with self._lock:
            for index in sorted(indices, reverse=True):
                if index < 0 or index >= len(self._items):
                    continue
                item = self._items[index]
                item.message.retry_count = 0
                item.message.status = "pending"
                try:
                    queue_manager.push_message(item.source_queue, item.message)
                except Exception:
                    continue
                del self._items[index]
                ok += 1
        return ok

    def requeue_all(self, queue_manager) -> int:
        with self._lock:
            return self.batch_requeue(list(range(len(self._items))), queue_manager)
