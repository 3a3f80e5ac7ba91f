"""MultiLevelQueue (component C3) over the native bucket-queue core (N6).

Reference: `internal/priorityqueue/queue.go`.  The API keeps the reference's
method set (AddQueue/Push/Pop/Peek/Size/GetStats/GetAllStats/CompleteMessage/
FailMessage) in snake_case; the storage is the C++ ``_mlq`` module, which
carries integer handles only.  Message objects live in ``self._store``.
"""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np

from .. import _native
from ..models.message import Message, QueueStats


class QueueError(Exception):
    """``QueueError{Code, Message}`` (`queue.go:213-226`)."""

    code = "QUEUE_ERROR"
    message = "queue error"

    def __init__(self, message: Optional[str] = None):
        super().__init__(message or self.message)

    def __str__(self) -> str:
        return self.args[0] if self.args else self.message


class QueueNotFound(QueueError):
    code = "QUEUE_NOT_FOUND"
    message = "queue not found"


class QueueFull(QueueError):
    code = "QUEUE_FULL"
    message = "queue is full"


class QueueEmpty(QueueError):
    code = "QUEUE_EMPTY"
    message = "queue is empty"


class IndexOutOfRange(QueueError):
    """`dead_letter_queue.go:273-275`."""
    code = "INDEX_OUT_OF_RANGE"
    message = "index out of range"


# Go-style sentinel aliases
ErrQueueNotFound = QueueNotFound
ErrQueueFull = QueueFull
ErrQueueEmpty = QueueEmpty
ErrIndexOutOfRange = IndexOutOfRange

_STATUS_ERR = {1: QueueNotFound, 2: QueueFull, 3: QueueEmpty}

# monotonic <-> wall clock conversion for timestamps surfaced to users
_WALL_MINUS_MONO = time.time_ns() - time.monotonic_ns()


def mono_to_wall_ns(mono_ns: int) -> int:
    return int(mono_ns) + _WALL_MINUS_MONO


class MultiLevelQueue:
    """Named (priority, FIFO) queues with per-queue locks and copy-out stats."""

    def __init__(self, max_size: int = 0):
        self._q = _native.mlq().MultiLevelQueue(int(max_size))
        self._store: Dict[int, Message] = {}
        self._max_size = int(max_size)

    # ------------------------------------------------------------- admin
    def add_queue(self, name: str, max_size: int = -1) -> None:
        self._q.add_queue(name, int(max_size))

    def remove_queue(self, name: str) -> bool:
        for h in self._q.snapshot(name):
            self._store.pop(h, None)
        return self._q.remove_queue(name)

    def has_queue(self, name: str) -> bool:
        return self._q.has_queue(name)

    def queue_names(self) -> List[str]:
        return list(self._q.names())

    @property
    def native(self):
        return self._q

    # ------------------------------------------------------------- ops
    def push(self, queue_name: str, message: Message, priority: Optional[int] = None) -> None:
        prio = int(message.priority if priority is None else priority)
        self._store[message.handle] = message
        status, enq = self._q.push(queue_name, message.handle, prio)
        if status:
            self._store.pop(message.handle, None)
            raise _STATUS_ERR[status]()
        message.enqueued_at = enq

    def push_many(self, queue_names: Sequence[str], messages: Sequence[Message]) -> List[Optional[QueueError]]:
        """Batch push; returns a per-message error (None on success)."""
        if not messages:
            return []
        names = sorted(set(queue_names))
        idx = {n: i for i, n in enumerate(names)}
        qidx = np.fromiter((idx[n] for n in queue_names), dtype=np.int32, count=len(messages))
        handles = np.fromiter((m.handle for m in messages), dtype=np.int64, count=len(messages))
        prios = np.fromiter((m.priority for m in messages), dtype=np.int32, count=len(messages))
        store = self._store
        for m in messages:
            store[m.handle] = m
        status = self._q.push_batch(names, qidx, handles, prios)
        out: List[Optional[QueueError]] = []
        now = _native.mlq().mono_ns()
        for m, s in zip(messages, status):
            if s:
                store.pop(m.handle, None)
                out.append(_STATUS_ERR[s]())
            else:
                m.enqueued_at = now
                out.append(None)
        return out

    def pop(self, queue_name: str) -> Message:
        status, h, _prio, _enq = self._q.pop(queue_name)
        if status:
            raise QueueEmpty()
        return self._store.pop(h)

    def pop_batch(self, queue_name: str, count: int) -> List[Message]:
        store = self._store
        return [store.pop(h) for h in self._q.pop_batch(queue_name, int(count))]

    def pop_tiers(self, tiers: Sequence[str], count: int, aging_ns: Sequence[int],
                  budget: Sequence[int], lifo_ns: Optional[Sequence[int]] = None,
                  skip: Optional[np.ndarray] = None) -> Tuple[List[Message], np.ndarray, np.ndarray]:
        """Dispatcher pop: strict priority with aging + per-tier budgets.
        ``budget[i] < 0`` means unlimited.  ``lifo_ns`` (optional): adaptive
        LIFO thresholds per tier (serve newest while the head is older).
        ``skip`` (optional int64 handles): requests to pass over, left queued
        in place."""
        args = (list(tiers), int(count), list(aging_ns), list(budget), list(lifo_ns or []))
        hs, tier_idx, enq = (self._q.pop_tiers(*args, skip) if skip is not None and len(skip)
                             else self._q.pop_tiers(*args))
        store = self._store
        return [store.pop(int(h)) for h in hs], tier_idx, enq

    def peek(self, queue_name: str) -> Message:
        status, h, _p, _e = self._q.peek(queue_name)
        if status:
            raise QueueEmpty()
        return self._store[h]

    def size(self, queue_name: str) -> int:
        n = self._q.size(queue_name)
        if n < 0:
            raise QueueNotFound()
        return n

    def total_size(self) -> int:
        return self._q.total_size()

    def remove(self, queue_name: str, message: Message) -> bool:
        ok = self._q.remove(queue_name, message.handle)
        if ok:
            self._store.pop(message.handle, None)
        return ok

    def messages(self, queue_name: str) -> List[Message]:
        store = self._store
        return [store[h] for h in self._q.snapshot(queue_name) if h in store]

    def find(self, message_id: str) -> Optional[Message]:
        for m in list(self._store.values()):
            if m.id == message_id:
                return m
        return None

    # ------------------------------------------------------------- stats
    def get_stats(self, queue_name: str) -> QueueStats:
        d = self._q.stats(queue_name)
        if d is None:
            raise QueueNotFound()
        return QueueStats(d["pending"], d["processing"], d["completed"], d["failed"],
                          d["total_wait_ns"], d["total_process_ns"],
                          mono_to_wall_ns(d["last_update_ns"]) if d["last_update_ns"] else 0)

    def raw_stats(self, queue_name: str) -> Optional[dict]:
        return self._q.stats(queue_name)

    def get_all_stats(self) -> Dict[str, QueueStats]:
        return {n: self.get_stats(n) for n in self._q.names()}

    def complete_message(self, queue_name: str, process_ns: int = 0) -> None:
        self._q.complete(queue_name, int(process_ns))

    def fail_message(self, queue_name: str) -> None:
        self._q.fail(queue_name)

    def unprocess(self, queue_name: str) -> None:
        self._q.unprocess(queue_name)

    def clear(self, queue_name: str) -> None:
        for h in self._q.snapshot(queue_name):
            self._store.pop(h, None)
        self._q.clear(queue_name)
