"""QueueManager (component C4): named queues + rules + metrics + monitor loop.

Reference: `internal/priorityqueue/queue_manager.go`.
  * ``create_queue`` is idempotent; ``max_size<=0`` falls back to
    ``default_max_size`` (`:170-188`).
  * ``push_message`` applies the FIRST matching priority-adjust rule
    (`:451-466`) then pushes (`:210-243`).
  * ``batch_push_messages``/``batch_pop_messages`` (`:246-367`).
  * monitor loop refreshes gauges and logs threshold breaches every
    ``monitor_interval``; cleanup every ``cleanup_interval`` (`:469-553`).
    Here cleanup really expires messages older than ``max_retention_period``.

Fixes: metrics live in one shared registry labelled by manager (D5); the
complete/fail series carry the real priority (D23); a ``dead_letter`` hook
receives messages that exhaust retries (D15).
"""
from __future__ import annotations

import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence

from ..models.message import Message, QueueStats, priority_name, now_ns
from ..utils.logging import get_logger
from ..utils.metrics import QueueMetrics, default_metrics
from .core import MultiLevelQueue, QueueError, QueueFull, QueueNotFound


@dataclass
class PriorityAdjustRule:
    """`queue_manager.go:39-43`."""
    condition: Callable[[Message], bool]
    new_priority: int
    description: str = ""


@dataclass
class QueueManagerConfig:
    """`queue_manager.go:27-36`."""
    default_max_size: int = 10000
    monitor_interval: int = 5_000_000_000
    cleanup_interval: int = 60_000_000_000
    max_retention_period: int = 24 * 3600 * 1_000_000_000
    enable_metrics: bool = True
    enable_auto_scaling: bool = True
    scaling_thresholds: Dict[str, int] = field(default_factory=dict)
    priority_adjust_rules: List[PriorityAdjustRule] = field(default_factory=list)


class QueueManager:
    def __init__(self, config: Optional[QueueManagerConfig] = None, name: str = "default",
                 metrics: Optional[QueueMetrics] = None, logger=None):
        self.config = config or QueueManagerConfig()
        self.name = name
        self.mlq = MultiLevelQueue(self.config.default_max_size)
        self._lock = threading.RLock()
        self._queues: Dict[str, int] = {}      # name -> max size
        self.metrics = (metrics or default_metrics()) if self.config.enable_metrics else None
        self.logger = logger or get_logger("queue_manager").with_fields(manager=name)
        self._stop = threading.Event()
        self._monitor: Optional[threading.Thread] = None
        self.threshold_events: List[dict] = []   # observable autoscale recommendations
        self.expired_count = 0
        # called with each message taken out of a queue other than by a pop
        # (admin delete, peer dequeue, retention cleanup): the gateway
        # releases the message's (home GPU, tier) pin here
        self.on_remove: List[Callable[[Message], None]] = []

    # ------------------------------------------------------------- lifecycle
    def start(self) -> None:
        if self._monitor is not None:
            return
        self._stop.clear()
        self._monitor = threading.Thread(target=self._monitor_loop, name=f"qm-monitor-{self.name}",
                                         daemon=True)
        self._monitor.start()

    def stop(self) -> None:
        self._stop.set()
        t = self._monitor
        if t is not None:
            t.join(timeout=5)
        self._monitor = None

    # ------------------------------------------------------------- queues
    def create_queue(self, name: str, max_size: int = 0) -> None:
        with self._lock:
            if name in self._queues:
                return
            if max_size <= 0:
                max_size = self.config.default_max_size
            self.mlq.add_queue(name, max_size)
            self._queues[name] = max_size
        self.logger.info("Created new queue", queue=name, max_size=max_size)
        if self.metrics:
            self.metrics.operations.labels(self.name, name, "create").inc()

    def delete_queue(self, name: str) -> None:
        with self._lock:
            if name not in self._queues:
                raise QueueNotFound()
            del self._queues[name]
            self.mlq.remove_queue(name)
        if self.metrics:
            self.metrics.operations.labels(self.name, name, "delete").inc()

    def has_queue(self, name: str) -> bool:
        return name in self._queues

    def queue_names(self) -> List[str]:
        return list(self._queues)

    # ------------------------------------------------------------- push/pop
    def apply_priority_rules(self, message: Message) -> None:
        for rule in self.config.priority_adjust_rules:
            try:
                hit = rule.condition(message)
            except Exception:
                hit = False
            if hit:
                old = message.priority
                message.priority = int(rule.new_priority)
                self.logger.debug("Adjusted message priority", message_id=message.id,
                                  old=old, new=message.priority, rule=rule.description)
                break

    def push_message(self, queue_name: str, message: Message) -> None:
        if queue_name not in self._queues:
            raise QueueNotFound()
        self.apply_priority_rules(message)
        if not message.queue_name:
            message.queue_name = queue_name
        self.mlq.push(queue_name, message, message.priority)
        if self.metrics:
            self.metrics.operations.labels(self.name, queue_name, "push").inc()
            self.metrics.pending.labels(self.name, queue_name, priority_name(message.priority)).inc()

    def batch_push_messages(self, queue_name: str, messages: Sequence[Message]) -> int:
        if queue_name not in self._queues:
            raise QueueNotFound()
        for m in messages:
            self.apply_priority_rules(m)
            if not m.queue_name:
                m.queue_name = queue_name
        errs = self.mlq.push_many([queue_name] * len(messages), messages)
        ok = sum(1 for e in errs if e is None)
        if self.metrics:
            for m, e in zip(messages, errs):
                if e is None:
                    self.metrics.pending.labels(self.name, queue_name, priority_name(m.priority)).inc()
            self.metrics.operations.labels(self.name, queue_name, "batch_push").inc()
        self.logger.debug("Batch pushed messages to queue", queue=queue_name,
                          total=len(messages), success=ok)
        return ok

    def push_routed(self, messages: Sequence[Message]) -> List[Optional[QueueError]]:
        """Push each message to ``message.queue_name`` (gateway ingress path)."""
        if self.config.priority_adjust_rules:
            for m in messages:
                self.apply_priority_rules(m)
        errs = self.mlq.push_many([m.queue_name for m in messages], messages)
        if self.metrics:
            # one labelled increment per (queue, priority), not per message
            cnt: Dict[tuple, int] = {}
            for m, e in zip(messages, errs):
                if e is None:
                    k = (m.queue_name, m.priority)
                    cnt[k] = cnt.get(k, 0) + 1
            pend = self.metrics.pending
            for (q, p), n in cnt.items():
                pend.labels(self.name, q, priority_name(p)).inc(n)
        return errs

    def pop_message(self, queue_name: str) -> Message:
        if queue_name not in self._queues:
            raise QueueNotFound()
        m = self.mlq.pop(queue_name)
        if self.metrics:
            self.metrics.operations.labels(self.name, queue_name, "pop").inc()
            p = priority_name(m.priority)
            self.metrics.pending.labels(self.name, queue_name, p).dec()
            self.metrics.processing.labels(self.name, queue_name, p).inc()
            self._observe_wait([m])
        return m

    def _observe_wait(self, msgs) -> None:
        """``llm_queue_messages_wait_time_seconds``: enqueue -> taken off the
        queue, per (manager, queue, priority) -- the reference's histogram,
        which its code never observed (D23)."""
        now = time.monotonic_ns()                 # enqueued_at: the queue's steady clock
        h = self.metrics.wait_time
        for m in msgs:
            if m.enqueued_at:
                h.labels(self.name, m.queue_name, priority_name(m.priority)).observe(
                    max(0, now - m.enqueued_at) / 1e9)

    def batch_pop_messages(self, queue_name: str, count: int) -> List[Message]:
        if queue_name not in self._queues:
            raise QueueNotFound()
        msgs = self.mlq.pop_batch(queue_name, count)
        if self.metrics:
            for m in msgs:
                p = priority_name(m.priority)
                self.metrics.pending.labels(self.name, queue_name, p).dec()
                self.metrics.processing.labels(self.name, queue_name, p).inc()
            self.metrics.operations.labels(self.name, queue_name, "batch_pop").inc()
            self._observe_wait(msgs)
        return msgs

    def pop_tiers(self, tiers: Sequence[str], count: int, aging_ns: Sequence[int],
                  budget: Sequence[int], lifo_ns: Optional[Sequence[int]] = None, skip=None):
        msgs, tier_idx, enq = self.mlq.pop_tiers(tiers, count, aging_ns, budget, lifo_ns, skip)
        if self.metrics and msgs:
            cnt: Dict[tuple, int] = {}
            for m in msgs:
                k = (m.queue_name, m.priority)
                cnt[k] = cnt.get(k, 0) + 1
            for (q, pr), n in cnt.items():
                p = priority_name(pr)
                self.metrics.pending.labels(self.name, q, p).dec(n)
                self.metrics.processing.labels(self.name, q, p).inc(n)
            self._observe_wait(msgs)
        return msgs, tier_idx, enq

    def peek_message(self, queue_name: str) -> Message:
        return self.mlq.peek(queue_name)

    # ------------------------------------------------------------- completion
    def complete_message(self, queue_name: str, message_id: str, processing_time_ns: int = 0,
                         priority: Optional[int] = None) -> None:
        if queue_name not in self._queues:
            return
        self.mlq.complete_message(queue_name, processing_time_ns)
        if self.metrics:
            p = priority_name(priority) if priority is not None else "unknown"
            self.metrics.processing.labels(self.name, queue_name, p).dec()
            self.metrics.completed.labels(self.name, queue_name, p).inc()
            self.metrics.process_time.labels(self.name, queue_name, p).observe(processing_time_ns / 1e9)

    def fail_message(self, queue_name: str, message_id: str, err: Optional[BaseException] = None,
                     priority: Optional[int] = None, quiet: bool = False) -> None:
        if queue_name not in self._queues:
            return
        self.mlq.fail_message(queue_name)
        if not quiet:   # bulk callers (overload shedding) log once themselves
            self.logger.warning("Failed message", queue=queue_name, message_id=message_id, error=str(err))
        if self.metrics:
            p = priority_name(priority) if priority is not None else "unknown"
            self.metrics.processing.labels(self.name, queue_name, p).dec()
            self.metrics.failed.labels(self.name, queue_name, p).inc()

    def requeue_after_failure(self, queue_name: str, message: Message) -> bool:
        """A popped message goes back (retry): push, then processing--.
        False when its tier is full (an overloaded queue): the message is
        counted failed instead, and the caller decides where it goes (the
        gateway dead-letters it) -- a retry must not raise into a serve loop."""
        try:
            self.push_message(queue_name, message)
        except QueueFull:
            self.fail_message(queue_name, message.id, None, message.priority, quiet=True)
            return False
        if queue_name in self._queues:
            self.mlq.unprocess(queue_name)
            if self.metrics:
                self.metrics.processing.labels(self.name, queue_name,
                                               priority_name(message.priority)).dec()
        return True

    # ------------------------------------------------------------- stats
    def get_queue_stats(self, queue_name: str) -> QueueStats:
        if queue_name not in self._queues:
            raise QueueNotFound()
        return self.mlq.get_stats(queue_name)

    def get_all_queue_stats(self) -> Dict[str, QueueStats]:
        return {n: self.mlq.get_stats(n) for n in list(self._queues)}

    def size(self, queue_name: str) -> int:
        return self.mlq.size(queue_name)

    def total_pending(self) -> int:
        return self.mlq.total_size()

    # ------------------------------------------------------------- monitor
    def _monitor_loop(self) -> None:
        mi = max(self.config.monitor_interval, 1_000_000) / 1e9
        ci = max(self.config.cleanup_interval, 1_000_000) / 1e9
        next_m = time.monotonic() + mi
        next_c = time.monotonic() + ci
        while not self._stop.is_set():
            now = time.monotonic()
            wait = max(0.0, min(next_m, next_c) - now)
            if self._stop.wait(wait):
                break
            now = time.monotonic()
            if now >= next_m:
                self.update_queue_metrics()
                if self.config.enable_auto_scaling:
                    self.check_queue_thresholds()
                next_m = now + mi
            if now >= next_c:
                self.cleanup_stale_messages()
                next_c = now + ci

    def update_queue_metrics(self) -> None:
        if not self.metrics:
            return
        for name in list(self._queues):
            st = self.mlq.get_stats(name)
            self.metrics.pending.labels(self.name, name, "all").set(st.pending_count)
            self.metrics.processing.labels(self.name, name, "all").set(st.processing_count)

    def check_queue_thresholds(self) -> List[dict]:
        events = []
        for name in list(self._queues):
            thr = self.config.scaling_thresholds.get(name)
            if thr is None:
                continue
            size = self.mlq.size(name)
            if size > thr:
                ev = {"queue": name, "size": size, "threshold": thr, "ts": now_ns()}
                events.append(ev)
                self.logger.info("Queue threshold exceeded, scaling up recommended", **ev)
        self.threshold_events = (self.threshold_events + events)[-100:]
        return events

    def remove_message(self, name: str, m: Message) -> bool:
        """Take one queued message out of ``name`` (not a dispatch): every
        removal path goes through here so ``on_remove`` hooks see it."""
        if not self.mlq.remove(name, m):
            return False
        for fn in self.on_remove:
            fn(m)
        return True

    def cleanup_stale_messages(self) -> int:
        """Expire pending messages older than ``max_retention_period``
        (a no-op stub in the reference, `queue_manager.go:549-553`)."""
        ret = self.config.max_retention_period
        if ret <= 0:
            return 0
        cutoff = time.monotonic_ns() - ret
        n = 0
        for name in list(self._queues):
            for m in self.mlq.messages(name):
                if m.enqueued_at and m.enqueued_at < cutoff and self.remove_message(name, m):
                    m.status = "timeout"
                    n += 1
        self.expired_count += n
        return n
