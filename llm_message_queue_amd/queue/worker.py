"""Worker + backoff strategies (components C5, C6).

Reference `internal/priorityqueue/worker.go`:
  * every ``process_interval`` the worker batch-pops up to ``max_batch_size``
    messages and runs each under a ``max_concurrent`` semaphore (`:109-159`);
  * each message runs with a deadline of ``msg.timeout`` (`:162-188`);
  * success -> ``complete_message``; failure -> retry while
    ``retry_count < backoff.max_retries()`` else ``fail_message``
    (`:191-239`).

Fixes:
  * D15: retries go through the DelayedQueue at ``now + backoff`` instead of
    being re-pushed immediately, and exhausted messages go to the DLQ;
  * D22: ``get_metrics`` returns a copy; the retry counter is incremented;
  * D16: a zero timeout means the 30 s default, never an expired context;
  * the tick loop drains back-to-back full batches instead of sleeping a full
    tick between them (the reference caps a worker at batch/tick = 100 msg/s).
"""
from __future__ import annotations

import dataclasses
import threading
import time
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from typing import Callable, Optional

from ..models.message import DEFAULT_TIMEOUT_NS, Message, MessageStatus
from ..utils.logging import get_logger


# ----------------------------------------------------------------------------- context
class DeadlineExceeded(TimeoutError):
    def __str__(self) -> str:
        return "context deadline exceeded"


class Cancelled(Exception):
    def __str__(self) -> str:
        return "context canceled"


class Context:
    """Minimal ``context.Context``: deadline + cancellation."""

    __slots__ = ("deadline", "_cancel")

    def __init__(self, deadline_mono_ns: Optional[int], cancel: threading.Event):
        self.deadline = deadline_mono_ns
        self._cancel = cancel

    def done(self) -> bool:
        return self._cancel.is_set() or (self.deadline is not None and time.monotonic_ns() >= self.deadline)

    def err(self) -> Optional[Exception]:
        if self._cancel.is_set():
            return Cancelled()
        if self.deadline is not None and time.monotonic_ns() >= self.deadline:
            return DeadlineExceeded()
        return None

    def remaining_s(self) -> Optional[float]:
        if self.deadline is None:
            return None
        return max(0.0, (self.deadline - time.monotonic_ns()) / 1e9)


ProcessFunc = Callable[[Context, Message], Optional[BaseException]]


# ----------------------------------------------------------------------------- backoff
class BackoffStrategy:
    def next_backoff(self, retry_count: int) -> int:
        raise NotImplementedError

    def max_retries(self) -> int:
        raise NotImplementedError


class ExponentialBackoff(BackoffStrategy):
    """``min(initial * factor^(n-1), max)`` (`worker.go:258-294`)."""

    def __init__(self, initial_ns: int, max_ns: int, factor: float, max_retries: int):
        self.initial = int(initial_ns)
        self.max = int(max_ns)
        self.factor = float(factor)
        self._max_retries = int(max_retries)

    def next_backoff(self, retry_count: int) -> int:
        if retry_count <= 0:
            return self.initial
        b = float(self.initial)
        for _ in range(1, retry_count):
            b *= self.factor
            if b > self.max:
                break
        return self.max if b > self.max else int(b)

    def max_retries(self) -> int:
        return self._max_retries


class FixedBackoff(BackoffStrategy):
    """`worker.go:297-315`."""

    def __init__(self, backoff_ns: int, max_retries: int):
        self.backoff = int(backoff_ns)
        self._max_retries = int(max_retries)

    def next_backoff(self, retry_count: int) -> int:
        return self.backoff

    def max_retries(self) -> int:
        return self._max_retries


# ----------------------------------------------------------------------------- worker
@dataclass
class WorkerMetrics:
    """`worker.go:42-49` (durations in ns)."""
    processed_count: int = 0
    success_count: int = 0
    failure_count: int = 0
    retry_count: int = 0
    dead_lettered: int = 0
    total_process_time: int = 0
    last_process_time: int = 0

    def to_dict(self) -> dict:
        return {"ProcessedCount": self.processed_count, "SuccessCount": self.success_count,
                "FailureCount": self.failure_count, "RetryCount": self.retry_count,
                "DeadLettered": self.dead_lettered,
                "TotalProcessTime": self.total_process_time,
                "LastProcessTime": self.last_process_time}


@dataclass
class WorkerConfig:
    id: str
    queue_name: str
    max_batch_size: int = 10
    process_interval: int = 100_000_000
    max_concurrent: int = 50
    backoff_strategy: Optional[BackoffStrategy] = None


class Worker:
    def __init__(self, config: WorkerConfig, queue_manager, process_func: ProcessFunc,
                 logger=None, delayed_queue=None, dead_letter_queue=None):
        self.id = config.id
        self.config = config
        self.queue_manager = queue_manager
        self.queue_name = config.queue_name
        self.process_func = process_func
        self.backoff = config.backoff_strategy or ExponentialBackoff(1_000_000_000, 60_000_000_000, 2.0, 3)
        self.logger = (logger or get_logger("worker")).with_fields(worker_id=config.id)
        self.delayed_queue = delayed_queue
        self.dead_letter_queue = dead_letter_queue
        self._metrics = WorkerMetrics()
        self._mlock = threading.Lock()
        self._cancel = threading.Event()
        self._sem = threading.BoundedSemaphore(max(1, config.max_concurrent))
        self._pool = ThreadPoolExecutor(max_workers=max(1, config.max_concurrent),
                                        thread_name_prefix=f"w-{config.id}")
        self._thread: Optional[threading.Thread] = None
        self._inflight = 0
        self._idle = threading.Condition(self._mlock)

    # ------------------------------------------------------------------ lifecycle
    def start(self) -> None:
        self.logger.info("Starting worker", queue=self.queue_name,
                         max_concurrent=self.config.max_concurrent,
                         max_batch_size=self.config.max_batch_size)
        self._thread = threading.Thread(target=self._loop, name=f"worker-{self.id}", daemon=True)
        self._thread.start()

    def stop(self, wait: bool = True) -> None:
        self.logger.info("Stopping worker")
        self._cancel.set()
        if self._thread is not None:
            self._thread.join(timeout=10)
        if wait:
            with self._idle:
                self._idle.wait_for(lambda: self._inflight == 0, timeout=10)
        self._pool.shutdown(wait=wait)

    def get_metrics(self) -> WorkerMetrics:
        with self._mlock:
            return dataclasses.replace(self._metrics)

    # ------------------------------------------------------------------ loop
    def _loop(self) -> None:
        interval = max(self.config.process_interval, 100_000) / 1e9
        while not self._cancel.is_set():
            n = self.process_batch()
            # a full batch means more work is likely waiting: go again now
            if n >= self.config.max_batch_size:
                continue
            if self._cancel.wait(interval):
                break

    def process_batch(self) -> int:
        try:
            msgs = self.queue_manager.batch_pop_messages(self.queue_name, self.config.max_batch_size)
        except Exception as e:
            self.logger.error("Failed to pop messages from queue", error=str(e))
            return 0
        for m in msgs:
            while not self._sem.acquire(timeout=0.1):
                if self._cancel.is_set():
                    # shutting down: put it back so it is not lost
                    self.queue_manager.requeue_after_failure(self.queue_name, m)
                    break
            else:
                with self._mlock:
                    self._inflight += 1
                self._pool.submit(self._run_one, m)
        return len(msgs)

    def _run_one(self, m: Message) -> None:
        try:
            self.process_message(m)
        finally:
            self._sem.release()
            with self._idle:
                self._inflight -= 1
                if self._inflight == 0:
                    self._idle.notify_all()

    def process_message(self, message: Message) -> None:
        start = time.monotonic_ns()
        timeout = message.timeout if message.timeout > 0 else DEFAULT_TIMEOUT_NS
        ctx = Context(start + timeout, self._cancel)
        message.status = MessageStatus.PROCESSING
        try:
            err = self.process_func(ctx, message)
        except Exception as e:  # a raising ProcessFunc == returning an error
            err = e
        elapsed = time.monotonic_ns() - start
        self._update_metrics(err, elapsed)
        if err:
            self.handle_failure(message, err)
        else:
            self.handle_success(message, elapsed)

    def handle_success(self, message: Message, elapsed_ns: int) -> None:
        message.status = MessageStatus.COMPLETED
        message.completed_at = time.time_ns()
        self.queue_manager.complete_message(self.queue_name, message.id, elapsed_ns, message.priority)

    def handle_failure(self, message: Message, err: BaseException) -> None:
        self.logger.warning("Failed to process message", message_id=message.id, error=str(err),
                            retry_count=message.retry_count)
        if message.retry_count < self.backoff.max_retries():
            message.retry_count += 1
            backoff = self.backoff.next_backoff(message.retry_count)
            ready = time.time_ns() + backoff
            message.scheduled_at = ready
            message.status = MessageStatus.PENDING
            with self._mlock:
                self._metrics.retry_count += 1
            self.queue_manager.mlq.unprocess(self.queue_name)
            if self.delayed_queue is not None:
                qm, qn = self.queue_manager, self.queue_name
                self.delayed_queue.schedule(message, ready,
                                            target=lambda m, qm=qm, qn=qn: qm.push_message(qn, m))
            else:
                self.queue_manager.push_message(self.queue_name, message)
        else:
            message.status = MessageStatus.FAILED
            self.queue_manager.fail_message(self.queue_name, message.id, err, message.priority)
            if self.dead_letter_queue is not None:
                try:
                    self.dead_letter_queue.push(message, str(err), self.queue_name)
                    with self._mlock:
                        self._metrics.dead_lettered += 1
                except Exception as e:
                    self.logger.error("Dead letter queue full", message_id=message.id, error=str(e))

    def _update_metrics(self, err, elapsed_ns: int) -> None:
        with self._mlock:
            m = self._metrics
            m.processed_count += 1
            m.total_process_time += elapsed_ns
            m.last_process_time = elapsed_ns
            if err:
                m.failure_count += 1
            else:
                m.success_count += 1
