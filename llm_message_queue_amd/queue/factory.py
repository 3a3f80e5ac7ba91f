"""QueueFactory (component C7).

Reference `internal/priorityqueue/queue_factory.go`:
  * ``create_queue_manager(name, type)`` is idempotent and starts the manager
    (`:43-74`);
  * ``create_workers(queue, count, fn)`` builds workers with exponential
    backoff from ``queue.retry`` and IDs ``"<queue>-worker-<i>"``
    (`:86-134`, `:236-238`);
  * ``priority`` typed managers get the VIP->High and >10000-byte->Low rules
    (`:211-233`).
Fixes: the factory owns ONE DelayedQueue and ONE DeadLetterQueue and wires
every worker to them (retries -> delayed, exhausted -> DLQ; D15).  The
reference's "delayed"/"dead_letter" typed managers were plain managers; they
stay plain managers here too (for API compatibility), while the real
delayed/DLQ machinery is ``factory.delayed_queue`` / ``factory.dead_letter_queue``.
"""
from __future__ import annotations

import threading
from typing import Dict, List, Optional

from ..models.message import PRIORITY_HIGH, PRIORITY_LOW
from ..utils.config import QueueConfig
from ..utils.logging import get_logger
from ..utils.metrics import QueueMetrics, default_metrics
from .dead_letter import DeadLetterQueue
from .delayed import DelayedQueue
from .manager import PriorityAdjustRule, QueueManager, QueueManagerConfig
from .worker import ExponentialBackoff, ProcessFunc, Worker, WorkerConfig, WorkerMetrics


class QueueType:
    STANDARD = "standard"
    DELAYED = "delayed"
    DEAD_LETTER = "dead_letter"
    PRIORITY = "priority"
    ALL = ("standard", "delayed", "dead_letter", "priority")


def default_priority_rules() -> List[PriorityAdjustRule]:
    """`queue_factory.go:211-233`."""
    return [
        PriorityAdjustRule(lambda m: "vip_user" in m.metadata, PRIORITY_HIGH,
                           "VIP user messages are promoted"),
        PriorityAdjustRule(lambda m: len(m.content.encode("utf-8")) > 10000, PRIORITY_LOW,
                           "very long messages are demoted"),
    ]


class QueueFactory:
    def __init__(self, config: Optional[QueueConfig] = None, logger=None,
                 metrics: Optional[QueueMetrics] = None):
        self.config = config or QueueConfig()
        self.logger = logger or get_logger("queue_factory")
        self.metrics = metrics or (default_metrics() if self.config.enable_metrics else None)
        self._managers: Dict[str, QueueManager] = {}
        self._types: Dict[str, str] = {}
        self._workers: Dict[str, List[Worker]] = {}
        self._lock = threading.RLock()
        self.delayed_queue = DelayedQueue(logger=self.logger.with_fields(component="delayed"))
        self.delayed_queue.start()
        self.dead_letter_queue = DeadLetterQueue(self.config.dead_letter_max_size,
                                                 logger=self.logger.with_fields(component="dlq"))

    def create_queue_manager(self, name: str, queue_type: str = QueueType.STANDARD) -> QueueManager:
        with self._lock:
            mgr = self._managers.get(name)
            if mgr is not None:
                return mgr
            mgr = QueueManager(self._manager_config(queue_type), name=name, metrics=self.metrics,
                               logger=self.logger.with_fields(component="queue_manager", queue=name,
                                                              type=queue_type))
            self._managers[name] = mgr
            self._types[name] = queue_type
            mgr.start()
        self.logger.info("Created queue manager", name=name, type=queue_type)
        return mgr

    def get_queue_manager(self, name: str) -> Optional[QueueManager]:
        with self._lock:
            return self._managers.get(name)

    def managers(self) -> Dict[str, QueueManager]:
        with self._lock:
            return dict(self._managers)

    def manager_type(self, name: str) -> Optional[str]:
        return self._types.get(name)

    def create_workers(self, manager_name: str, count: int, process_func: ProcessFunc,
                       queue_name: Optional[str] = None) -> Optional[List[Worker]]:
        """Workers drain ``queue_name`` (default: the manager's own name, as in
        the reference) of manager ``manager_name``."""
        with self._lock:
            mgr = self._managers.get(manager_name)
            if mgr is None:
                self.logger.error("Cannot create workers for non-existent queue", queue=manager_name)
                return None
            qn = queue_name or manager_name
            mgr.create_queue(qn)
            w = self.config.worker
            r = self.config.retry
            start = len(self._workers.get(manager_name, []))
            out = []
            for i in range(count):
                cfg = WorkerConfig(id=self.generate_worker_id(qn, start + i), queue_name=qn,
                                   max_batch_size=w.max_batch_size,
                                   process_interval=w.process_interval,
                                   max_concurrent=w.max_concurrent,
                                   backoff_strategy=ExponentialBackoff(
                                       r.initial_backoff, r.max_backoff, r.factor, r.max_retries))
                wk = Worker(cfg, mgr, process_func,
                            logger=self.logger.with_fields(component="worker", queue=qn),
                            delayed_queue=self.delayed_queue,
                            dead_letter_queue=self.dead_letter_queue)
                out.append(wk)
                wk.start()
            self._workers.setdefault(manager_name, []).extend(out)
        self.logger.info("Created workers for queue", queue=qn, count=count)
        return out

    def stop_all(self) -> None:
        with self._lock:
            for ws in self._workers.values():
                for w in ws:
                    w.stop()
            for m in self._managers.values():
                m.stop()
            self._workers = {}
            self._managers = {}
            self._types = {}
        self.delayed_queue.stop()

    def close(self) -> None:
        self.stop_all()
        self.delayed_queue.close()

    def get_worker_stats(self) -> Dict[str, List[WorkerMetrics]]:
        with self._lock:
            return {q: [w.get_metrics() for w in ws] for q, ws in self._workers.items()}

    def _manager_config(self, queue_type: str) -> QueueManagerConfig:
        c = self.config
        cfg = QueueManagerConfig(
            default_max_size=c.default_max_size, monitor_interval=c.monitor_interval,
            cleanup_interval=c.cleanup_interval, max_retention_period=c.max_retention_period,
            enable_metrics=c.enable_metrics, enable_auto_scaling=c.enable_auto_scaling,
            scaling_thresholds=dict(c.scaling_thresholds))
        if queue_type == QueueType.PRIORITY:
            cfg.priority_adjust_rules = default_priority_rules()
        return cfg

    @staticmethod
    def generate_worker_id(queue_name: str, index: int) -> str:
        return f"{queue_name}-worker-{index}"
