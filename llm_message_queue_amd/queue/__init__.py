"""Queueing core: MultiLevelQueue (C3/N6), QueueManager (C4), Worker (C5/C6),
QueueFactory (C7), DelayedQueue (C8/N7), DeadLetterQueue (C9)."""
from .core import (IndexOutOfRange, MultiLevelQueue, QueueEmpty, QueueError, QueueFull,
                   QueueNotFound, ErrIndexOutOfRange, ErrQueueEmpty, ErrQueueFull,
                   ErrQueueNotFound)
from .dead_letter import DeadLetterItem, DeadLetterQueue
from .delayed import DelayedQueue
from .factory import QueueFactory, QueueType, default_priority_rules
from .manager import PriorityAdjustRule, QueueManager, QueueManagerConfig
from .worker import (Context, DeadlineExceeded, ExponentialBackoff, FixedBackoff, Worker,
                     WorkerConfig, WorkerMetrics)

__all__ = [n for n in dir() if not n.startswith("_")]
