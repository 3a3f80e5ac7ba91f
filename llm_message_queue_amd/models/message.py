"""Domain objects: priorities, messages, conversations (component C1).

Parity notes (reference `pkg/models/message.go`):
  * ``Priority`` is a plain int where LOWER is more urgent: realtime=1, high=2,
    normal=3, low=4 (`message.go:15-22`).  ``priority_name`` reproduces
    ``Priority.String()`` (`message.go:24-37`), which maps every other value to
    ``"unknown"``.
  * JSON priority is emitted as an int.  On input we ALSO accept the strings the
    reference docs use (`README.md:180-186`, `docs/api.md:55-66`) -- the Go code
    rejects them with a 400 (defect D4 in SURVEY.md §8).
  * ``new_message`` defaults MaxRetries=3 / Timeout=30 s (`message.go:76-91`).
    REST-bound messages in the reference get Timeout=0 (defect D16); here the
    timeout always defaults to 30 s.
"""
from __future__ import annotations

import datetime as _dt
import itertools
import math
import re
import time
import uuid
from typing import Any, Dict, List, Optional

# --------------------------------------------------------------------------- priority
PRIORITY_REALTIME = 1
PRIORITY_HIGH = 2
PRIORITY_NORMAL = 3
PRIORITY_LOW = 4
PRIORITY_LEVELS = (PRIORITY_REALTIME, PRIORITY_HIGH, PRIORITY_NORMAL, PRIORITY_LOW)
LEVEL_NAMES = ("realtime", "high", "normal", "low")

_NAME_BY_PRIO = {1: "realtime", 2: "high", 3: "normal", 4: "low"}
_PRIO_BY_NAME = {
    "realtime": 1, "urgent": 1,  # "urgent" is the docs' realtime alias
    "high": 2, "normal": 3, "medium": 3, "low": 4,
}


class Priority(int):
    """Integer priority with the reference's ``String()`` naming.

    Subclassing int keeps arithmetic/comparison/JSON behaviour identical to the
    Go ``type Priority int``.
    """

    REALTIME = PRIORITY_REALTIME
    HIGH = PRIORITY_HIGH
    NORMAL = PRIORITY_NORMAL
    LOW = PRIORITY_LOW

    def __str__(self) -> str:  # Priority.String()
        return priority_name(int(self))

    def __repr__(self) -> str:
        return f"Priority({int(self)}:{priority_name(int(self))})"


def priority_name(p: int) -> str:
    """``Priority.String()`` -- queue names used everywhere as ``fmt.Sprint(p)``."""
    return _NAME_BY_PRIO.get(int(p), "unknown")


class PriorityParseError(ValueError):
    pass


_ASCII_WS = " \t\n\r\x0b\x0c"
_INT_TEXT = re.compile(r"[+-]?[0-9]+\Z")


def parse_priority(value: Any, default: int = 0) -> int:
    """Accept an integral number 0..4 (0 = let the preprocessor decide), a
    decimal string of one, or a level name (case-insensitive, ASCII-trimmed;
    ``urgent`` = realtime, ``medium`` = normal).  Anything else raises.  The
    C++ front door applies the same rule (``csrc/ingress/http_ingress.cpp:
    priority_from_string``), so both front doors accept and assign alike."""
    if value is None:
        return default
    if isinstance(value, bool):
        raise PriorityParseError(f"invalid priority {value!r}")
    if isinstance(value, float):
        if not math.isfinite(value) or value != int(value):
            raise PriorityParseError(f"invalid priority {value!r}")
        value = int(value)
    if isinstance(value, int):
        if not 0 <= value <= PRIORITY_LOW:
            raise PriorityParseError(f"invalid priority {value!r}")
        return int(value)
    if isinstance(value, str):
        s = value.strip(_ASCII_WS).lower()
        if s in _PRIO_BY_NAME:
            return _PRIO_BY_NAME[s]
        if _INT_TEXT.match(s) and len(s.lstrip("+-").lstrip("0")) <= 1:
            return parse_priority(int(s))
        raise PriorityParseError(f"invalid priority {value!r}")
    raise PriorityParseError(f"invalid priority {value!r}")


def level_priority_from_name(name: str) -> Optional[int]:
    """Map ``realtime|high|normal|low`` (any case) to its int, else None."""
    return {"realtime": 1, "high": 2, "normal": 3, "low": 4}.get(str(name).lower())


# --------------------------------------------------------------------------- enums
class MessageStatus:
    PENDING = "pending"
    PROCESSING = "processing"
    COMPLETED = "completed"
    FAILED = "failed"
    TIMEOUT = "timeout"
    CANCELLED = "cancelled"      # DELETE /api/v1/messages/{id} aborted it in flight
    ALL = ("pending", "processing", "completed", "failed", "timeout", "cancelled")


class ConversationState:
    ACTIVE = "active"
    INACTIVE = "inactive"
    COMPLETED = "completed"
    ARCHIVED = "archived"
    ALL = ("active", "inactive", "completed", "archived")


class ConversationNotFound(KeyError):
    """``ErrConversationNotFound`` (`message.go:11-13`)."""

    def __str__(self) -> str:  # KeyError quotes its arg; keep the Go text
        return "conversation not found"


# --------------------------------------------------------------------------- time helpers
_EPOCH = _dt.datetime(1970, 1, 1, tzinfo=_dt.timezone.utc)
GO_ZERO_TIME = "0001-01-01T00:00:00Z"
DEFAULT_TIMEOUT_NS = 30 * 1_000_000_000
DEFAULT_MAX_RETRIES = 3


def now_ns() -> int:
    return time.time_ns()


def format_time(ns: Optional[int]) -> Optional[str]:
    """RFC3339Nano in UTC (Go's ``time.Time`` JSON encoding)."""
    if ns is None:
        return None
    if ns == 0:
        return GO_ZERO_TIME
    sec, rem = divmod(int(ns), 1_000_000_000)
    t = _dt.datetime.fromtimestamp(sec, tz=_dt.timezone.utc)
    frac = f".{rem:09d}".rstrip("0") if rem else ""
    if frac == ".":
        frac = ""
    return t.strftime("%Y-%m-%dT%H:%M:%S") + frac + "Z"


def parse_time(value: Any) -> Optional[int]:
    """Parse RFC3339 / epoch-ns into ns since epoch; None passes through."""
    if value is None or value == "":
        return None
    if isinstance(value, (int, float)):
        return int(value)
    s = str(value).strip()
    if s.startswith("0001-01-01"):
        return 0
    frac_ns = 0
    main = s
    tz = "+00:00"
    if s.endswith("Z"):
        main = s[:-1]
    else:
        for sep in ("+", "-"):
            idx = s.rfind(sep)
            if idx > 10:
                main, tz = s[:idx], s[idx:]
                break
    if "." in main:
        main, frac = main.split(".", 1)
        frac_ns = int((frac + "000000000")[:9])
    t = _dt.datetime.fromisoformat(main + tz)
    return int((t - _EPOCH).total_seconds()) * 1_000_000_000 + frac_ns


# --------------------------------------------------------------------------- message
_handle_counter = itertools.count(1)


class Message:
    """A queued LLM request (`message.go:58-74`).

    ``handle`` is a process-local integer id used by the native queue core
    (the C++ rings carry handles, never Python objects).
    """

    __slots__ = (
        "id", "conversation_id", "user_id", "content", "priority", "status",
        "queue_name", "retry_count", "max_retries", "timeout", "created_at",
        "updated_at", "scheduled_at", "completed_at", "metadata", "handle",
        "enqueued_at", "dispatched_at", "arrival_ns", "prompt_ids", "endpoint_id", "tier", "pin_key",
        "ingest_ns", "popped_ns", "recv_ns", "lc",
    )

    def __init__(self, id: str = "", conversation_id: str = "", user_id: str = "",
                 content: str = "", priority: int = 0, status: str = MessageStatus.PENDING,
                 queue_name: str = "", retry_count: int = 0,
                 max_retries: int = DEFAULT_MAX_RETRIES, timeout: int = DEFAULT_TIMEOUT_NS,
                 created_at: int = 0, updated_at: int = 0,
                 scheduled_at: Optional[int] = None, completed_at: Optional[int] = None,
                 metadata: Optional[Dict[str, Any]] = None):
        self.id = id
        self.conversation_id = conversation_id
        self.user_id = user_id
        self.content = content
        self.priority = int(priority)
        self.status = status
        self.queue_name = queue_name
        self.retry_count = int(retry_count)
        self.max_retries = int(max_retries)
        self.timeout = int(timeout)
        self.created_at = int(created_at)
        self.updated_at = int(updated_at)
        self.scheduled_at = scheduled_at
        self.completed_at = completed_at
        self.metadata = metadata if metadata is not None else {}
        self.handle = next(_handle_counter)
        self.enqueued_at = 0      # ns, set by the queue on push
        self.dispatched_at = 0    # ns, set by the dispatcher
        self.arrival_ns = 0       # ns, set by ingress (request received)
        self.prompt_ids = None    # token ids from the GPU tokenizer (backend prompt)
        self.endpoint_id = ""     # backend chosen at dispatch
        self.tier = -1            # tier index at dispatch
        self.pin_key = -1         # (home GPU, tier) the queued message is counted under (gateway pins)
        self.ingest_ns = 0        # ns, taken from the gateway inbox into a preprocess batch
        self.popped_ns = 0        # ns, popped from its queue by a dispatch decision
        self.recv_ns = 0          # ns, handed to this process's gateway (Gateway.submit)
        self.lc = 0               # lifecycle state at the origin router (gateway.request_table)

    # -- JSON ------------------------------------------------------------------
    def to_dict(self) -> Dict[str, Any]:
        return {
            "id": self.id,
            "conversation_id": self.conversation_id,
            "user_id": self.user_id,
            "content": self.content,
            "priority": int(self.priority),
            "status": self.status,
            "queue_name": self.queue_name,
            "retry_count": self.retry_count,
            "max_retries": self.max_retries,
            "timeout": self.timeout,
            "created_at": format_time(self.created_at),
            "updated_at": format_time(self.updated_at),
            "scheduled_at": format_time(self.scheduled_at),
            "completed_at": format_time(self.completed_at),
            "metadata": self.metadata,
        }

    @classmethod
    def from_dict(cls, d: Dict[str, Any], *, default_timeout_ns: int = DEFAULT_TIMEOUT_NS) -> "Message":
        """Bind a JSON body.  Raises ``PriorityParseError``/``ValueError`` on bad input."""
        if not isinstance(d, dict):
            raise ValueError("message body must be a JSON object")
        md = d.get("metadata")
        if md is not None and not isinstance(md, dict):
            raise ValueError("metadata must be an object")
        timeout = d.get("timeout")
        if timeout in (None, 0):
            timeout = default_timeout_ns
        elif isinstance(timeout, str):
            from ..utils.duration import parse_duration_ns
            timeout = parse_duration_ns(timeout)
        max_retries = d.get("max_retries")
        m = cls(
            id=str(d.get("id") or ""),
            conversation_id=str(d.get("conversation_id") or ""),
            user_id=str(d.get("user_id") or ""),
            content=str(d.get("content") or ""),
            priority=parse_priority(d.get("priority"), 0),
            status=str(d.get("status") or MessageStatus.PENDING),
            queue_name=str(d.get("queue_name") or ""),
            retry_count=int(d.get("retry_count") or 0),
            max_retries=DEFAULT_MAX_RETRIES if max_retries in (None, 0) else int(max_retries),
            timeout=int(timeout),
            created_at=parse_time(d.get("created_at")) or 0,
            updated_at=parse_time(d.get("updated_at")) or 0,
            scheduled_at=parse_time(d.get("scheduled_at")),
            completed_at=parse_time(d.get("completed_at")),
            metadata=dict(md) if md else {},
        )
        return m

    def copy(self) -> "Message":
        m = Message(self.id, self.conversation_id, self.user_id, self.content, self.priority,
                    self.status, self.queue_name, self.retry_count, self.max_retries,
                    self.timeout, self.created_at, self.updated_at, self.scheduled_at,
                    self.completed_at, dict(self.metadata))
        return m

    def __repr__(self) -> str:
        return (f"Message(id={self.id!r}, prio={self.priority}, queue={self.queue_name!r}, "
                f"status={self.status!r}, retry={self.retry_count})")


def new_message(conversation_id: str, user_id: str, content: str, priority: int) -> Message:
    """``NewMessage`` (`message.go:76-91`)."""
    t = now_ns()
    return Message(id=str(uuid.uuid4()), conversation_id=conversation_id, user_id=user_id,
                   content=content, priority=priority, status=MessageStatus.PENDING,
                   retry_count=0, max_retries=DEFAULT_MAX_RETRIES, timeout=DEFAULT_TIMEOUT_NS,
                   created_at=t, updated_at=t, metadata={})


# --------------------------------------------------------------------------- conversation
class Conversation:
    """`message.go:93-109`, plus the summary state produced by the
    ``context_summarise`` kernel (N5)."""

    __slots__ = (
        "id", "user_id", "title", "context", "status", "state", "priority",
        "message_count", "last_activity", "last_active_time", "created_at",
        "updated_at", "completed_at", "messages", "metadata", "summary_vec",
        "summary_tokens", "evicted_count", "home_gpu",
    )

    def __init__(self, id: str, user_id: str = "", *, created_at: Optional[int] = None,
                 state: str = ConversationState.ACTIVE, metadata: Optional[Dict[str, Any]] = None):
        t = now_ns() if created_at is None else created_at
        self.id = id
        self.user_id = user_id
        self.title = ""
        self.context = ""
        self.status = ""
        self.state = state
        self.priority = 0
        self.message_count = 0
        self.last_activity = t
        self.last_active_time = t
        self.created_at = t
        self.updated_at = t
        self.completed_at = 0
        self.messages: List[Message] = []
        self.metadata: Dict[str, Any] = metadata if metadata is not None else {}
        self.summary_vec = None        # list[float] | None  (N5 output)
        self.summary_tokens: List[int] = []  # salient token hashes (N5 output)
        self.evicted_count = 0
        self.home_gpu = -1             # KV-residency hint (sticky routing)

    def to_dict(self, include_messages: bool = True) -> Dict[str, Any]:
        d = {
            "id": self.id,
            "user_id": self.user_id,
            "title": self.title,
            "context": self.context,
            "status": self.status,
            "state": self.state,
            "priority": int(self.priority),
            "message_count": self.message_count,
            "last_activity": format_time(self.last_activity),
            "last_active_time": format_time(self.last_active_time),
            "created_at": format_time(self.created_at),
            "updated_at": format_time(self.updated_at),
            "completed_at": format_time(self.completed_at),
            "messages": [m.to_dict() for m in self.messages] if include_messages else [],
            "metadata": self.metadata,
        }
        if self.summary_tokens or self.summary_vec is not None:
            d["summary"] = {"evicted_messages": self.evicted_count,
                            "salient_tokens": list(self.summary_tokens)}
        if self.home_gpu >= 0:
            d["home_gpu"] = self.home_gpu
        return d

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "Conversation":
        c = cls(str(d.get("id", "")), str(d.get("user_id", "")),
                created_at=parse_time(d.get("created_at")) or 0,
                state=str(d.get("state") or ConversationState.ACTIVE),
                metadata=dict(d.get("metadata") or {}))
        c.title = str(d.get("title") or "")
        c.context = str(d.get("context") or "")
        c.status = str(d.get("status") or "")
        c.priority = int(d.get("priority") or 0)
        c.message_count = int(d.get("message_count") or 0)
        c.last_activity = parse_time(d.get("last_activity")) or 0
        c.last_active_time = parse_time(d.get("last_active_time")) or 0
        c.updated_at = parse_time(d.get("updated_at")) or 0
        c.completed_at = parse_time(d.get("completed_at")) or 0
        c.messages = [Message.from_dict(m) for m in (d.get("messages") or [])]
        s = d.get("summary") or {}
        c.evicted_count = int(s.get("evicted_messages", 0))
        c.summary_tokens = list(s.get("salient_tokens", []))
        c.home_gpu = int(d.get("home_gpu", -1))
        return c


class QueueStats:
    """Per-named-queue counters (`queue.go:60-68`).  Always returned as a copy
    (the reference returns its live pointer -- defect D22)."""

    __slots__ = ("pending_count", "processing_count", "completed_count", "failed_count",
                 "total_wait_time", "total_process_time", "last_update")

    def __init__(self, pending_count=0, processing_count=0, completed_count=0, failed_count=0,
                 total_wait_time=0, total_process_time=0, last_update=0):
        self.pending_count = pending_count
        self.processing_count = processing_count
        self.completed_count = completed_count
        self.failed_count = failed_count
        self.total_wait_time = total_wait_time
        self.total_process_time = total_process_time
        self.last_update = last_update

    def to_dict(self) -> Dict[str, Any]:
        return {
            "PendingCount": self.pending_count,
            "ProcessingCount": self.processing_count,
            "CompletedCount": self.completed_count,
            "FailedCount": self.failed_count,
            "TotalWaitTime": self.total_wait_time,
            "TotalProcessTime": self.total_process_time,
            "LastUpdate": format_time(self.last_update),
        }

    def __repr__(self) -> str:
        return (f"QueueStats(pending={self.pending_count}, processing={self.processing_count}, "
                f"completed={self.completed_count}, failed={self.failed_count})")
