"""Queue checkpoint / resume (SURVEY.md §5 "checkpoint/resume").

The reference persists conversations only; queue contents, the DLQ and the
retry schedule are in-memory and lost on restart, and queue snapshots are
doc-only (`docs/configuration.md:290-309`).  Here a snapshot is one JSONL
file (written to a temp name and renamed, so a crash never leaves a torn
file) holding, per message:

  * ``queued``      -- waiting in a manager's level queue (order preserved);
  * ``inflight``    -- dispatched but not completed (re-queued on resume:
                       at-least-once delivery);
  * ``delayed``     -- a scheduled retry, with its wall-clock ready time;
  * ``dead_letter`` -- a DLQ entry with reason / source / retry count.

Messages carry their preprocessing (priority, analysis metadata, GPU
tokenizer prompt ids), so a resumed gateway does not re-run it.
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Iterable, Optional

import numpy as np

from ..models.message import Message, MessageStatus
from .dead_letter import DeadLetterItem

VERSION = 1


def _msg(m: Message) -> dict:
    d = m.to_dict()
    if m.prompt_ids is not None:
        d["_prompt_ids"] = np.asarray(m.prompt_ids, dtype=np.uint32).tolist()
    return d


def _unmsg(d: dict) -> Message:
    ids = d.pop("_prompt_ids", None)
    m = Message.from_dict(d)
    if ids is not None:
        m.prompt_ids = np.asarray(ids, dtype=np.uint32)
    return m


def write_snapshot(factory, path: str, inflight: Iterable[Message] = ()) -> Dict[str, int]:
    """Write every manager's queued messages, ``inflight``, the delayed
    retries and the DLQ of ``factory`` (a QueueFactory) to ``path``."""
    counts = {"queued": 0, "inflight": 0, "delayed": 0, "dead_letter": 0}
    tmp = f"{path}.tmp{os.getpid()}"
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(tmp, "w") as f:
        f.write(json.dumps({"kind": "header", "version": VERSION, "created_at_ns": time.time_ns()}) + "\n")
        for mname, mgr in factory.managers().items():
            for q in mgr.queue_names():
                for m in mgr.mlq.messages(q):
                    f.write(json.dumps({"kind": "queued", "manager": mname, "queue": q, "message": _msg(m)}) + "\n")
                    counts["queued"] += 1
        for m in inflight:
            f.write(json.dumps({"kind": "inflight", "queue": m.queue_name, "message": _msg(m)}) + "\n")
            counts["inflight"] += 1
        for m, ready_at, _target in factory.delayed_queue.items():
            f.write(json.dumps({"kind": "delayed", "queue": m.queue_name, "ready_at_ns": ready_at,
                                "message": _msg(m)}) + "\n")
            counts["delayed"] += 1
        for it in factory.dead_letter_queue.get_all():
            f.write(json.dumps({"kind": "dead_letter", "reason": it.fail_reason, "failed_at_ns": it.failed_at,
                                "source_queue": it.source_queue, "retry_count": it.retry_count,
                                "message": _msg(it.message)}) + "\n")
            counts["dead_letter"] += 1
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, path)
    return counts


def read_snapshot(factory, path: str, default_manager: str = "standard",
                  retry_target=None) -> Optional[Dict[str, int]]:
    """Replay ``path`` into ``factory``.  ``retry_target(msg)`` receives due
    delayed retries (default: push to the default manager's level queue).
    Returns counts, or None if there is no snapshot."""
    if not path or not os.path.exists(path):
        return None
    counts = {"queued": 0, "inflight": 0, "delayed": 0, "dead_letter": 0, "rejected": 0}
    default = factory.get_queue_manager(default_manager)

    def push(mgr, q, m):
        if not mgr.has_queue(q):
            mgr.create_queue(q)
        mgr.push_message(q, m)

    def to_default(m: Message):
        push(default, m.queue_name, m)

    with open(path) as f:
        for line in f:
            line = line.strip()
            if not line:
                continue
            rec = json.loads(line)
            kind = rec.get("kind")
            if kind == "header":
                if rec.get("version") != VERSION:
                    raise ValueError(f"snapshot version {rec.get('version')} != {VERSION}")
                continue
            m = _unmsg(rec["message"])
            try:
                if kind == "queued":
                    mgr = factory.get_queue_manager(rec.get("manager", default_manager)) or default
                    push(mgr, rec["queue"], m)
                elif kind == "inflight":
                    m.status = MessageStatus.PENDING
                    push(default, rec.get("queue") or m.queue_name, m)
                elif kind == "delayed":
                    factory.delayed_queue.schedule(m, int(rec["ready_at_ns"]), target=retry_target or to_default)
                elif kind == "dead_letter":
                    factory.dead_letter_queue.restore(DeadLetterItem(m, rec["reason"], int(rec["failed_at_ns"]),
                                                                     rec["source_queue"], int(rec["retry_count"])))
                else:
                    continue
                counts[kind] += 1
            except Exception:
                counts["rejected"] += 1
    return counts
