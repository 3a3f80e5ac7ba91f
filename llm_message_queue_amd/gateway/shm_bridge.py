"""Cross-process request/event rings (fixes D14: the reference's api-gateway
and queue-manager never shared a queue, `cmd/api-gateway/main.go:66`,
`cmd/queue-manager/main.go:58`).

Ingress processes (HTTP workers, `cli api-gateway`) preprocess messages and
push them into the *request* ring; the dispatcher process (`cli
queue-manager`, owner of the GPU backend) pops them into its native
MultiLevelQueue and reports status changes back through the *event* ring.
Both rings are ``_shmring.ShmRing`` (POSIX shm, MPMC, futex wake-ups).

Wire format: msgpack.  A message travels with its preprocessing results
(priority, analysis metadata, GPU-tokenizer prompt ids), so the dispatcher
never re-runs the preprocessor, and with its monotonic arrival timestamp
(CLOCK_MONOTONIC is system-wide), so enqueue->dispatch latency is measured
from the moment the ingress process received the request.
"""
from __future__ import annotations

from typing import Iterable, List, Sequence

import msgpack
import numpy as np

from .. import _native
from ..models.message import Message

TAG_MESSAGE = 1          # preprocessed Message (msgpack), from a Python ingress
TAG_EVENT = 2            # status event back to the ingress
TAG_RAW = 3              # raw JSON body from the native HTTP ingress (not yet preprocessed)

_FIELDS = ("id", "conversation_id", "user_id", "content", "priority", "status", "queue_name",
           "retry_count", "max_retries", "timeout", "created_at", "updated_at", "scheduled_at",
           "completed_at", "metadata", "arrival_ns")


def encode_message(m: Message) -> bytes:
    rec = [getattr(m, f) for f in _FIELDS]
    p = m.prompt_ids
    rec.append(None if p is None else np.ascontiguousarray(p, dtype=np.uint32).tobytes())
    return msgpack.packb(rec, use_bin_type=True)


def decode_message(b: bytes) -> Message:
    rec = msgpack.unpackb(b, raw=False, strict_map_key=False)
    m = Message()
    for f, v in zip(_FIELDS, rec):
        setattr(m, f, v)
    if m.metadata is None:
        m.metadata = {}
    p = rec[len(_FIELDS)]
    m.prompt_ids = None if p is None else np.frombuffer(p, dtype=np.uint32).copy()
    return m


def decode_raw(b: bytes) -> Message:
    """TAG_RAW record of the native ingress: [u64 arrival monotonic ns][36 B
    id][u32 body length][JSON body].  Raises ValueError on a bad body."""
    import json
    arrival = int.from_bytes(b[0:8], "little", signed=True)
    mid = b[8:44].rstrip(b"\x00").decode()
    n = int.from_bytes(b[44:48], "little")
    body = json.loads(b[48:48 + n])
    m = Message.from_dict(body)
    m.id = mid
    m.arrival_ns = arrival
    return m


def encode_event(m: Message, error: str = "") -> bytes:
    return msgpack.packb([m.id, m.status, m.endpoint_id, int(m.dispatched_at or 0), m.completed_at,
                          int(m.retry_count), error], use_bin_type=True)


def decode_event(b: bytes) -> dict:
    i, st, ep, disp, comp, retries, err = msgpack.unpackb(b, raw=False)
    return {"id": i, "status": st, "endpoint_id": ep, "dispatched_at": disp, "completed_at": comp,
            "retry_count": retries, "error": err}


class RingPair:
    """The request ring and the event ring of one gateway deployment."""

    def __init__(self, name: str, capacity: int = 64 << 20, mode: str = "open", gen: int = 0):
        """``gen`` (job generation, ``parallel.comm.job_token``): "create"
        stamps it, "attach" refuses a ring of another generation."""
        R = _native.shmring().ShmRing
        self.name = name
        self.requests = R(f"llmq-{name}-req", capacity, mode, gen)
        self.events = R(f"llmq-{name}-evt", max(capacity // 4, 1 << 20), mode, gen)

    def unlink_names(self) -> None:
        """Remove the rings' names once every process of the job has mapped
        them (the mappings stay valid): a job that is SIGKILLed then leaves
        nothing in /dev/shm for a later job to find."""
        for r in (self.requests, self.events):
            r.unlink()

    # ingress side
    def put_messages(self, msgs: Sequence[Message]) -> int:
        """Push; returns how many fit (the rest were rejected: ring full)."""
        return self.requests.push_many([encode_message(m) for m in msgs], TAG_MESSAGE)

    def get_events(self, max_n: int = 4096, timeout_ms: int = 0) -> List[dict]:
        return [decode_event(b) for _, b in self.events.pop(max_n, timeout_ms)]

    # dispatcher side
    def get_messages(self, max_n: int = 4096, timeout_ms: int = 0) -> List[Message]:
        return [decode_message(b) for _, b in self.requests.pop(max_n, timeout_ms)]

    def get_records(self, max_n: int = 4096, timeout_ms: int = 0, share: int = 1, who: int = -1):
        """[(tag, payload)]: TAG_MESSAGE records and TAG_RAW records.
        ``share``: consumers draining this ring together; ``who`` (0 ..
        share-1): this consumer's id -- take only up to an even share of
        everything taken so far (``ShmRing::pop``, balanced); without it a
        per-pop 1/share part of what is queued."""
        return self.requests.pop(max_n, timeout_ms, share, who)

    def put_events(self, msgs: Iterable[Message], error: str = "") -> int:
        recs = [encode_event(m, error) for m in msgs]
        return self.events.push_many(recs, TAG_EVENT) if recs else 0

    def stats(self) -> dict:
        return {"requests": self.requests.stats(), "events": self.events.stats()}

    def wake_all(self) -> None:
        self.requests.wake_all()
        self.events.wake_all()

    def close(self, unlink: bool = False) -> None:
        for r in (self.requests, self.events):
            if unlink:
                r.unlink()
            r.close()
