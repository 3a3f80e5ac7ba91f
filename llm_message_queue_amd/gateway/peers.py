"""Cross-rank message lookups for the multi-GPU `cli serve` front door.

With the native front door every GPU rank drains the shared request ring, so
a message lives in the message store of whichever rank popped it.  The REST
API runs on rank 0; a status or admin request for a message rank 0 does not
hold is answered by a scatter-gather query over node-local shared-memory
rings: rank 0 pushes ``[qid, op, args]`` into each peer's query ring, a
responder thread on every peer answers from its own store into the shared
reply ring.  Admin-rate traffic only (the hot submit path never queries).
The same channel carries the preprocessor's admin state (``pre_state``):
every rank preprocesses the requests it pops, so a keyword rule or user
priority set through rank 0's API must reach every rank.

The reference serves every route from one process and keeps no per-message
state at all (`api/handlers.go:222-256` are stubs); this keeps the whole
job's messages addressable from one API endpoint.
"""
from __future__ import annotations

import threading
import time
from typing import Any, Callable, Dict, List, Optional

import msgpack

from .. import _native

OPS = ("get", "list", "set_status", "remove", "stats", "reset_latency", "pre_state", "dlq", "dequeue", "metrics")


def _is_error(res: Any) -> bool:
    return isinstance(res, dict) and set(res) == {"error"}


class PeerDirectory:
    """Rank 0 asks, ranks > 0 answer.  Each peer answers into a reply ring of
    its own (``REPLY_RING`` bytes), so one peer's large answer can never
    crowd another's out; an answer larger than ``CHUNK`` travels in pages
    (``[qid, rank, seq, n, bytes]``), so its size is bounded only by
    ``ANSWER_MAX``.  A page that does not fit is retried until the query's
    deadline and then counted in ``dropped`` -- never silently lost -- and
    rank 0 reports the ranks that did not answer (``last_missing``,
    ``missing_total``).  Late pages of a query that already timed out are
    discarded on the next ask, so they take no space from it."""

    CHUNK = 1 << 20                  # bytes per reply page
    REPLY_RING = 4 << 20             # per-peer reply ring (>= 2 pages in flight plus slack)
    ANSWER_MAX = 256 << 20           # larger answers are replaced by an explicit error

    def __init__(self, name: str, rank: int, world: int, handler: Optional[Callable[[str, list], Any]] = None,
                 comm=None, gen: int = 0):
        """``handler(op, args)`` answers a query on ranks > 0 (the app's
        local store); rank 0 asks with ``ask``.  With ``comm`` (every rank
        constructs the directory at the same point): rank 0 CREATES the rings
        stamped with the job generation ``gen``, a barrier, then the peers
        attach (refusing a ring of another generation) and rank 0 drops the
        names -- nothing of this job survives a SIGKILL in /dev/shm.  Without
        ``comm`` every rank opens the rings by name (tests, one process)."""
        R = _native.shmring().ShmRing
        self.rank, self.world, self.name = rank, world, name
        self.handler = handler
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.asked = self.answered = self.timeouts = self.dropped = self.missing_total = 0
        self.last_missing: List[int] = []
        coll = comm is not None and world > 1
        if rank == 0:
            mode = "create" if coll else "open"
            self.qrings = {r: R(f"llmq-{name}-q{r}", 1 << 20, mode, gen) for r in range(1, world)}
            self.replies = {r: R(f"llmq-{name}-qrep{r}", self.REPLY_RING, mode, gen) for r in range(1, world)}
            self._lock = threading.Lock()
            self._qid = 0
        if coll:
            comm.barrier()                             # rank 0's rings exist
        if rank != 0:
            mode = "attach" if coll else "open"
            self.qring = R(f"llmq-{name}-q{rank}", 1 << 20, mode, gen)
            self.reply = R(f"llmq-{name}-qrep{rank}", self.REPLY_RING, mode, gen)
        if coll:
            comm.barrier()                             # every peer mapped them
            if rank == 0:
                for r in list(self.qrings.values()) + list(self.replies.values()):
                    r.unlink()
        if rank != 0:
            self._thread = threading.Thread(target=self._serve, name="peer-queries", daemon=True)
            self._thread.start()

    # ------------------------------------------------------------------ rank 0
    def ask(self, op: str, args: list, timeout_s: float = 2.0) -> Dict[int, Any]:
        """Send ``op`` to every peer and collect ``{rank: result}`` (ranks
        that did not answer within ``timeout_s`` are missing, and listed in
        ``last_missing``)."""
        if self.rank != 0 or self.world <= 1:
            return {}
        if op not in OPS:
            raise ValueError(f"unknown peer op {op!r}")
        with self._lock:
            self._qid += 1
            qid = self._qid
            deadline = time.monotonic() + timeout_s
            # the responder stops retrying a page that does not fit at the deadline
            rec = msgpack.packb([qid, op, list(args), int(deadline * 1e9)], use_bin_type=True)
            for r, ring in self.replies.items():
                while ring.pop(64, 0):                # late pages of earlier queries
                    pass
            for r, q in self.qrings.items():
                q.push(rec, 1)
            self.asked += 1
            out: Dict[int, Any] = {}
            pages: Dict[int, Dict[int, bytes]] = {}
            pending = set(self.replies)

            def take(r: int, recs) -> bool:
                for _tag, b in recs:
                    q, _rr, seq, n, chunk = msgpack.unpackb(b, raw=False, strict_map_key=False)
                    if q != qid:
                        continue
                    pg = pages.setdefault(r, {})
                    pg[int(seq)] = chunk
                    if len(pg) == int(n):
                        out[r] = msgpack.unpackb(b"".join(pg[i] for i in range(int(n))), raw=False,
                                                 strict_map_key=False)
                        pending.discard(r)
                return bool(recs)

            while pending:
                left = deadline - time.monotonic()
                if left <= 0:
                    self.timeouts += 1
                    break
                got = False
                for r in sorted(pending):
                    got |= take(r, self.replies[r].pop(64, 0))
                if not got and pending:                # block briefly on one outstanding peer's ring
                    r0 = min(pending)
                    take(r0, self.replies[r0].pop(64, max(1, min(20, int(left * 1000)))))
            self.last_missing = sorted(pending)
            self.missing_total += len(pending)
            return out

    def first(self, op: str, args: list, timeout_s: float = 2.0) -> Any:
        """The first non-None answer (a message lives on one rank).  A peer
        whose handler raised answers ``{"error": ...}``: that is no answer."""
        for _r, res in sorted(self.ask(op, args, timeout_s).items()):
            if res is None or res is False or _is_error(res):
                continue
            return res
        return None

    # ------------------------------------------------------------------ ranks > 0
    def _answer(self, qid: int, res: Any, deadline_ns: int) -> bool:
        body = msgpack.packb(res, use_bin_type=True, default=str)
        if len(body) > self.ANSWER_MAX:
            body = msgpack.packb({"error": f"reply of {len(body)} B exceeds {self.ANSWER_MAX} B"},
                                 use_bin_type=True)
        n = max(1, -(-len(body) // self.CHUNK))
        for seq in range(n):
            rec = msgpack.packb([qid, self.rank, seq, n, body[seq * self.CHUNK:(seq + 1) * self.CHUNK]],
                                use_bin_type=True)
            # rank 0 drains the pages while it waits: retry a full ring until
            # the query's deadline, then give the answer up explicitly
            while not self.reply.push(rec, 1):
                if self._stop.is_set() or time.monotonic_ns() > deadline_ns:
                    self.dropped += 1
                    return False
                time.sleep(0.001)
        return True

    def _serve(self) -> None:
        while not self._stop.is_set():
            for _tag, b in self.qring.pop(16, 100):
                qid, deadline_ns = -1, 0
                try:
                    qid, op, args, deadline_ns = msgpack.unpackb(b, raw=False, strict_map_key=False)
                    res = self.handler(op, args) if self.handler is not None else None
                except Exception as e:                # noqa: BLE001 -- answered, never fatal
                    res = {"error": str(e)}
                if self._answer(qid, res, int(deadline_ns)):
                    self.answered += 1

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self.qring.wake_all()
            self._thread.join(timeout=5)

    def close(self, unlink: bool = False) -> None:
        self.stop()
        rings = (list(self.qrings.values()) + list(self.replies.values())) if self.rank == 0 \
            else [self.qring, self.reply]
        for r in rings:
            if unlink:
                r.unlink()
            r.close()
