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
from typing import Any, Callable, Dict, Optional

import msgpack

from .. import _native

OPS = ("get", "list", "set_status", "remove", "stats", "reset_latency", "pre_state", "dlq", "dequeue", "metrics")


def _is_error(res: Any) -> bool:
    return isinstance(res, dict) and set(res) == {"error"}


class PeerDirectory:
    REPLY_MAX = 2 << 20              # bytes per answer (the reply ring holds 8 MiB for all peers)

    def __init__(self, name: str, rank: int, world: int, handler: Optional[Callable[[str, list], Any]] = None):
        """``handler(op, args)`` answers a query on ranks > 0 (the app's
        local store); rank 0 asks with ``ask``."""
        R = _native.shmring().ShmRing
        self.rank, self.world, self.name = rank, world, name
        self.handler = handler
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None
        self.reply = R(f"llmq-{name}-qrep", 8 << 20, "open")
        self.asked = self.answered = self.timeouts = 0
        if rank == 0:
            self.qrings = {r: R(f"llmq-{name}-q{r}", 1 << 20, "open") for r in range(1, world)}
            self._lock = threading.Lock()
            self._qid = 0
        else:
            self.qring = R(f"llmq-{name}-q{rank}", 1 << 20, "open")
            self._thread = threading.Thread(target=self._serve, name="peer-queries", daemon=True)
            self._thread.start()

    # ------------------------------------------------------------------ rank 0
    def ask(self, op: str, args: list, timeout_s: float = 2.0) -> Dict[int, Any]:
        """Send ``op`` to every peer and collect ``{rank: result}`` (ranks
        that did not answer within ``timeout_s`` are missing)."""
        if self.rank != 0 or self.world <= 1:
            return {}
        if op not in OPS:
            raise ValueError(f"unknown peer op {op!r}")
        with self._lock:
            self._qid += 1
            qid = self._qid
            rec = msgpack.packb([qid, op, list(args)], use_bin_type=True)
            for r, q in self.qrings.items():
                q.push(rec, 1)
            self.asked += 1
            out: Dict[int, Any] = {}
            deadline = time.monotonic() + timeout_s
            while len(out) < self.world - 1:
                left = deadline - time.monotonic()
                if left <= 0:
                    self.timeouts += 1
                    break
                for _tag, b in self.reply.pop(64, max(1, int(left * 1000))):
                    q, r, res = msgpack.unpackb(b, raw=False, strict_map_key=False)
                    if q == qid:                       # (late answers to an earlier query are dropped)
                        out[int(r)] = res
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
    def _serve(self) -> None:
        while not self._stop.is_set():
            for _tag, b in self.qring.pop(16, 100):
                qid = -1
                try:
                    qid, op, args = msgpack.unpackb(b, raw=False, strict_map_key=False)
                    res = self.handler(op, args) if self.handler is not None else None
                except Exception as e:                # noqa: BLE001 -- answered, never fatal
                    res = {"error": str(e)}
                rec = msgpack.packb([qid, self.rank, res], use_bin_type=True, default=str)
                if len(rec) > self.REPLY_MAX:          # never wedge the shared reply ring
                    rec = msgpack.packb([qid, self.rank, {"error": f"reply of {len(rec)} B too large"}],
                                        use_bin_type=True)
                self.reply.push(rec, 1)
                self.answered += 1

    def stop(self) -> None:
        self._stop.set()
        if self._thread is not None:
            self.qring.wake_all()
            self._thread.join(timeout=5)

    def close(self, unlink: bool = False) -> None:
        self.stop()
        rings = [self.reply] + (list(self.qrings.values()) if self.rank == 0 else [self.qring])
        for r in rings:
            if unlink:
                r.unlink()
            r.close()
