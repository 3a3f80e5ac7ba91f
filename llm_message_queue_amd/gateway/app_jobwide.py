"""Job-wide admin and lookups of ``GatewayApp`` (split out of app.py): in a
multi-GPU job every rank keeps the messages, dead letters and counters of
the requests it popped, so rank 0's API answers by asking its peers over
the shared-memory peer directory (``gateway.peers``).  The reference has one
process and answers from its own maps (`api/handlers.go:160-559`)."""
from __future__ import annotations

import time
from typing import Dict, List, Optional, Tuple

import numpy as np

from ..models.message import Message, MessageStatus
from .request_table import NONE, RETRY
from .router import StageRecorder

# cancel answers that mean "this request will not complete"
CANCEL_ACCEPTED = ("cancelled", "forwarded", "pending")


class JobWideMixin:
    # ------------------------------------------------------------------ cross-rank lookups
    def peer_op(self, op: str, args: list):
        """Answer a rank-0 query about messages this rank popped."""
        if op == "get":
            m = self.messages.get(str(args[0]))
            return None if m is None else m.to_dict()
        if op == "list":
            user_id, conversation_id, status, limit = str(args[0]), str(args[1]), str(args[2]), int(args[3])
            total, msgs = self.messages.query(user_id, conversation_id, status, limit, 0)
            return [total, [m.to_dict() for m in msgs]]
        if op == "set_status":
            m = self.messages.get(str(args[0]))
            if m is None:
                return False
            m.status = str(args[1])
            m.updated_at = time.time_ns()
            return True
        if op == "remove":
            m = self.messages.remove(str(args[0]))
            if m is None:
                return False
            removed = bool(m.queue_name and self.standard.has_queue(m.queue_name)
                           and self.standard.remove_message(m.queue_name, m))
            res = "" if removed else self.cancel_inflight(m)
            return {"dequeued": removed or res == "dequeued", "cancelled": res in CANCEL_ACCEPTED}
        if op == "stats":
            return self._rank_stats()
        if op == "reset_latency":
            self.reset_latency()
            return True
        if op == "pre_state":
            self.preprocessor.load_state(args[0])
            return True
        if op == "dlq":
            return self._dlq_local(str(args[0]), str(args[1]) if len(args) > 1 else "")
        if op == "dequeue":
            return self._dequeue_local(str(args[0]), str(args[1]))
        if op == "metrics":
            return self.metrics.render().decode()
        raise ValueError(f"unknown op {op!r}")

    # ------------------------------------------------------------------ job-wide admin
    def _dlq_local(self, action: str, mid: str = ""):
        from ..queue.core import QueueError
        dlq = self.factory.dead_letter_queue
        if action == "list":                       # mid = the item limit per rank
            return [dict(it.to_dict(), rank=self.gateway.rank) for it in dlq.get_all()[:int(mid or 1000)]]
        if action == "requeue_all":
            return dlq.requeue_all(self.standard)
        try:
            if action == "requeue":
                dlq.requeue_by_id(mid, self.standard)
            elif action == "remove":
                i = dlq.index_of(mid)
                if i < 0:
                    return False
                dlq.remove(i)
            else:
                raise ValueError(f"unknown dead-letter action {action!r}")
        except QueueError as e:
            return False if e.code == "INDEX_OUT_OF_RANGE" else {"error": str(e)}
        return True

    def dead_letters(self, action: str, mid: str = ""):
        """Dead-letter admin over the whole job: every GPU rank keeps the
        dead letters of the requests it popped, so ``list`` and
        ``requeue_all`` gather from all ranks and ``requeue`` / ``remove``
        act on the rank that holds ``mid`` (True; False: nowhere; a dict
        ``{"error"}``: the requeue push failed)."""
        res = self._dlq_local(action, mid)
        if self.peers is None:
            return res
        if action == "list":
            for _r, part in sorted(self.peers.ask("dlq", [action, mid]).items()):
                if isinstance(part, list):
                    res.extend(part)
            return res
        if action == "requeue_all":
            return res + sum(int(n) for n in self.peers.ask("dlq", [action]).values() if isinstance(n, int))
        if res is False:
            got = self.peers.first("dlq", [action, mid])
            return got if got is not None else False
        return res

    def cancel_inflight(self, m: Message, timeout_s: float = 1.5) -> str:
        """Cancel ``m`` wherever it is in this router's request lifecycle
        (``DELETE /api/v1/messages/{id}``; ``gateway.request_table``): inbox,
        preprocess batch, queue, retry backoff, held for its KV, running on
        this rank's GPU or on another's.  Gated on the lifecycle state, not
        on ``status`` (a request placed on another rank's GPU
        keeps status pending).  Returns the serve loop's answer ("dequeued",
        "cancelled", "forwarded"), "pending" when the serve loop did not
        answer in time (the request is tombstoned all the same: it ends at
        the next tick and never completes), or "" (it had already ended)."""
        if m.lc == NONE:
            return ""
        f = self.gateway.request_cancel(m)
        try:
            return f.result(timeout=timeout_s)
        except Exception:                      # noqa: BLE001 -- serve loop busy / stopping
            return "pending" if m.handle in self.gateway.table.tomb else ""

    def _dequeue_local(self, queue_type: str, mid: str) -> bool:
        if queue_type == "delayed":
            # a request waiting out a retry backoff (the gateway's retry queue
            # is the factory's DelayedQueue): ended through the lifecycle, so
            # no later delivery can requeue it
            dq = self.factory.delayed_queue
            m = self.messages.get(mid) or dq.find(mid)
            if m is None:
                return False
            if m.lc == RETRY:
                return self.cancel_inflight(m) in ("cancelled", "pending")
            return dq.remove(m)
        mgr = self.factory.get_queue_manager(queue_type)
        m = self.messages.get(mid)
        return bool(mgr is not None and m is not None and m.queue_name and mgr.has_queue(m.queue_name)
                    and mgr.remove_message(m.queue_name, m))

    def dequeue(self, queue_type: str, mid: str) -> bool:
        """Remove a queued message from ``queue_type`` on whichever rank
        queued it (``DELETE /api/v1/admin/queues/{type}/{id}``)."""
        if self._dequeue_local(queue_type, mid):
            return True
        return bool(self.peers is not None and self.peers.first("dequeue", [queue_type, mid]))

    def sync_preprocessor(self) -> List[int]:
        """Copy this rank's preprocessor admin state (keyword rules, user
        priorities) to every peer rank, which preprocess the requests they
        pop with their own preprocessor.  Returns the ranks that did NOT
        confirm (empty: the whole job applies the same rules).  The full
        state travels each time, so a later successful sync repairs a rank
        that missed one."""
        if self.peers is None or self.peers.world <= 1:
            return []
        got = self.peers.ask("pre_state", [self.preprocessor.export_state()])
        return [r for r in range(1, self.peers.world) if got.get(r) is not True]

    def _rank_stats(self) -> dict:
        gw = self.gateway
        gw.flush_latency()
        return {"rank": gw.rank, "counters": dict(gw.counters), "accepted": self._accepted,
                "arr": gw.rec.arr.tolist(), "enq": gw.rec.enq.tolist(), "done": gw.rec_done.arr.tolist(),
                "pending": [self.standard.size(n) for n in gw.tiers],
                "tier_stats": [self._tier_counts(n) for n in gw.tiers],
                "dead_letter": self.factory.dead_letter_queue.size(), "delayed": self.factory.delayed_queue.size(),
                # where this rank's serve loop spends a tick (same fields as bench.py's JSON)
                "profile": {"ticks": int(gw.counters["ticks"] - gw._ticks0), "host_ms_per_tick": gw.host_profile(),
                            "collective": gw.lockstep_stats(),
                            "latency_breakdown": StageRecorder.summary(gw.rec_stage.h, gw.rec_stage.paths)}}

    def metrics_exposition(self) -> bytes:
        """``/metrics``: this process's registry; in a multi-GPU job every
        rank's, merged with a ``rank`` label (each rank counts the requests it
        popped, so rank 0 alone is a partial view)."""
        if self.peers is None or self.peers.world <= 1:
            return self.metrics.render()
        from ..utils.metrics import merge_expositions
        parts = {self.gateway.rank: self.metrics.render().decode()}
        for r, text in self.peers.ask("metrics", []).items():
            if isinstance(text, str):
                parts[int(r)] = text
        return merge_expositions(parts)

    def _tier_counts(self, name: str) -> List[int]:
        st = self.standard.get_queue_stats(name)
        return [int(st.pending_count), int(st.processing_count), int(st.completed_count), int(st.failed_count)]

    def job_stats(self) -> dict:
        """Dispatch counters and latency summed over every rank of the job
        (multi-GPU front door): this rank's plus each peer's answer."""
        from .router import LatencyRecorder
        parts = [self._rank_stats()]
        if self.peers is not None:
            parts += [r for _k, r in sorted(self.peers.ask("stats", []).items())
                      if isinstance(r, dict) and "counters" in r]      # (not a peer's {"error": ...})
        cnt: Dict[str, int] = {}
        for p in parts:
            for k, v in p["counters"].items():
                cnt[k] = cnt.get(k, 0) + int(v)
        arr = sum(np.asarray(p["arr"], dtype=np.int64) for p in parts)
        enq = sum(np.asarray(p["enq"], dtype=np.int64) for p in parts)
        done = sum(np.asarray(p["done"], dtype=np.int64) for p in parts)
        rec = LatencyRecorder(len(self.gateway.tiers))
        tiers = self.gateway.tiers
        return {"ranks": sorted(int(p["rank"]) for p in parts), "dispatch": cnt,
                # ranks whose answer did not arrive (timed out / dropped): the totals leave them out
                "missing_ranks": list(self.peers.last_missing) if self.peers is not None else [],
                # the C++ front door's counters: accepted, ring-full 503s, proxied routes, proxy errors
                "front_door": self.front_door.stats() if self.front_door is not None else None,
                "accepted_by_rank": {int(p["rank"]): int(p["accepted"]) for p in parts},
                "pending_by_tier": {n: sum(int(p.get("pending", [0] * len(tiers))[t]) for p in parts)
                                    for t, n in enumerate(tiers)},
                "tiers": {n: dict(zip(("pending", "processing", "completed", "failed"),
                                      (sum(int(p["tier_stats"][t][k]) for p in parts if "tier_stats" in p)
                                       for k in range(4))))
                          for t, n in enumerate(tiers)},
                "dead_letter": sum(int(p.get("dead_letter", 0)) for p in parts),
                "delayed": sum(int(p.get("delayed", 0)) for p in parts),
                "profile_by_rank": {int(p["rank"]): p.get("profile") for p in parts},
                "latency": rec.summary(arr, enq), "latency_e2e": rec.summary(done, done)}

    def reset_latency_all(self) -> None:
        self.reset_latency()
        if self.peers is not None:
            self.peers.ask("reset_latency", [])

    def find_message(self, mid: str) -> Optional[dict]:
        """A message by id from this process's store, else from the rank that
        popped it (multi-GPU front door)."""
        m = self.messages.get(mid)
        if m is not None:
            return m.to_dict()
        if self.peers is not None:
            return self.peers.first("get", [mid])
        return None

    def query_messages(self, user_id: str, conversation_id: str, status: str, limit: int,
                       offset: int) -> Tuple[int, List[dict]]:
        total, msgs = self.messages.query(user_id, conversation_id, status, limit + offset, 0)
        out = [m.to_dict() for m in msgs]
        if self.peers is not None:
            for _r, res in sorted(self.peers.ask("list", [user_id, conversation_id, status,
                                                          limit + offset]).items()):
                if isinstance(res, list) and len(res) == 2:
                    total += int(res[0])
                    out.extend(res[1])
        return total, out[offset:offset + limit]

