"""Failure handling of the gateway (``Gateway`` mixin): overload shedding of
expired queued requests, the in-flight processing timeout and cancellation
(``K_TIMEOUT`` / ``K_CANCELLED`` / ``K_CANCEL`` across ranks), the retry path
(DelayedQueue backoff, dead-letter queue when spent -- the reference's
handleFailure, `internal/priorityqueue/worker.go:202-239`), and GPU health
(evacuation).

Threads: everything here runs on the serve loop (inside the tick) except
``request_cancel`` (API / peer threads: queues the request under
``_cancel_lock``), ``_retry_ready`` (the DelayedQueue's thread: appends under
``_retry_lock``) and ``set_healthy`` (telemetry / API threads: takes the
tick lock first)."""
from __future__ import annotations

import time
from typing import Dict, List, Optional

import numpy as np

from ..backend.engine import Request
from ..models.message import Message, MessageStatus
from ..queue.core import QueueError
from .descriptors import FAIL_FAILED, FAIL_UNTOUCHED, K_CANCELLED, K_FAIL, K_TIMEOUT, _get64
from .request_table import HELD, INBOX, LOCAL, NONE, PREPROCESS, QUEUED, REMOTE, RETRY


class FailureMixin:
    def expire_queued(self, now: Optional[int] = None) -> int:
        """Overload shedding: pop every tier head whose deadline (arrival +
        ``timeout``) has passed and move it to the dead-letter queue (status
        ``timeout``).  Tiers are FIFO, so the expired requests of a tier are
        its head run; the cost when nothing expired is one peek per tier.
        Runs before the load exchange, so multi-rank plans only see live
        requests."""
        now = time.monotonic_ns() if now is None else now
        out: List[Message] = []
        for name in self.tiers:
            while True:
                try:
                    m = self.qm.peek_message(name)
                except QueueError:
                    break
                if not self._expired(m, now):
                    break
                try:
                    m = self.qm.pop_message(name)
                except QueueError:
                    break
                self._pin(m, -1)
                out.append(m)
        self._shed(out)
        return len(out)

    @staticmethod
    def _expired(m: Message, now: int) -> bool:
        # a retried request (backend failure, processing timeout) gets a fresh
        # queue deadline from its requeue: its first deadline has passed
        t0 = (m.enqueued_at if m.retry_count > 0 else 0) or m.arrival_ns or m.enqueued_at
        return bool(m.timeout > 0 and t0 and now - t0 > m.timeout)

    def _shed(self, out: List[Message]) -> None:
        """Popped, expired requests -> status timeout + dead-letter queue."""
        for m in out:
            m.status = MessageStatus.TIMEOUT
            self.table.end(m)
            self.qm.fail_message(m.queue_name, m.id, None, m.priority, quiet=True)
        if out:
            self.counters["expired"] += len(out)
            if self.metrics is not None:
                self.metrics.requests_rejected.labels("deadline_exceeded").inc(len(out))
            if self.dead_letter is not None:
                by_q: Dict[str, List[Message]] = {}
                for m in out:
                    by_q.setdefault(m.queue_name, []).append(m)
                for q, ms in by_q.items():
                    self.dead_letter.push_many(ms, "deadline exceeded before dispatch", q)
            if self.on_expire is not None:
                for m in out:
                    self.on_expire(m)

    def _remote_fail(self, row: np.ndarray) -> None:
        """The backend my request was sent to handed it back (K_FAIL).  The
        record's admitted field is 1 when that backend failed while running
        it: the retry path (backoff, retry count, dead letter).  0: it never
        ran there (a held turn, an over-committed plan, an operator's drain):
        back into its tier at once, no retry spent."""
        r1 = row.reshape(1, -1)
        handle = int(_get64(r1, 1)[0])
        m = self.remote_out.pop(handle, None)
        if m is None:
            return
        failed = int(_get64(r1, 5)[0]) == FAIL_FAILED
        self.inflight_by_tier[m.tier] -= 1
        if self.lb is not None and m.endpoint_id:
            self.lb.release_endpoint(m.endpoint_id, 0, failed)   # (note_dispatch counted it)
        m.endpoint_id = ""
        if failed:
            self._retry(m, "backend failed while running the request")
        else:
            self._requeue(m)
        self.counters["handed_back"] += 1

    def _remote_abort(self, row: np.ndarray) -> None:
        """K_TIMEOUT / K_CANCELLED: the GPU running my request aborted it."""
        r1 = row.reshape(1, -1)
        m = self.remote_out.pop(int(_get64(r1, 1)[0]), None)
        if m is None:
            return
        self.inflight_by_tier[m.tier] -= 1
        self._abort_local(m, int(row[0]), max(0, int(_get64(r1, 7)[0] - _get64(r1, 5)[0])))

    # ------------------------------------------------------------------ in-flight timeout / cancel
    EXPIRE_EVERY_NS = 5_000_000      # deadline scan period (a vectorised pass over the slots)

    def _expire_inflight(self) -> None:
        """Abort this GPU's requests whose processing deadline passed."""
        eng = self.engine
        if eng is None or not self.inflight_timeout or not hasattr(eng, "expire"):
            return
        now = time.monotonic_ns()
        if now < self._expire_next_ns:
            return
        self._expire_next_ns = now + self.EXPIRE_EVERY_NS
        for r in eng.expire(now):
            self._aborted(r, K_TIMEOUT, now)

    def _aborted(self, r: Request, kind: int, now: int) -> None:
        """My engine aborted ``r`` (processing timeout / cancel): my own
        message takes the timeout / cancel path here; a foreign one is
        reported to its origin router with the next completion records."""
        if isinstance(r.meta, Message):
            m = r.meta
            self.local.pop(m.handle, None)
            if 0 <= r.tier < len(self.inflight_by_tier):
                self.inflight_by_tier[r.tier] -= 1
            self._abort_local(m, kind, max(0, now - r.admitted_ns))
        else:
            origin, handle, tier = self.foreign.pop(r.req_id)
            self._done_owed[origin].append((handle, tier, r.admitted_ns, now, kind))

    def _abort_local(self, m: Message, kind: int, ran_ns: int) -> None:
        """One of my messages was aborted on the GPU that ran it: a processing
        timeout is a failure (retry with backoff, dead-letter when retries
        are spent -- the reference's handleFailure); a cancel ends it."""
        if self.lb is not None and m.endpoint_id:
            self.lb.release_endpoint(m.endpoint_id, ran_ns, kind == K_TIMEOUT)
        if isinstance(m.metadata, dict):
            m.metadata["last_error"] = "processing timeout" if kind == K_TIMEOUT else "cancelled"
        if kind == K_TIMEOUT:
            self.counters["inflight_timeout"] += 1
            if self.metrics is not None:
                self.metrics.requests_rejected.labels("processing_timeout").inc()
            self._retry(m, f"processing timeout ({m.timeout / 1e9:.3g} s)")
            return
        m.endpoint_id = ""                               # (released above)
        self._finish_cancel(m, dispatched=True)

    def _finish_cancel(self, m: Message, ran_ns: int = 0, dispatched: bool = False) -> None:
        """End ``m`` as cancelled (wherever it was: the caller took it out of
        its container).  ``dispatched``: it was popped for a GPU, so its
        tier's processing count is closed as failed (as a backend failure
        would be) and its balancer endpoint released."""
        self.table.end(m)
        self.table.ended_cancelled += 1
        self.counters["cancelled"] += 1
        m.status = MessageStatus.CANCELLED
        m.updated_at = time.time_ns()
        if dispatched:
            if self.lb is not None and m.endpoint_id:
                self.lb.release_endpoint(m.endpoint_id, ran_ns, False)
                m.endpoint_id = ""
            self.qm.fail_message(m.queue_name, m.id, None, m.priority, quiet=True)
        if isinstance(m.metadata, dict):
            m.metadata["last_error"] = "cancelled"

    def request_cancel(self, m: Message):
        """Any thread: cancel ``m`` wherever it is in this router's lifecycle
        (``gateway.request_table``).  Returns a Future the serve loop
        resolves with "dequeued" (taken out of its tier queue), "cancelled"
        (ended here: inbox, preprocess batch, retry backoff, held for its
        KV, or aborted on this rank's GPU), "forwarded" (K_CANCEL sent to the
        GPU running it, which reports the abort back) or "" (not live here:
        it had already ended).  From the moment this returns, the request
        can no longer complete or re-enter service: its handle is
        tombstoned and every re-entry point checks the tombstone."""
        from concurrent.futures import Future
        f: Future = Future()
        with self._cancel_lock:
            if m.lc == NONE:
                f.set_result("")
                return f
            self.table.tomb[m.handle] = m
            self._cancel_req.append((m, f))
        return f

    def _process_cancels(self) -> None:
        if not self._cancel_req:
            return
        with self._cancel_lock:
            reqs, self._cancel_req = self._cancel_req, []
        now = time.monotonic_ns()
        for m, f in reqs:
            res = self._cancel_one(m, now)
            if not f.done():
                f.set_result(res)

    def _cancel_one(self, m: Message, now: int) -> str:
        st = m.lc
        if st == NONE:                                   # ended before the serve loop got here:
            self.table.tomb.pop(m.handle, None)          # by a re-entry check of the tombstone, or otherwise
            return "cancelled" if m.status == MessageStatus.CANCELLED else ""
        if st == INBOX:
            with self._inbox_lock:
                k = next((i for i, x in enumerate(self._inbox) if x is m), -1)
                if k >= 0:
                    del self._inbox[k]
            if k >= 0:
                self._finish_cancel(m)
            return "cancelled"                           # (else taken meanwhile: the enqueue ends it)
        if st == PREPROCESS:
            return "cancelled"                           # ended by _enqueue when its batch lands
        if st == QUEUED:
            if m.queue_name and self.qm.has_queue(m.queue_name) and self.qm.remove_message(m.queue_name, m):
                self._finish_cancel(m)                   # (on_remove released its pin)
                return "dequeued"
            return "cancelled"                           # popped this tick: the dispatch drops it
        if st == RETRY:
            q = self.retry_queue
            took = q is not None and q.remove(m)
            if not took:
                with self._retry_lock:
                    k = next((i for i, x in enumerate(self._retry_due) if x is m), -1)
                    if k >= 0:
                        del self._retry_due[k]
                        took = True
            if took:
                self._finish_cancel(m, dispatched=True)      # (popped once: its processing count is open)
            return "cancelled"                           # (else delivered meanwhile: the requeue ends it)
        if st == HELD:
            for d in (self._await_kv, self._await_import):
                for ck, rs in list(d.items()):
                    keep = [(r, h) for r, h in rs if r.meta is not m]
                    if len(keep) != len(rs):
                        if keep:
                            d[ck] = keep
                        else:
                            del d[ck]
            self._finish_cancel(m, dispatched=True)
            return "cancelled"
        if st == LOCAL:
            got = self.engine.cancel([m.handle]) if self.engine is not None else []
            for r in got:
                self._aborted(r, K_CANCELLED, now)
            return "cancelled"                           # (else its last token is launched: ends at completion)
        if st == REMOTE:
            if str(m.endpoint_id).startswith("gpu"):
                j = int(m.endpoint_id[3:])
                if 0 <= j < self.world and j != self.rank:
                    self._cancel_out.setdefault(j, []).append(m.handle)
            return "forwarded"                           # ends when that GPU reports back
        return ""

    def _cancel_foreign(self, origin: int, handles, held_prev=None) -> None:
        """K_CANCEL rows from ``origin``: abort those of its requests my GPU
        is running or holds for their KV (one that already completed is
        reported done as usual; the origin's tombstone ends it there)."""
        hs = {int(h) for h in handles}
        ids = [rid for rid, (o, h, _t) in self.foreign.items() if o == origin and h in hs]
        now = time.monotonic_ns()
        if ids and self.engine is not None:
            for r in self.engine.cancel(ids):
                self._aborted(r, K_CANCELLED, now)
        for key in [k for k in self._await_hist if k[0] == origin and k[1] in hs]:   # waiting for its history
            r = self._await_hist.pop(key)
            self._hist_wait.pop(key, None)
            self._done_owed[origin].append((r.meta[1], r.meta[2], now, now, K_CANCELLED))
        for d in (self._await_kv, self._await_import, held_prev or {}):
            for ck, rs in list(d.items()):
                keep = []
                for r, h in rs:
                    if not isinstance(r.meta, Message) and r.meta[0] == origin and r.meta[1] in hs:
                        self._done_owed[origin].append((r.meta[1], r.meta[2], now, now, K_CANCELLED))
                    else:
                        keep.append((r, h))
                if len(keep) != len(rs):
                    if keep:
                        d[ck] = keep
                    else:
                        del d[ck]

    def attach_retry_queue(self, delayed, backoff=None) -> None:
        """Route backend-failure retries through ``delayed`` (a
        ``queue.delayed.DelayedQueue``) with ``backoff`` (default: the
        config's exponential ``queue.retry``)."""
        from ..queue.worker import ExponentialBackoff
        r = self.cfg.queue.retry
        self.retry_queue = delayed
        self.retry_backoff = backoff or ExponentialBackoff(r.initial_backoff, r.max_backoff, r.factor,
                                                           r.max_retries)

    def _retry(self, m: Message, reason: str) -> None:
        """A request a backend failure handed back: retry after a backoff, or
        dead-letter it once its retries are spent."""
        if self.table.cancelled(m):
            self._finish_cancel(m, dispatched=True)
            return
        if self.retry_queue is None:
            self._requeue(m)
            return
        # the reference's handleFailure (`worker.go:202-239`): retry while
        # RetryCount < MaxRetries (counting this retry), else dead-letter with
        # RetryCount == MaxRetries (the count was one too high)
        if m.retry_count >= self.retry_backoff.max_retries():
            m.status = MessageStatus.FAILED
            m.endpoint_id = ""
            self.table.end(m)
            self.counters["retry_exhausted"] += 1
            self.qm.fail_message(m.queue_name, m.id, None, m.priority, quiet=True)
            if self.dead_letter is not None:
                try:
                    self.dead_letter.push(m, f"retries exhausted: {reason}", m.queue_name)
                except QueueError:
                    self.log.warning("dead-letter queue full; failed request dropped", message_id=m.id)
            return
        m.retry_count += 1
        m.status = MessageStatus.PENDING
        m.endpoint_id = ""
        m.dispatched_at = 0
        self.counters["retried"] += 1
        self.table.move(m, RETRY)
        self.retry_queue.schedule_after(m, self.retry_backoff.next_backoff(m.retry_count), target=self._retry_ready)

    def retrying(self) -> int:
        """Requests waiting out a retry backoff (or handed back, not yet requeued)."""
        q = self.retry_queue
        return (q.size() if q is not None else 0) + len(self._retry_due)

    def _retry_ready(self, m: Message) -> None:
        """DelayedQueue delivery (its own thread): hand back to the tick."""
        with self._retry_lock:
            self._retry_due.append(m)

    def _drain_retries(self) -> None:
        q = self.retry_queue
        if q is None:
            return
        if getattr(q, "_thread", None) is None:            # no drain thread: deliver here
            for m in q.poll_ready(1024, 0.0):
                self._retry_due.append(m)
        if not self._retry_due:
            return
        with self._retry_lock:
            due, self._retry_due = self._retry_due, []
        for m in due:
            self._requeue(m)

    def _requeue(self, m: Message) -> None:
        if self.table.cancelled(m):
            self._finish_cancel(m, dispatched=True)          # (every requeue follows a pop)
            return
        m.status = MessageStatus.PENDING
        m.endpoint_id = ""
        m.dispatched_at = 0
        self.table.local.pop(m.handle, None)
        self.table.remote_out.pop(m.handle, None)
        self.table.move(m, QUEUED)
        if not self.qm.requeue_after_failure(m.queue_name, m):
            # its tier is full (overload): it cannot go back -- dead-letter it
            # rather than raise into the serve loop (found by the round-6
            # 4-rank overload soak, a fatal 'queue is full')
            m.status = MessageStatus.FAILED
            self.table.end(m)
            self.counters["rejected"] += 1
            if self.dead_letter is not None:
                try:
                    self.dead_letter.push(m, "tier full on requeue", m.queue_name)
                except QueueError:
                    self.log.warning("dead-letter queue full; failed request dropped", message_id=m.id)
            return
        if self.world > 1:
            self._pin(m, +1)

    # ------------------------------------------------------------------ health
    def set_healthy(self, healthy: bool, reason: str = "", failure: bool = True) -> int:
        """Mark this rank's GPU (un)healthy.  Going unhealthy evacuates the
        backend: local requests are re-queued here (the planner then places
        them on healthy GPUs), foreign ones are handed back to their origin
        router (K_FAIL).  ``failure``: the GPU failed (backend error, ECC,
        telemetry) -- the requests it was running take the retry path
        (backoff, retry count, dead letter when spent); an operator's drain
        (``failure`` False) requeues them at once, untouched.  Returns the
        number of evacuated requests."""
        with self._tick_lock:
            return self._set_healthy(healthy, reason, failure)

    def _set_healthy(self, healthy: bool, reason: str, failure: bool = True) -> int:
        was = self.healthy
        self.healthy, self.health_reason = bool(healthy), ("" if healthy else reason)
        if healthy or not was or self.engine is None:
            return 0
        self.log.warning("GPU backend unhealthy; evacuating", rank=self.rank, reason=reason)
        self._err_ewma = 0.9 * self._err_ewma + 0.1
        n = 0
        held = [r for d in (self._await_kv, self._await_import) for rs in d.values() for r, _h in rs]
        held += list(self._await_hist.values())           # foreign turns waiting for their history
        self._await_kv = {}
        self._await_import = {}
        self._await_hist = {}
        self._hist_wait = {}
        for r in held:                                  # turns waiting for a KV that will not be used here
            n += 1
            if isinstance(r.meta, Message):
                # never launched on this GPU: nothing failed for it -- back
                # into its tier at once, no retry spent
                self._requeue(r.meta)
            else:
                origin, handle, tier = r.meta[:3]
                self._done_owed[origin].append((handle, tier, FAIL_UNTOUCHED, 0, K_FAIL))
        if self.migrator is not None:
            # imports still landing on the side stream write into reserved
            # slots that abort_all hands back to the free list: the next
            # forward must wait for them, and their results are void
            self.engine.fence(self.migrator.abandon())
        for r in self.engine.abort_all():
            n += 1
            if isinstance(r.meta, Message):
                m = r.meta
                self.local.pop(m.handle, None)
                if 0 <= r.tier < len(self.inflight_by_tier):
                    self.inflight_by_tier[r.tier] -= 1
                if m.metadata and m.metadata.get("home_gpu") == self.rank:
                    del m.metadata["home_gpu"]
                if failure:
                    self._retry(m, reason)
                else:
                    self._requeue(m)
            else:
                origin, handle, tier = self.foreign.pop(r.req_id)
                self._done_owed[origin].append((handle, tier, FAIL_FAILED if failure else FAIL_UNTOUCHED,
                                                0, K_FAIL))
        self.counters["evacuated"] += n
        return n
