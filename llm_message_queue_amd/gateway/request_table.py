"""Request lifecycle at the origin router: ONE owner of where every request
is.

A request this router accepted is in exactly one state until it ends:

  INBOX       submitted, not yet taken into a preprocess batch (``Gateway._inbox``)
  PREPROCESS  inside an outstanding GPU preprocess batch
  QUEUED      in its tier of the native queue (``qm``)
  RETRY       waiting out a retry backoff (the DelayedQueue or ``_retry_due``)
  HELD        dispatched to this GPU, waiting for its dialog's KV (``_await_kv`` /
              ``_await_import``)
  LOCAL       in a slot of this rank's GPU (``local``)
  REMOTE      sent to another rank's GPU (``remote_out``)
  NONE        ended (completed, cancelled, failed, shed, dead-lettered) or never ours

The state lives on the message (``Message.lc``); every transition goes
through :meth:`RequestTable.move` (checked against the allowed source states
when ``debug`` is on -- the tests run that way).  The dictionaries of the
in-flight states live here, so ``Gateway.local`` / ``remote_out`` are this
table's.  Threads: INBOX is entered by ingest threads under the inbox lock
before the message is visible to anyone else; a queued message removed by
an API / peer thread (``qm.on_remove``) leaves QUEUED there -- the native
queue's removal is atomic, so it and a dispatch pop never both win (the
pop may then fill less than the tick plan granted; the exchange sends empty
rows for the difference, ``ExchangeMixin._dispatch_global``).  All other
transitions run on the serve loop.

Cancellation is a tombstone: ``tomb`` holds the requests a cancel was asked
for (any thread, under the gateway's cancel lock) and not yet ended.  The
serve loop ends them where they are (``Gateway._process_cancels``) and every
re-entry point -- enqueue after preprocess, requeue, retry scheduling,
dispatch pops, held-turn admission, a completion or hand-back from a GPU --
checks it first, so a request never re-enters service after a cancel was
acknowledged.  The reference's removal surface: `api/handlers.go:622-658`,
`docs/api.md:240-261`; its per-state stats, `internal/priorityqueue/queue.go:197-211`.
"""
from __future__ import annotations

import os
from typing import Dict, Iterable, Optional, Sequence, Tuple

NONE, INBOX, PREPROCESS, QUEUED, RETRY, HELD, LOCAL, REMOTE = range(8)
NAMES = ("none", "inbox", "preprocess", "queued", "retry", "held", "local", "remote")

# the states each state may be entered from (debug checks)
_FROM = {
    INBOX: (NONE,),
    PREPROCESS: (INBOX,),
    QUEUED: (PREPROCESS, QUEUED, RETRY, HELD, LOCAL, REMOTE, NONE),   # NONE: an admin requeue
    # (NONE as a source of the dispatch states: a message an admin path put
    # back into a tier directly -- a dead-letter requeue, a snapshot restore)
    RETRY: (LOCAL, REMOTE, HELD, QUEUED),
    HELD: (QUEUED, NONE),
    LOCAL: (QUEUED, HELD, NONE),
    REMOTE: (QUEUED, NONE),
    NONE: (INBOX, PREPROCESS, QUEUED, RETRY, HELD, LOCAL, REMOTE, NONE),
}


class LifecycleError(AssertionError):
    """A transition from a state it may not come from (debug mode)."""


class RequestTable:
    def __init__(self, debug: Optional[bool] = None):
        self.debug = bool(int(os.environ.get("LLMQ_LIFECYCLE_DEBUG", "0"))) if debug is None else bool(debug)
        self.local: Dict[int, object] = {}          # handle -> msg dispatched to my engine (my origin)
        self.remote_out: Dict[int, object] = {}     # handle -> msg I sent to another rank
        self.tomb: Dict[int, object] = {}           # handle -> msg: cancel asked, not yet ended
        self.ended_cancelled = 0

    # ------------------------------------------------------------------ transitions
    def move(self, m, to: int) -> None:
        if self.debug and m.lc not in _FROM[to]:
            raise LifecycleError(f"message {m.id!r}: {NAMES[m.lc]} -> {NAMES[to]}")
        m.lc = to

    def move_many(self, msgs: Iterable, to: int) -> None:
        if self.debug:
            ok = _FROM[to]
            for m in msgs:
                if m.lc not in ok:
                    raise LifecycleError(f"message {m.id!r}: {NAMES[m.lc]} -> {NAMES[to]}")
                m.lc = to
            return
        for m in msgs:
            m.lc = to

    def to_local(self, m) -> None:
        self.move(m, LOCAL)
        self.local[m.handle] = m

    def to_remote(self, m) -> None:
        self.move(m, REMOTE)
        self.remote_out[m.handle] = m

    def end(self, m) -> None:
        """The request ended (whatever way): out of every in-flight map."""
        self.local.pop(m.handle, None)
        self.remote_out.pop(m.handle, None)
        self.tomb.pop(m.handle, None)
        self.move(m, NONE)

    # ------------------------------------------------------------------ cancellation
    def cancelled(self, m) -> bool:
        return bool(self.tomb) and m.handle in self.tomb

    def split_cancelled(self, msgs: Sequence, extra: Optional[Sequence] = None) -> Tuple[list, list, Optional[list]]:
        """(live, cancelled, extra of the live) -- ``extra`` is a parallel
        sequence (e.g. tier indices) filtered the same way."""
        if not self.tomb:
            return list(msgs), [], (list(extra) if extra is not None else None)
        live, dead, ex = [], [], ([] if extra is not None else None)
        for k, m in enumerate(msgs):
            if m.handle in self.tomb:
                dead.append(m)
            else:
                live.append(m)
                if ex is not None:
                    ex.append(extra[k])
        return live, dead, ex

    # ------------------------------------------------------------------ views
    @staticmethod
    def census(msgs: Iterable) -> Dict[str, int]:
        """Requests per state among ``msgs`` (tests / debugging)."""
        out = {n: 0 for n in NAMES}
        for m in msgs:
            out[NAMES[m.lc]] += 1
        return out
