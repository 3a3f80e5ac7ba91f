"""Serve-loop health of ``GatewayApp`` (split out of app.py): the stall
watchdog, its escalation to a fatal exit for a launcher restart, and the
``/health`` answer.  The reference's health is an LB
loop that always reports healthy (`internal/loadbalancer/load_balancer.go:561-616`)."""
from __future__ import annotations

import time
from typing import Tuple


class HealthMixin:
    def _stall_watchdog(self) -> None:
        """``server.stall_dump_after``: the serve loop has completed no tick
        for that long while requests wait -> one error log and a dump of
        every thread's stack (faulthandler, stderr), and the process reports
        itself unhealthy (``/health`` 503, also on the C++ front door) until
        ticks resume.  ``server.stall_fatal_after``: still no tick -> the
        stall is fatal (``self.fatal``; ``cli serve`` exits non-zero so the
        launcher starts a fresh incarnation -- a stalled rank used to keep
        answering ``/health`` 200 forever)."""
        import faulthandler
        gw = self.gateway
        limit = self.cfg.server.stall_dump_after / 1e9
        fatal = self.cfg.server.stall_fatal_after / 1e9
        period = min(1.0, limit / 4) if limit > 0 else min(1.0, fatal / 4)
        last, since, dumped = -1, time.monotonic(), False
        while not self._stop.wait(period):
            t = gw.counters["ticks"]
            now = time.monotonic()
            if t != last:
                last, since, dumped = t, now, False
                self._set_stalled("")
                continue
            # requests still in the inbox wait too (a loop stuck before its
            # ingest never moves them into the queues)
            waiting = (gw.pending() + gw.inbox_size() + gw.preprocessing()
                       + (gw.engine.inflight() if gw.engine is not None else 0))
            if waiting <= 0:
                since = now                  # an idle loop may sleep; only a stall with work counts
                continue
            if limit > 0 and not dumped and now - since >= limit:
                dumped = True
                self._set_stalled(f"serve loop stalled: no tick for {now - since:.0f} s while {int(waiting)} "
                                  f"requests wait")
                self.log.error("serve loop stalled: no tick while requests wait; dumping thread stacks",
                               rank=gw.rank, stalled_s=round(now - since, 1), waiting=int(waiting), ticks=int(t))
                faulthandler.dump_traceback(all_threads=True)
            if fatal > 0 and now - since >= fatal:
                err = RuntimeError(f"rank {gw.rank}: serve loop completed no tick for {now - since:.0f} s while "
                                   f"{int(waiting)} requests waited (server.stall_fatal_after)")
                self._set_stalled(str(err))
                self.log.error("serve loop stall is fatal; exiting for a restart", rank=gw.rank,
                               stalled_s=round(now - since, 1), waiting=int(waiting))
                if not dumped:
                    faulthandler.dump_traceback(all_threads=True)
                if self.fatal is None:
                    self.fatal = err
                self._stop.set()
                return

    def _set_stalled(self, reason: str) -> None:
        """Health of this process's serve loop: "" = ticking."""
        if reason == self.stalled:
            return
        self.stalled = reason
        fd = self.front_door
        if fd is not None and hasattr(fd, "set_health"):
            fd.set_health(not reason, reason)

    def health(self) -> Tuple[bool, str]:
        """(ok, reason) for ``/health``: false while the serve loop is stalled
        (``server.stall_dump_after``) or after a fatal error (the process is
        on its way out)."""
        if self.fatal is not None:
            return False, f"fatal: {self.fatal}"
        if self.stalled:
            return False, self.stalled
        return True, ""

