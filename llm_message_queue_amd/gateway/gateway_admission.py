"""Own-GPU admission between the per-tick collectives (``Gateway`` mixin):
the realtime lane, admission into this rank's own free slots while a
collective is in flight (only into the capacity held back from the published
load), and the extra local forward a faster GPU takes while its peers are
behind.  Serve-loop only.  The reference dispatches from a ticker that
batch-pops each queue every ``ProcessInterval``
(`internal/priorityqueue/worker.go:110-130`)."""
from __future__ import annotations

import time
from typing import Sequence

from ..models.message import Message, MessageStatus
from .latency import P_LANE, P_OWN


class OwnAdmissionMixin:
    def _lane_budget(self, taken: int, taken0: int) -> int:
        """How many more tier-0 requests the realtime lane may admit now
        (``taken`` requests, ``taken0`` of them tier 0, already popped)."""
        if not self.realtime_lane or self.engine is None or not self.tiers:
            return 0
        if self.qm.size(self.tiers[0]) <= 0:
            return 0
        room = self.engine.lane_capacity() - taken
        b = self._budgets()[0]
        if b >= 0:
            room = min(room, b - taken0)
        return max(0, room)

    def _admit_between(self) -> int:
        if self.world == 1:
            return self._dispatch_local()
        return self._dispatch_own()

    def _overlap(self, pend) -> None:
        """A collective is in flight (this rank's contribution is published,
        a peer has not reached it yet): keep pulling arrivals and
        preprocessing + enqueueing them instead of idling, so the front end
        never stalls for the slowest GPU.  Admission here uses only the
        capacity this rank held back from its published load (``_reserve``):
        the rest must stay as published until the plan is applied.""" 
        if pend.ready():
            return
        pump = self._pump
        self._in_wait = True
        try:
            self._overlap_loop(pend, pump)
        finally:
            self._in_wait = False

    def _overlap_loop(self, pend, pump) -> None:
        while not pend.ready():
            did = self._while_waiting(pump, admit=False)
            if did and (self._reserve[0] > 0 or self._reserve[1] > 0):
                self._dispatch_own(reserved=True)
            if not did:
                time.sleep(0.0001)

    def _dispatch_own(self, reserved: bool = False) -> int:
        """Multi-rank, between the per-tick collectives: a router admits its
        own queued requests straight into free capacity of its OWN GPU --
        every tier into the next step's prefill headroom (strict priority +
        aging, as the tick's plan would), then the realtime tier into any
        free slot (the realtime lane).  A local placement needs no cross-rank
        decision: the next load vector reports the slots taken, and the plan
        spreads what this GPU cannot take.  So no request waits a whole tick
        for the exchange while its own GPU has room (the
        non-realtime tiers used to dispatch only at the collective, and the
        realtime lane switched off whenever any realtime turn was homed
        elsewhere).  Turns homed on another GPU are passed over in place
        (``pop_tiers(skip=...)``) and left to the planner -- they follow
        their KV -- while the rest of their tier, before or behind them, is
        still admitted here; under round robin / weighted random only the
        realtime lane runs (their rotation is the plan's).
        ``reserved``: while this rank's published load is awaiting the plan,
        admit only into the capacity it held back (``_reserve``)."""
        eng = self.engine
        if (eng is None or not self.healthy or self.stopping or not self.tiers
                or self.rank in self.excluded_peers):
            return 0
        held = self.awaiting_kv()
        nt = len(self.tiers)
        skip = self._skip_away()
        # between publishing its load and popping its grant, a rank may only
        # take what arrived since: the plan grants up to the published depth
        spare = ([max(0, self.qm.size(n_) - d) for n_, d in zip(self.tiers, self._pub_depth)]
                 if self._pub_depth is not None else None)
        n = 0
        head = eng.admit_capacity() - held
        if reserved:
            head = min(head, self._reserve[0])
        if head > 0 and self.plan_state.strategy not in self.ROTATING_STRATEGIES:
            b = self._budgets()
            budgets = [head if b[t] < 0 else min(head, b[t]) for t in range(nt)]
            if spare is not None:
                budgets = [min(x, y) for x, y in zip(budgets, spare)]
            if any(budgets):
                msgs, tier_idx, _e = self.qm.pop_tiers(self.tiers, head, self.aging_ns, budgets, self.lifo_ns, skip)
                tl = [int(t) for t in tier_idx]
                if spare is not None:
                    for t in tl:
                        spare[t] -= 1
                k = self._admit_own(msgs, tl, P_OWN)
                n += k
                self.counters["realtime_local"] += tl.count(0)
                if reserved:
                    self._reserve[0] -= k
        if self.realtime_lane and self.qm.size(self.tiers[0]) > 0:
            room = eng.lane_capacity() - held
            if reserved:
                room = min(room, self._reserve[1])
            b0 = self._budgets()[0]
            if b0 >= 0:
                room = min(room, b0)
            if spare is not None:
                room = min(room, spare[0])
            if room > 0:
                budgets = [0] * nt
                budgets[0] = room
                msgs, _t, _e = self.qm.pop_tiers(self.tiers, room, [0] * nt, budgets, None, skip)
                k = self._admit_own(msgs, [0] * len(msgs), P_LANE)
                self.counters["realtime_local"] += k
                if reserved:
                    self._reserve[1] -= k
                n += k
        return n

    def _admit_own(self, msgs: Sequence[Message], tiers: Sequence[int], path: int = P_OWN) -> int:
        """Admit popped queued requests into this rank's OWN GPU (no
        cross-rank decision: the next load vector reports the slots taken)."""
        if not msgs:
            return 0
        self._popped(msgs, tiers)
        msgs, tiers = self._drop_cancelled(msgs, tiers)
        if not len(msgs):
            return 0
        eng = self.engine
        reqs = []
        for m, t in zip(msgs, tiers):
            self._pin(m, -1)
            m.tier = int(t)
            reqs.append(self._make_request(m, int(t)))
        admitted = eng.admit(reqs)
        now = time.monotonic_ns()
        for r in admitted:
            m = r.meta
            m.dispatched_at = now
            m.status = MessageStatus.PROCESSING
            m.endpoint_id = f"gpu{self.rank}"
            self.table.to_local(m)
            self.inflight_by_tier[r.tier] += 1
        if len(admitted) < len(reqs):              # cannot happen (room was counted); requeue defensively
            got = {id(r) for r in admitted}
            for r in reqs:
                if id(r) not in got:
                    self._requeue(r.meta)
        self._record([r.tier for r in admitted], [r.meta.arrival_ns for r in admitted],
                     [r.meta.enqueued_at for r in admitted], now, [r.meta.popped_ns for r in admitted], path)
        self.counters["dispatched"] += len(admitted)
        return len(admitted)

    # An extra step must carry at least this fraction of the token budget: a
    # forward's GEMM cost is quantised in 256-row tiles, so many small steps
    # would cost more GPU time than the idle they fill.
    EXTRA_STEP_MIN_FRAC = 0.5

    ROTATING_STRATEGIES = ("round_robin", "weighted_random")

    def _extra_local_step(self) -> bool:
        """Multi-rank, before the tick's exchange: if the engine's run-ahead
        queue has room (this GPU finishes its steps faster than the job's
        tick cadence -- a faster GPU than the slowest peer) and a peer has not
        reached the exchange yet (so joining now means waiting), admit this
        rank's own queued requests into its free slots and launch one more
        forward.  Lock-step would otherwise leave the faster GPU idle for the
        speed difference every tick (``lockstep.gpu_busy_frac_by_rank``);
        with it the job serves the SUM of its GPUs' capacities, and the
        planner, seeing the faster GPU's free slots, moves the slower GPUs'
        excess there.  At most one per tick, so a rank always joins the
        exchange promptly; placement of own requests onto the own GPU is what
        least-connections would choose for a GPU with free slots, and is
        skipped for tiers holding turns homed on another GPU and while this
        GPU is parked; under round robin / weighted random the step runs only
        work already admitted.  Engines without an asynchronous device (the
        CPU reference engine runs its forward on the host) never idle, so
        never take one."""
        eng = self.engine
        if (not self.extra_steps or eng is None or not getattr(eng, "async_device", False) or not self.healthy
                or self.stopping or not self.tiers or eng.queued_steps() >= eng.max_inflight):
            return False
        behind = getattr(self.comm, "peers_behind", None)
        if behind is None or not behind():
            return False
        if (self._exclude_mask() >> self.rank) & 1:
            return False
        room = eng.admit_capacity() - self.awaiting_kv()
        # own-GPU admission is what a load-aware strategy picks for a GPU with
        # free slots; round robin / weighted random keep their rotation (the
        # extra step then runs only the work already admitted)
        if room > 0 and self.plan_state.strategy not in self.ROTATING_STRATEGIES:
            b = self._budgets()
            budgets = [room if b[t] < 0 else min(room, b[t]) for t in range(len(self.tiers))]
            if any(budgets):
                msgs, tier_idx, _e = self.qm.pop_tiers(self.tiers, room, self.aging_ns, budgets, self.lifo_ns,
                                                       self._skip_away())
                self.counters["extra_admitted"] += self._admit_own(msgs, [int(t) for t in tier_idx])
        if eng.ready_tokens() < self.EXTRA_STEP_MIN_FRAC * eng.token_budget:
            return False
        try:
            eng.launch()
            self.finish_backend()
        except RuntimeError as e:                   # HIP error / OOM: as in _tick, this GPU leaves placement
            self._set_healthy(False, f"backend error: {e}")
            return False
        self.counters["extra_steps"] += 1
        return True
