"""Conversation affinity of the gateway (``Gateway`` mixin): where a
dialog's KV lives (home GPU), the per-(home GPU, tier) pin counts every rank
publishes to the planner, the handles of queued turns homed elsewhere, and
the KV-migration orders and their execution (``parallel.migration``).
The reference's only affinity is a session map keyed on a ``sessionID`` no
caller passes (`internal/loadbalancer/load_balancer.go:233-240`); here the
key is the conversation id and the target is the GPU holding its KV.

Threads: the pin counts and the homed-away set are also changed from API /
peer threads (``qm.on_remove`` when a queued turn is deleted), so ``_pin``
and ``_skip_away`` hold ``_pin_lock``; everything else runs on the serve
loop."""
from __future__ import annotations

from typing import Dict, List, Tuple

import numpy as np

from ..backend.engine import Request
from ..models.message import Message
from ..parallel import planner
from .descriptors import conv_key


class AffinityMixin:
    def _remember_dialog(self, m: Message, gpu: int, tokens=None) -> None:
        """Completion of a conversation turn: its home GPU (KV residency) and
        the dialog tokens a non-resident replay needs -- exactly what the
        home GPU's parked KV holds for the turn: its prompt (as the engine
        took it) and every generated id but the last (never fed back).
        ``tokens``: the turn's generated ids, read back with the step that
        sampled them (``Request.out_tokens``; carried in the K_DONE record
        when another GPU ran it).  Without them (a backend that keeps no ids)
        placeholders keep the replay's cost right."""
        cid = m.conversation_id
        if not cid:
            return
        self.conv_home[cid] = gpu
        self.conv_home.move_to_end(cid)
        p = np.asarray(m.prompt_ids if m.prompt_ids is not None else [], dtype=np.uint32)[:self.prompt_cap]
        p = p.astype(np.int64).astype(np.int32)
        if not len(p):
            p = np.zeros(1, dtype=np.int32)                   # (the engine's stand-in for an empty prompt)
        h = self.conv_hist.get(cid)
        g = max(0, self.gen_tokens - 1)
        real = tokens is not None and len(tokens) >= g
        gen = np.asarray(tokens, dtype=np.int32)[:g] if real else np.zeros(g, dtype=np.int32)
        self.counters["dialog_ids_real" if real else "dialog_ids_placeholder"] += 1
        add = np.concatenate([p, gen])
        h = add if h is None else np.concatenate([h, add])[-self.history_cap:]
        self.conv_hist[cid] = h
        self.conv_hist.move_to_end(cid)
        while len(self.conv_home) > self.max_dialogs:
            self.conv_home.popitem(last=False)
        while len(self.conv_hist) > self.max_dialogs:
            self.conv_hist.popitem(last=False)

    def _pin(self, m: Message, delta: int) -> None:
        """Count a queued request against its (home GPU, tier) pin.  The key
        it was counted under is remembered on the message and released
        exactly (the conversation may be re-homed -- migration, a completed
        turn elsewhere -- while this turn waits, and recomputing the home at
        pop time would decrement the wrong GPU and leave the old one
        inflated for good).  Removals also arrive from API and peer-query
        threads (``qm.on_remove``), hence the lock."""
        if delta < 0:
            with self._pin_lock:
                k = m.pin_key
                if k >= 0:
                    h, t = divmod(k, planner.NTIERS)
                    if h < self.world:
                        self.pinned[h, t] = max(0, int(self.pinned[h, t]) - 1)
                    m.pin_key = -1
                    self._away.discard(m.handle)
            return
        if m.pin_key >= 0:
            return                                   # already counted
        h = self._home(m)
        if 0 <= h < self.world:
            t = self.tier_of_queue.get(m.queue_name, 2) if m.tier < 0 else m.tier
            t = min(max(int(t), 0), planner.NTIERS - 1)
            with self._pin_lock:
                self.pinned[h, t] += 1
                m.pin_key = h * planner.NTIERS + t
                if h != self.rank:
                    self._away.add(m.handle)

    def _skip_away(self):
        """Handles of queued turns homed on another GPU: a rank admitting into
        its own GPU leaves them queued, in place, for the tick's plan."""
        if not self._away:
            return None
        with self._pin_lock:
            return np.fromiter(self._away, dtype=np.int64, count=len(self._away))

    def _avoid_home(self, pool: List[Message], room: List[int], dest: Dict[int, List[Message]]) -> List[Message]:
        """Place each homed turn on a GPU other than its home (bench knob);
        returns the turns still unplaced."""
        left = []
        for m in pool:
            h = self._home(m)
            if h < 0:
                left.append(m)
                continue
            js = [j for j in range(self.world) if j != h and room[j] > 0]
            if not js:
                left.append(m)
                continue
            j = max(js, key=lambda x: room[x])
            dest[j].append(m)
            room[j] -= 1
        return left

    def awaiting_kv(self) -> int:
        """Turns dispatched here that wait for their KV (next tick, or an
        RCCL transfer still in flight) or for their dialog history."""
        return (sum(len(v) for v in self._await_kv.values())
                + sum(len(v) for v in self._await_import.values()) + len(self._await_hist))

    def _dialog_context(self, m: Message):
        """(history, prefix) a replay of ``m``'s dialog prefills: the real
        token history (``conv_hist``) and, when the conversation's window
        was evicted, its N5 salient tokens as compressed context."""
        cid = m.conversation_id
        if not cid:
            return None, None
        hist = self.conv_hist.get(cid)
        pre = None
        if self.state_manager is not None and hasattr(self.state_manager, "summary_tokens"):
            sal = self.state_manager.summary_tokens(cid)
            if sal:
                pre = np.asarray(sal, dtype=np.uint32).astype(np.int64).astype(np.int32)
        return hist, pre

    def _plan_migrations(self, dest: Dict[int, List[Message]]) -> Dict[int, int]:
        """Turns placed on a GPU other than their (alive) home GPU move their
        dialog KV with them: record the order (sent to the home GPU in the next
        tick's all_to_all) and re-home the conversation now."""
        out: Dict[int, int] = {}
        if self.migrator is None or not self.kv_migrate:
            return out
        W = self.world
        seen = set()
        for j in range(W):
            for m in dest[j]:
                if not m.conversation_id:
                    continue
                h = self._home(m)
                if not 0 <= h < W or h == j or h in self.unhealthy_peers or (h == self.rank and not self.healthy):
                    continue
                ck = conv_key(m.conversation_id)
                if ck in seen:
                    continue                               # one move per conversation per tick
                seen.add(ck)
                out[id(m)] = h
                self._mig_out.append((ck, h, j))
                self.conv_home[m.conversation_id] = j
                if m.metadata and "home_gpu" in m.metadata:
                    m.metadata["home_gpu"] = j
        return out

    def _migrate(self, loads: np.ndarray, src_orders: List[Tuple[int, int, int]],
                 held: Dict[int, List[Tuple[Request, int]]]) -> List[Request]:
        """Execute last tick's migration orders -- as the home GPU
        (``src_orders``) and as the destination (the turns ``held`` for their
        KV) -- and return the held turns that may be admitted now: KV landed
        (synchronous data plane, or an RCCL transfer of an earlier tick that
        completed), or nothing will come (dialog replay).  Turns whose KV is
        still in flight on the device wait in ``_await_import``.

        A home GPU that is down (by this tick's loads, the view every rank
        shares) is not asked; a home only sends to a destination that is up
        AND still wants the KV (the header exchange matches both sides, so a
        destination that dropped its held turns never leaves an unmatched
        RCCL send behind).  Every rank joins the header collective on a
        migration tick (``L_MIGBUSY`` set anywhere)."""
        W = self.world
        ready: List[Request] = []
        if self.migrator is None:
            for rs in held.values():
                ready.extend(r for r, _h in rs)
            return ready
        up = [bool(x) for x in loads[:, planner.L_HEALTHY]]
        result: Dict[int, int] = {}
        wanted = set()
        if loads[:, planner.L_MIGBUSY].any():
            orders = [(c, d) for c, h, d in src_orders if up[self.rank] and 0 <= d < W and up[d]]
            wants = []
            if up[self.rank]:
                for ck, rs in held.items():
                    # ONE source per conversation: the home its latest held
                    # turn names.  Wanting from two homes could land a stale
                    # import over the slot a replay of the other wrote
                    h = next((h for _, h in reversed(rs) if 0 <= h < W and h != self.rank and up[h]), -1)
                    if h >= 0:
                        wants.append((ck, h))
                        wanted.add(ck)
            result = self.migrator.execute(orders, wants, self.engine, self.rank)
            if orders or wants:
                self.epoch += 1
        for ck, rs in held.items():
            if ck in wanted and ck not in result:
                self._await_import.setdefault(ck, []).extend(rs)     # in flight on the device
                continue
            got = result.get(ck, 0)
            for r, _h in rs:
                self.counters["kv_migrated" if got > 0 else "kv_migrate_replays"] += 1
                ready.append(r)
        for ck, n in self.migrator.poll(self.engine).items():
            for r, _h in self._await_import.pop(ck, []):
                self.counters["kv_migrated"] += 1
                ready.append(r)
        return ready

    def _home(self, m: Message, effective: bool = False) -> int:
        """GPU holding the conversation's KV (-1: none).  ``effective``: -1
        as well when that GPU is unhealthy (the conversation is re-homed)."""
        h = m.metadata.get("home_gpu") if m.metadata else None
        if h is None and self.state_manager is not None and m.conversation_id:
            h = self.state_manager.home_gpu(m.conversation_id)
            if h is not None and h < 0:
                h = None
        if h is None and m.conversation_id:
            h = self.conv_home.get(m.conversation_id)
        h = -1 if h is None else int(h)
        if effective and (h in self.unhealthy_peers or h in self.excluded_peers
                          or (h == self.rank and not self.healthy)):
            return -1
        return h
