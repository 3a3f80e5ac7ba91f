"""Deterministic global dispatch / rebalance plan (N10).

Every rank all-gathers the same ``[world, LOAD_WIDTH]`` load matrix and runs
``plan_dispatch`` on it with the same ``PlanState``, so all ranks agree on the
plan without a leader round-trip (collectives are issued in the same order
everywhere).  The plan answers: how many tier-t requests does router i hand
to backend j this tick?

Policy (the gateway-level generalisation of the reference's strict-priority
poll, `cmd/queue-manager/main.go:112-124`, plus the anti-starvation it lacks,
and of its per-request endpoint choice, `internal/loadbalancer/load_balancer.go:234-294`):
  1. tiers whose oldest request is past its ``max_wait_time`` are served
     first (aging), then tiers in priority order;
  2. within a tier, scarce capacity is split between routers in proportion to
     their demand (largest remainder, ties to the lower rank);
  3. conversations homed on GPU j (KV residency, ``L_PIN``) go to j while it
     has room -- the reference's session affinity (`load_balancer.go:501-558`)
     made real: the KV of the dialog lives there;
  4. the rest of the tier's grant is spread over the ELIGIBLE GPUs by the
     configured ``loadbalancer.algorithm`` -- the reference's selectors
     (`load_balancer.go:381-498`) applied to a batch of identical requests:
       * round_robin: a cursor over the GPUs (persisted in ``PlanState``),
         one request per GPU per turn -> an exact 1/W split over time;
       * least_connections: water-filling on slot utilisation
         (in-flight + assigned) / slots, ties to lower HBM use, then index;
       * weighted_random: multinomial draw (seeded by the shared tick
         counter, identical on every rank) with weight = endpoint weight x
         free-slot fraction x free-HBM fraction;
       * adaptive_load: water-filling on the reference's score
         0.4 load + 0.4 min(rt_s, 10) + 0.2 (10 err) plus an HBM-pressure
         term; the reference's 10 % runner-up exploration is a seeded draw;
       * local_first (MI355X addition): every router keeps what its own GPU
         can take, the excess goes least-connections;
  5. the per-GPU counts from step 4 are matched to routers LOCAL FIRST
     (a router's requests go to its own GPU when the strategy sends work
     there), so the all_to_all only carries the imbalance.
A GPU is eligible when it is healthy, not excluded by any rank's balancer
view (parked by the autoscaler, removed, or marked unhealthy by an operator:
``L_EXCLUDE`` bitmask) and not shutting down.  Tier 0 may use every free slot
(the realtime lane, ``L_SLOTS``); the other tiers only the next step's prefill
headroom (``L_FREE``).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional, Sequence

import numpy as np

MAX_WORLD = 8
NTIERS = 4
# ---- load vector layout (int64)
L_FREE, L_INFLIGHT = 0, 1        # admits the next step's prefill headroom takes; slots in use
L_DEPTH = 2                      # 4 tiers: 2..5 queued (within tier budget)
L_AGE_US = 6                     # 4 tiers: 6..9 (oldest head wait, microseconds)
# MiB of the GPU's serving footprint in use / in total: model weights + LIVE
# KV (active contexts + parked dialogs) over weights + the KV pool.  The pool
# is preallocated, so allocator or amd-smi figures never move; resident KV is
# what varies between GPUs and what placement should avoid filling
L_HBM_USED, L_HBM_TOTAL = 10, 11
L_HEALTHY, L_EPOCH = 12, 13      # epoch: KV migrations this rank has completed
L_STOP = 14                      # the rank is shutting down: every rank leaves after this same tick
L_SLOTS = 15                     # free batch slots (realtime lane capacity)
L_DONE = 16                      # [16 + r] completion records this rank owes router r
L_PIN = L_DONE + MAX_WORLD       # [24 + 4 j + t] queued tier-t requests here whose conversation is homed on GPU j
L_EXCLUDE = L_PIN + MAX_WORLD * NTIERS   # 56: bitmask of GPUs this rank's balancer view excludes
L_RT_US = L_EXCLUDE + 1          # EWMA service time (admit -> done) on this GPU, microseconds
L_ERR_PPM = L_EXCLUDE + 2        # EWMA backend error rate, parts per million
L_SLOTS_TOTAL = L_EXCLUDE + 3    # batch slots of this GPU
L_MIGBUSY = L_EXCLUDE + 4        # this rank takes part in a KV migration this tick (header collective)
L_KV_TOKENS = L_EXCLUDE + 5      # KV positions resident on this GPU (active + parked dialogs)
L_KV_CAP = L_EXCLUDE + 6         # KV positions the pool holds (slots x max_ctx)
L_WEIGHT = L_EXCLUDE + 8         # [64 + j] endpoint weight of GPU j in this rank's balancer (rank 0 row is used)
# KV migration: [72 + h] = K_MIGRATE rows this router sends rank h in THIS
# tick's all_to_all (orders decided last tick; h = the conversation's home,
# which sends the KV) -- announced here so every receiver knows its row count
L_MIGC = L_WEIGHT + MAX_WORLD
LOAD_WIDTH = L_MIGC + MAX_WORLD

STRATEGIES = ("round_robin", "least_connections", "weighted_random", "adaptive_load", "local_first")


def make_load(free: int, inflight: int, depth: Sequence[int], age_us: Sequence[int], hbm_used_mib: int = 0,
              hbm_total_mib: int = 0, healthy: bool = True, epoch: int = 0,
              done_for: Sequence[int] = (), pinned=None, stopping: bool = False,
              slots_free: Optional[int] = None, slots_total: int = 0, exclude_mask: int = 0,
              rt_us: int = 0, err_ppm: int = 0, weights: Sequence[int] = (),
              migrate_rows: Sequence[int] = (), migrate_busy: bool = False, kv_tokens: int = 0,
              kv_capacity: int = 0) -> np.ndarray:
    """``pinned``: [W, 4] (home GPU x tier) queued counts, or a [W] vector
    (all counted as tier 2, normal -- legacy callers)."""
    v = np.zeros(LOAD_WIDTH, dtype=np.int64)
    v[L_FREE], v[L_INFLIGHT] = free, inflight
    v[L_DEPTH:L_DEPTH + NTIERS] = list(depth)[:NTIERS]
    v[L_AGE_US:L_AGE_US + NTIERS] = list(age_us)[:NTIERS]
    v[L_HBM_USED], v[L_HBM_TOTAL], v[L_HEALTHY], v[L_EPOCH] = hbm_used_mib, hbm_total_mib, int(healthy), epoch
    v[L_STOP] = int(stopping)
    v[L_SLOTS] = free if slots_free is None else slots_free
    for r, n in enumerate(done_for):
        v[L_DONE + r] = n
    if pinned is not None:
        p = np.asarray(pinned, dtype=np.int64)
        if p.ndim == 1:
            q = np.zeros((len(p), NTIERS), dtype=np.int64)
            q[:, 2] = p
            p = q
        for j in range(min(MAX_WORLD, p.shape[0])):
            v[L_PIN + NTIERS * j:L_PIN + NTIERS * (j + 1)] = p[j, :NTIERS]
    v[L_EXCLUDE] = exclude_mask
    v[L_RT_US], v[L_ERR_PPM], v[L_SLOTS_TOTAL] = rt_us, err_ppm, slots_total
    for j, w in enumerate(list(weights)[:MAX_WORLD]):
        v[L_WEIGHT + j] = w
    for h, n in enumerate(list(migrate_rows)[:MAX_WORLD]):
        v[L_MIGC + h] = n
    v[L_MIGBUSY] = int(bool(migrate_busy))
    v[L_KV_TOKENS], v[L_KV_CAP] = kv_tokens, kv_capacity
    return v


@dataclass
class PlanState:
    """Plan inputs that persist across ticks; every rank holds an identical
    copy and advances it identically (``plan_dispatch`` mutates it)."""
    strategy: str = "least_connections"
    rr_cursor: int = 0
    tick: int = 0
    seed: int = 0x5EED

    def __post_init__(self):
        if self.strategy not in STRATEGIES:
            # the reference falls back to round robin for unknown names
            # (`load_balancer.go:272-275`; its shipped "weighted_round_robin")
            self.strategy = "round_robin"


def _split(cap: int, demand: np.ndarray) -> np.ndarray:
    tot = int(demand.sum())
    if tot <= cap:
        return demand.copy()
    if cap <= 0:
        return np.zeros_like(demand)
    exact = demand.astype(np.float64) * cap / tot
    g = np.floor(exact).astype(np.int64)
    rem = cap - int(g.sum())
    order = sorted(range(len(demand)), key=lambda i: (-(exact[i] - g[i]), i))
    for i in order[:rem]:
        g[i] += 1
    return np.minimum(g, demand)


def _waterfill(n: int, cap: np.ndarray, level0: np.ndarray, slope: np.ndarray, tie: np.ndarray) -> np.ndarray:
    """Place ``n`` identical units on bins with capacity ``cap`` so the bins'
    levels ``level0 + slope * units`` rise evenly: the batch equivalent of
    giving each unit to the currently lowest bin (ties by ``tie``, then
    index).  Exact and O(W^2) in plain Python floats (W <= 8 bins: numpy
    per-call overhead would dominate): the fill level is found between the
    bins' start/saturation breakpoints, whole units are taken below it and
    the remainder goes to the lowest next levels."""
    W = len(cap)
    capl = [max(0, int(c)) for c in cap]
    l0 = [float(x) for x in level0]
    sl = [max(float(x), 1e-12) for x in slope]
    n = min(int(n), sum(capl))
    out = [0] * W
    if n <= 0:
        return np.zeros(W, dtype=np.int64)
    live = [j for j in range(W) if capl[j] > 0]
    pts = sorted({l0[j] for j in live} | {l0[j] + sl[j] * capl[j] for j in live})

    def units(L):                      # continuous units below level L
        return sum(min(capl[j], max(0.0, (L - l0[j]) / sl[j])) for j in live)

    L = pts[-1]
    for k in range(1, len(pts)):
        if units(pts[k]) >= n:
            lo, hi = pts[k - 1], pts[k]
            ulo = units(lo)
            rate = sum(1.0 / sl[j] for j in live if l0[j] <= lo and l0[j] + sl[j] * capl[j] > lo)
            L = lo + (n - ulo) / rate if rate > 0 else hi
            break
    for j in live:                     # whole units strictly below L
        k = int(np.ceil((L - l0[j]) / sl[j] - 1e-9))
        out[j] = min(capl[j], max(0, k))
    over = sum(out) - n
    while over > 0:                    # integer rounding: undo the last-placed units
        j = max((j for j in live if out[j] > 0), key=lambda j: (l0[j] + sl[j] * (out[j] - 1), float(tie[j]), j))
        out[j] -= 1
        over -= 1
    rem = n - sum(out)
    while rem > 0:
        cand = [j for j in live if out[j] < capl[j]]
        if not cand:
            break
        j = min(cand, key=lambda j: (l0[j] + sl[j] * out[j], float(tie[j]), j))
        out[j] += 1
        rem -= 1
    return np.asarray(out, dtype=np.int64)


def _targets(G: int, cap: np.ndarray, loads: np.ndarray, assigned: np.ndarray, elig: np.ndarray,
             st: PlanState, t: int, demand_local: np.ndarray) -> np.ndarray:
    """Per-GPU counts for ``G`` units of tier t under the strategy."""
    W = len(cap)
    cap = np.where(elig, cap, 0)
    G = int(min(G, cap.sum()))
    if G <= 0:
        return np.zeros(W, dtype=np.int64)
    slots = np.maximum(loads[:, L_SLOTS_TOTAL], 1).astype(np.float64)
    inflight = (loads[:, L_INFLIGHT] + assigned).astype(np.float64)
    hbm_tot = loads[:, L_HBM_TOTAL].astype(np.float64)
    hbm_frac = np.where(hbm_tot > 0, loads[:, L_HBM_USED] / np.maximum(hbm_tot, 1), 0.0)
    s = st.strategy
    if s == "round_robin":
        # the cursor walks the FULL GPU list (a GPU leaving does not shift
        # everybody's turn, as in balancer.load_balancer); per pass every
        # live GPU gets left // live, the remainder goes to the next ones
        # from the cursor, which then moves past the last of them
        out = np.zeros(W, dtype=np.int64)
        left = G
        while left > 0:
            live = [(st.rr_cursor + k) % W for k in range(W) if out[(st.rr_cursor + k) % W] < cap[(st.rr_cursor + k) % W]]
            if not live:
                break
            q, r = divmod(left, len(live))
            for k, j in enumerate(live):
                add = min(q + (1 if k < r else 0), int(cap[j] - out[j]))
                out[j] += add
                left -= add
            if r:
                st.rr_cursor = (live[r - 1] + 1) % W
        return out
    if s == "weighted_random":
        w0 = loads[0, L_WEIGHT:L_WEIGHT + W].astype(np.float64)
        w0 = np.where(w0 > 0, w0, 1.0)
        free = np.clip(slots - inflight, 0, None) / slots
        w = np.where(cap > 0, w0 * free * (1.0 - hbm_frac), 0.0)
        if w.sum() <= 0:
            w = (cap > 0).astype(np.float64)
        rng = np.random.default_rng([st.seed, st.tick, t])
        out = np.minimum(rng.multinomial(G, w / w.sum()), cap)
        short = G - int(out.sum())
        if short > 0:                    # overflow of a full GPU: least-connections
            out += _waterfill(short, cap - out, inflight / slots + out / slots, 1.0 / slots, hbm_frac)
        return out
    if s == "adaptive_load":
        rt_s = np.minimum(loads[:, L_RT_US] / 1e6, 10.0)
        err = loads[:, L_ERR_PPM] / 1e6
        score = 0.4 * inflight / slots + 0.4 * rt_s + 0.2 * (10.0 * err) + 0.2 * hbm_frac
        out = _waterfill(G, cap, score, 0.4 / slots, hbm_frac)
        # the reference sends 10 % of picks to the runner-up (exploration)
        live = np.flatnonzero(cap > 0)
        if len(live) > 1 and G >= 10:
            rng = np.random.default_rng([st.seed, st.tick, t, 1])
            k = int(rng.binomial(G, 0.1))
            best = live[np.argsort(score[live], kind="stable")]
            a, b = int(best[0]), int(best[1])
            k = min(k, int(out[a]), int(cap[b] - out[b]))
            out[a] -= k
            out[b] += k
        return out
    if s == "local_first":
        out = np.minimum(demand_local, cap)
        rest = G - int(out.sum())
        if rest > 0:
            out += _waterfill(rest, cap - out, (inflight + out) / slots, 1.0 / slots, hbm_frac)
        return out
    # least_connections (default)
    return _waterfill(G, cap, inflight / slots, 1.0 / slots, hbm_frac)


def eligible(loads: np.ndarray) -> np.ndarray:
    W = loads.shape[0]
    mask = 0
    for i in range(W):
        mask |= int(loads[i, L_EXCLUDE])
    ex = np.array([(mask >> j) & 1 for j in range(W)], dtype=bool)
    return (loads[:, L_HEALTHY] > 0) & (loads[:, L_STOP] == 0) & ~ex


def plan_dispatch(loads: np.ndarray, aging_us: Sequence[int], state: Optional[PlanState] = None) -> np.ndarray:
    """Returns quota[i, j, t] (int64, shape [W, W, 4]).  ``state`` defaults
    to least-connections with no memory across ticks.  (Inner loops run on
    Python ints: W <= 8, so numpy scalar indexing would dominate.)"""
    st = state if state is not None else PlanState()
    loads = np.asarray(loads, dtype=np.int64)
    W = loads.shape[0]
    elig = eligible(loads)
    el = [bool(x) for x in elig]
    cap_head = [int(loads[j, L_FREE]) if el[j] else 0 for j in range(W)]
    cap_slot = [max(int(loads[j, L_SLOTS]), int(loads[j, L_FREE])) if el[j] else 0 for j in range(W)]
    depth = loads[:, L_DEPTH:L_DEPTH + NTIERS].tolist()
    age = loads[:, L_AGE_US:L_AGE_US + NTIERS].tolist()
    pin = loads[:, L_PIN:L_PIN + NTIERS * W].reshape(W, W, NTIERS).tolist()      # [router][home][tier]
    quota = [[[0] * NTIERS for _ in range(W)] for _ in range(W)]
    assigned = [0] * W
    overdue = [t for t in range(NTIERS)
               if aging_us[t] > 0 and any(age[i][t] > aging_us[t] for i in range(W))
               and sum(depth[i][t] for i in range(W)) > 0]
    order = overdue + [t for t in range(NTIERS) if t not in overdue]
    for t in order:
        cap = list(cap_slot) if t == 0 else [min(a, b) for a, b in zip(cap_slot, cap_head)]
        total_cap = sum(cap)
        if total_cap <= 0:
            continue
        dem = [depth[i][t] for i in range(W)]
        if sum(dem) <= 0:
            continue
        left = [int(x) for x in _split(total_cap, np.asarray(dem, dtype=np.int64))]
        used = [0] * W
        # 3) KV-residency affinity
        for i in range(W):
            if left[i] <= 0:
                continue
            for j in range(W):
                take = min(left[i], pin[i][j][t], cap[j])
                if take > 0:
                    quota[i][j][t] += take
                    cap[j] -= take
                    pin[i][j][t] -= take
                    left[i] -= take
                    used[j] += take
                    if left[i] <= 0:
                        break
        # 4) strategy: per-GPU counts for the rest of the tier's grant
        G = sum(left)
        if G > 0:
            tgt = [int(x) for x in _targets(G, np.asarray(cap, dtype=np.int64), loads,
                                            np.asarray([a + u for a, u in zip(assigned, used)], dtype=np.int64),
                                            elig, st, t,
                                            np.asarray(left, dtype=np.int64))]
            # 5) match routers to those counts, local first
            for i in range(W):
                take = min(left[i], tgt[i])
                if take > 0:
                    quota[i][i][t] += take
                    tgt[i] -= take
                    left[i] -= take
                    used[i] += take
            for i in range(W):
                for j in range(W):
                    if left[i] <= 0:
                        break
                    take = min(left[i], tgt[j])
                    if take > 0:
                        quota[i][j][t] += take
                        tgt[j] -= take
                        left[i] -= take
                        used[j] += take
        for j in range(W):
            cap_slot[j] = max(cap_slot[j] - used[j], 0)
            # a realtime request's prefill goes first, so it eats headroom too
            cap_head[j] = max(cap_head[j] - used[j], 0)
            assigned[j] += used[j]
    st.tick += 1
    return np.asarray(quota, dtype=np.int64).reshape(W, W, NTIERS)
