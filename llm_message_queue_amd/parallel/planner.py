"""Deterministic global dispatch / rebalance plan (N10).

Every rank all-gathers the same ``[world, LOAD_WIDTH]`` load matrix and runs
``plan_dispatch`` on it, so all ranks agree on the plan without a leader.
The plan answers: how many tier-t requests does router i hand to backend j
this tick?

Policy (the gateway-level generalisation of the reference's strict-priority
poll, `cmd/queue-manager/main.go:112-124`, plus the anti-starvation it lacks):
  1. tiers whose oldest request is past its ``max_wait_time`` are served
     first (aging), then tiers in priority order;
  2. within a tier, scarce capacity is split between routers in proportion to
     their demand (largest remainder, ties to the lower rank);
  3. a router's grant is placed on its LOCAL backend first (no transfer),
     then on the backend with the most free slots (least-connections),
     skipping unhealthy backends; ties go to the lower index.
"""
from __future__ import annotations

from typing import Sequence

import numpy as np

MAX_WORLD = 8
# [16 + r] = completion records this rank owes router r
# [24 + j] = queued requests at this router whose conversation is homed on GPU j
LOAD_WIDTH = 16 + 2 * MAX_WORLD
L_PIN = 16 + MAX_WORLD
L_FREE, L_INFLIGHT = 0, 1
L_DEPTH = 2          # 4 tiers: 2..5
L_AGE_US = 6         # 4 tiers: 6..9 (oldest head wait, microseconds)
L_HBM_USED, L_HBM_TOTAL, L_HEALTHY, L_EPOCH = 10, 11, 12, 13
L_STOP = 14          # the rank is shutting down: every rank leaves after this same tick
L_DONE = 16
NTIERS = 4


def make_load(free: int, inflight: int, depth: Sequence[int], age_us: Sequence[int], hbm_used_mib: int = 0,
              hbm_total_mib: int = 0, healthy: bool = True, epoch: int = 0,
              done_for: Sequence[int] = (), pinned: Sequence[int] = (), stopping: bool = False) -> np.ndarray:
    v = np.zeros(LOAD_WIDTH, dtype=np.int64)
    v[L_FREE], v[L_INFLIGHT] = free, inflight
    v[L_DEPTH:L_DEPTH + NTIERS] = list(depth)[:NTIERS]
    v[L_AGE_US:L_AGE_US + NTIERS] = list(age_us)[:NTIERS]
    v[L_HBM_USED], v[L_HBM_TOTAL], v[L_HEALTHY], v[L_EPOCH] = hbm_used_mib, hbm_total_mib, int(healthy), epoch
    v[L_STOP] = int(stopping)
    for r, n in enumerate(done_for):
        v[L_DONE + r] = n
    for j, n in enumerate(pinned):
        v[L_PIN + j] = n
    return v


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


def plan_dispatch(loads: np.ndarray, aging_us: Sequence[int]) -> np.ndarray:
    """Returns quota[i, j, t] (int64, shape [W, W, 4])."""
    loads = np.asarray(loads, dtype=np.int64)
    W = loads.shape[0]
    cap = np.where(loads[:, L_HEALTHY] > 0, loads[:, L_FREE], 0).astype(np.int64)
    depth = loads[:, L_DEPTH:L_DEPTH + NTIERS].copy()
    age = loads[:, L_AGE_US:L_AGE_US + NTIERS]
    quota = np.zeros((W, W, NTIERS), dtype=np.int64)
    pin = loads[:, L_PIN:L_PIN + W].copy() if loads.shape[1] >= L_PIN + W else np.zeros((W, W), np.int64)
    overdue = [t for t in range(NTIERS)
               if aging_us[t] > 0 and (age[:, t] > aging_us[t]).any() and depth[:, t].sum() > 0]
    order = overdue + [t for t in range(NTIERS) if t not in overdue]
    for t in order:
        total_cap = int(cap.sum())
        if total_cap <= 0:
            break
        grant = _split(total_cap, depth[:, t])
        for i in range(W):
            g = int(grant[i])
            if g <= 0:
                continue
            # KV-residency affinity: conversations homed on GPU j go to j
            for j in range(W):
                if g <= 0:
                    break
                take = min(g, int(pin[i, j]), int(cap[j]))
                if take > 0:
                    quota[i, j, t] += take
                    cap[j] -= take
                    pin[i, j] -= take
                    g -= take
            # then local first
            take = min(g, int(cap[i]))
            if take:
                quota[i, i, t] += take
                cap[i] -= take
                g -= take
            while g > 0:
                j = int(np.argmax(cap))          # most free slots, lowest index on ties
                if cap[j] <= 0:
                    break
                take = min(g, int(cap[j]))
                quota[i, j, t] += take
                cap[j] -= take
                g -= take
            depth[i, t] -= int(grant[i]) - g
    return quota
