"""The gateway's view of the GPUs as resources (``Gateway`` mixin): the
balancer's exclusions (parked / unhealthy endpoints), endpoint weights, HBM
occupancy, and the per-GPU usage fed to the ResourceScheduler from every
tick's load exchange (`internal/scheduler/resource_scheduler.go:336-398`).
Serve-loop only."""
from __future__ import annotations

import time
from typing import List, Optional, Tuple

import numpy as np

from ..parallel import planner


class ResourceMixin:
    def _exclude_mask(self) -> int:
        """GPUs this rank's balancer view rules out for new work: parked by
        the autoscaler (endpoint removed), or marked unhealthy by an operator
        or a health probe.  Only GPU endpoints (``gpu<j>``) count; a rank
        without a balancer excludes nothing."""
        lb = self.lb
        if lb is None:
            return 0
        mask = 0
        for j in range(self.world):
            try:
                ep = lb.get_endpoint_by_id(f"gpu{j}")
            except Exception:
                if j in self._gpu_eps_seen:       # registered once, now removed (parked)
                    mask |= 1 << j
                continue
            self._gpu_eps_seen.add(j)
            if not lb._eligible(ep):
                mask |= 1 << j
        return mask

    # ------------------------------------------------------------------ resource scheduler
    def attach_resource_scheduler(self, rs, act: bool = True) -> None:
        """Per-GPU usage (slots, HBM footprint, KV tokens) flows into ``rs``
        from every load exchange; with ``act`` its autoscale decisions park /
        unpark GPU endpoints in this rank's balancer (one rank -- rank 0 --
        should act: its ``L_EXCLUDE`` bit takes the GPU out of placement on
        every rank)."""
        self.resources = rs
        if act and self.lb is not None:
            rs.on_scale = self._on_resource_scale

    def _on_resource_scale(self, action: str, avg_load: float) -> Optional[str]:
        rs, lb = self.resources, self.lb
        rid = rs.scale_target(action)
        if rid is None or not rid.startswith("gpu"):
            return None
        if action == "scale_down":
            try:
                ep = lb.get_endpoint_by_id(rid)
            except Exception:
                return None
            lb.remove_endpoint(rid)
            self._parked_eps[rid] = ep
            rs.park(rid)
            self.log.info("resource scheduler parked a GPU", gpu=rid, average_load=round(avg_load, 3))
        else:
            ep = self._parked_eps.pop(rid, None)
            if ep is None:
                rs.unpark(rid)
                return None
            ep.pending = 0
            lb.add_endpoint(ep)
            rs.unpark(rid)
            self.log.info("resource scheduler unparked a GPU", gpu=rid, average_load=round(avg_load, 3))
        return rid

    def _weights(self) -> List[int]:
        lb = self.lb
        out = []
        for j in range(self.world):
            try:
                out.append(max(1, int(lb.get_endpoint_by_id(f"gpu{j}").weight)) if lb is not None else 1)
            except Exception:
                out.append(1)
        return out

    def _hbm_mib(self) -> Tuple[int, int]:
        """(used, total) MiB of this rank's GPU: the telemetry page (amd-smi)
        when the poller fills it, else the HIP allocator's view, refreshed at
        most every 250 ms (a device query per tick would cost more than the
        tick's planning)."""
        eng = self.engine
        page = getattr(eng, "page", None) if eng is not None else None
        if page is not None:
            try:
                w = page.words
                if int(w[6]) > 0:
                    return int(w[5]) >> 20, int(w[6]) >> 20
            except Exception:
                pass
        now = time.monotonic_ns()
        used, total, at = self._hbm_cache
        if now - at < 250_000_000:
            return used, total
        if self.hbm_fn is not None:
            used, total = self.hbm_fn()
        elif eng is not None and getattr(eng, "cuda", False):
            import torch
            free_b, tot_b = torch.cuda.mem_get_info(eng.device)
            used, total = (tot_b - free_b) >> 20, tot_b >> 20
        self._hbm_cache = (int(used), int(total), now)
        return int(used), int(total)

    def _observe_loads(self, loads: np.ndarray) -> None:
        """Per-tick bookkeeping on the gathered load matrix: peers' health and
        stop flags, and (at most every gpu.rebalance_interval_ms) the ResourceScheduler's
        per-GPU usage -- in-flight slots, HBM, KV tokens -- so
        ``/api/v1/resources/stats`` tracks real GPU use on every rank."""
        W = self.world
        self.loads = loads
        if loads[:, planner.L_STOP].any():
            self.peers_stopping = True
        self.cluster_idle = not (loads[:, planner.L_INFLIGHT].any()
                                 or loads[:, planner.L_DEPTH:planner.L_DEPTH + planner.NTIERS].any()
                                 or loads[:, planner.L_DONE:planner.L_DONE + W].any())
        self.unhealthy_peers = {i for i in range(W) if loads[i, planner.L_HEALTHY] == 0}
        ex = planner.eligible(loads)
        self.excluded_peers = {i for i in range(W) if not ex[i] and loads[i, planner.L_HEALTHY] != 0}
        rs = self.resources
        now = time.monotonic_ns()
        if rs is None or now < self._res_next_ns:
            return
        self._res_next_ns = now + self.res_interval_ns
        # job-wide backlog: queued requests beyond the free slots of the GPUs
        # in placement -- the autoscaler's "pending demand"
        el = planner.eligible(loads)
        queued = int(loads[:, planner.L_DEPTH:planner.L_DEPTH + planner.NTIERS].sum())
        rs.note_backlog(queued - int(loads[el, planner.L_SLOTS].sum()))
        from ..scheduler.resource_scheduler import ResourceType
        for j in range(W):
            rid = f"gpu{j}"
            slots = int(loads[j, planner.L_SLOTS_TOTAL])
            cap = {ResourceType.GPU: slots, ResourceType.MEMORY: int(loads[j, planner.L_HBM_TOTAL]) << 20,
                   ResourceType.TOKENS: int(loads[j, planner.L_KV_CAP])}
            used = {ResourceType.GPU: int(loads[j, planner.L_INFLIGHT]),
                    ResourceType.MEMORY: int(loads[j, planner.L_HBM_USED]) << 20,
                    ResourceType.TOKENS: int(loads[j, planner.L_KV_TOKENS])}
            try:
                rs.heartbeat(rid, used=used, capacity=cap)
            except Exception:            # first sight of a peer GPU: register it
                rs.register_gpu(j, "llm", slots, cap[ResourceType.MEMORY], cap[ResourceType.TOKENS])
                rs.heartbeat(rid, used=used, capacity=cap)
