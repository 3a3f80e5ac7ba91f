"""Conversation KV/context migration between GPU backends (N11).

Wired into multi-GPU dispatch (``gateway.router``): when the plan places a
conversation's turn on a GPU other than the one holding its KV (home GPU
saturated, parked by the autoscaler, or excluded by an operator -- but still
alive), the router records a migration order; the next tick the home GPU
(source) and the turn's GPU (destination) move the KV, and the destination
then admits the turn, which prefills only its new tokens.  The reference
approximates this "KV residency" with in-process session affinity
(`internal/loadbalancer/load_balancer.go:501-558`).

One migration tick (``execute``), identical call order on every rank:

1. **Headers on the host control plane** (``comm.all_to_all_var``, the shm
   segment on a node): each source OFFERs ``(conv, tokens)`` to the
   destination, each destination WANTs ``conv`` from the source.  Both sides
   then hold both lists and take the same intersection -- a transfer happens
   only if the source still has the KV AND the destination still waits for
   it (a destination that went unhealthy since the order posts no WANT, so
   the source never posts an unmatched send).  No device header, no
   ``.item()``: the host never waits for the two forwards queued ahead on
   the compute stream.
2. **Data on the device** (RCCL over the direct xGMI link of the pair): the
   source packs the conversation's K/V of all 32 layers with ONE gather
   kernel (``kv_move``) on the compute stream (stream order puts it after
   the forwards that wrote the KV and before any later reuse of the slot),
   and ``isend``s it from a dedicated side stream that waits on that pack
   event only.  The destination reserves a slot, and on the side stream --
   after the compute stream's current tail, so no queued forward still uses
   the slot -- ``irecv``s and scatters with ONE kernel.  ``Work.wait`` on
   RCCL orders the side stream, not the host.  ``poll`` reports imports
   whose completion event has fired; the held turn is admitted then.

A gloo / in-process data plane (CPU rehearsal) moves host copies
synchronously through the same header protocol.  A dead or unwilling
source sends nothing: the turn replays its dialog instead.

Llama-3-8B KV is 128 KiB per token, so a 512-token dialog moves 64 MiB --
~0.5 ms on one xGMI link at ~150 GB/s.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch

OFFER, WANT = 1, 2
HDR_W = 4           # int32 header row: [kind, conv lo, conv hi, tokens]


def _rows(items: Sequence[Tuple[int, int, int]]) -> np.ndarray:
    """[(kind, conv, tokens)] -> int32 [k, 4] header rows."""
    out = np.zeros((len(items), HDR_W), dtype=np.int32)
    for i, (kind, conv, n) in enumerate(items):
        c = int(conv)
        out[i, 0] = kind
        out[i, 1] = np.int64(c & 0xFFFFFFFF).astype(np.uint32).view(np.int32)
        out[i, 2] = c >> 32
        out[i, 3] = n
    return out


def _conv(row: np.ndarray) -> int:
    return (int(row[2]) << 32) | (int(row[1]) & 0xFFFFFFFF)


class KVMigrator:
    def __init__(self, model, comm):
        """``model`` is a ``LlamaStub`` (owns ``kcache``/``vcache`` lists)."""
        self.model = model
        self.comm = comm
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.sent = 0
        self.received = 0
        self.ticks = 0
        self.host_ns = 0                  # host time inside execute (all ticks)
        self.host_max_ns = 0
        kc = model.kcache[0]
        self.device = kc.device
        self.cuda = kc.is_cuda
        self._ops = None
        self._table = None
        self._stream = None
        # imports in flight on the side stream: (conv, slot, tokens, event, buf)
        self._pending: List[Tuple[int, int, int, object, torch.Tensor]] = []
        # sends in flight: (event, buf) -- buffers stay referenced until done
        self._sending: List[Tuple[object, torch.Tensor]] = []
        if self.cuda:
            from .. import _native
            self._ops = _native.require_hipops()
            ptrs = [t.data_ptr() for t in model.kcache] + [t.data_ptr() for t in model.vcache]
            self._table = torch.tensor(ptrs, dtype=torch.int64, device=self.device)
            self._stream = torch.cuda.Stream(device=self.device, priority=-1)

    # ------------------------------------------------------------------ pack / unpack
    def _shape(self, n: int):
        c = self.model.cfg
        return (c.layers, 2, c.kv_heads, n, c.head_dim)

    def _empty(self, n: int, device=None) -> torch.Tensor:
        m = self.model
        return torch.empty(self._shape(n), dtype=m.kcache[0].dtype, device=device or self.device)

    # kv_move kernel form (csrc/kernels/kv_migrate_kernels.h): 0 one workgroup
    # per (layer, k|v, head) run, 1 / 2 the run in 32 KiB chunks (plain /
    # non-temporal).  2 by default: 5.50 TB/s beyond the Infinity Cache, 1.09x
    # a torch copy of the same bytes, against 4.47 for 0
    # (profiles/r5_kernel_rework/kv_move_variants.json, bench/kv_move_bench.py)
    KV_VARIANT = 2

    def _kv_move(self, buf: torch.Tensor, slot: int, pack: bool, stream) -> None:
        m, c = self.model, self.model.cfg
        self._ops.kv_move(self._table.data_ptr(), c.layers, m.slots, int(slot), int(buf.shape[3]), m.max_ctx,
                          c.kv_heads, c.head_dim, buf.data_ptr(), bool(pack), stream.cuda_stream,
                          int(self.KV_VARIANT))

    def pack(self, slot: int, n: int) -> torch.Tensor:
        """The conversation's K/V rows of every layer, [L, 2, Hkv, n, 128]:
        one gather kernel on the current stream (HIP), else torch copies."""
        m = self.model
        if not 0 < n <= m.max_ctx:
            raise ValueError(f"bad token count {n}")
        buf = self._empty(n)
        if self.cuda:
            self._kv_move(buf, slot, True, torch.cuda.current_stream(self.device))
            return buf
        for layer in range(m.cfg.layers):
            buf[layer, 0].copy_(m.kcache[layer][slot, :, :n])
            buf[layer, 1].copy_(m.vcache[layer][slot, :, :n])
        return buf

    def unpack(self, buf: torch.Tensor, slot: int) -> None:
        m = self.model
        if self.cuda and buf.is_cuda:
            self._kv_move(buf, slot, False, torch.cuda.current_stream(self.device))
            return
        n = buf.shape[3]
        for layer in range(m.cfg.layers):
            m.kcache[layer][slot, :, :n].copy_(buf[layer, 0])
            m.vcache[layer][slot, :, :n].copy_(buf[layer, 1])

    def send(self, dst: int, slot: int, n: int) -> int:
        """Blocking one-off transfer of slot ``slot``'s first ``n`` positions
        to ``dst`` (tools / tests; serving goes through ``execute``)."""
        buf = self.pack(slot, n)
        self.comm.send_tensor(buf, dst)
        nb = buf.numel() * buf.element_size()
        self.bytes_sent += nb
        return nb

    def recv(self, src: int, slot: int, n: int) -> int:
        buf = self._empty(n)
        self.comm.recv_tensor(buf, src)
        self.unpack(buf, slot)
        nb = buf.numel() * buf.element_size()
        self.bytes_recv += nb
        return nb

    # ------------------------------------------------------------------ one tick
    def execute(self, orders: Sequence[Tuple[int, int]], wants: Sequence[Tuple[int, int]], engine,
                me: int) -> Dict[int, int]:
        """This tick's migrations: ``orders`` = [(conv, dst)] whose KV this
        rank (the home GPU) should send, ``wants`` = [(conv, src)] this rank
        (the destination) waits for.  Called by EVERY rank on a migration
        tick (the header exchange is a collective), possibly with nothing to
        do.  Returns ``{conv: tokens}`` for every wanted conversation whose
        fate is known now: > 0 imported (synchronous data planes), 0 nothing
        will come (replay).  Wanted conversations missing from the result are
        in flight on the device; ``poll`` reports them."""
        import time
        t0 = time.perf_counter_ns()
        W = self.comm.world
        offers: List[List[Tuple[int, int, int]]] = [[] for _ in range(W)]
        mine: Dict[Tuple[int, int], Tuple[int, int]] = {}        # (dst, conv) -> (slot, tokens)
        for conv, dst in orders:
            if dst == me or not 0 <= dst < W or (dst, conv) in mine:
                continue
            slot, n = engine.export_kv(conv)
            mine[(dst, conv)] = (slot, n)
            offers[dst].append((OFFER, conv, n))
        # one source per conversation (the last one listed): the result is
        # keyed by conversation, so two sources could not be told apart
        src_of: Dict[int, int] = {}
        for conv, src in wants:
            if src != me and 0 <= src < W:
                src_of[conv] = src
        want_set = set()
        for conv, src in src_of.items():
            want_set.add((src, conv))
            offers[src].append((WANT, conv, 0))
        got = self.comm.all_to_all_var([_rows(x) for x in offers], HDR_W)
        their_offer: Dict[Tuple[int, int], int] = {}
        their_want = set()
        for src in range(W):
            for row in got[src]:
                if row[0] == OFFER:
                    their_offer[(src, _conv(row))] = int(row[3])
                elif row[0] == WANT:
                    their_want.add((src, _conv(row)))
        # identical intersections on both sides; per pair in conv order
        sends = sorted((dst, conv) for (dst, conv), (slot, n) in mine.items()
                       if n > 0 and (dst, conv) in their_want)
        recvs = sorted((src, conv) for (src, conv) in want_set if their_offer.get((src, conv), 0) > 0)
        result: Dict[int, int] = {conv: 0 for (src, conv) in want_set
                                  if their_offer.get((src, conv), 0) <= 0}
        if sends or recvs:
            if self.cuda and self._p2p_on_device():
                self._device_transfer(sends, recvs, mine, their_offer, engine)
            else:
                result.update(self._host_transfer(sends, recvs, mine, their_offer, engine))
        self.ticks += 1
        dt = time.perf_counter_ns() - t0
        self.host_ns += dt
        self.host_max_ns = max(self.host_max_ns, dt)
        return result

    def _host_transfer(self, sends, recvs, mine, their_offer, engine) -> Dict[int, int]:
        """gloo / in-process data plane: synchronous host copies."""
        host = self.cuda                  # device KV staged through host memory for gloo
        p2p_s, p2p_r, land = [], [], []
        for dst, conv in sends:
            slot, n = mine[(dst, conv)]
            buf = self.pack(slot, n)
            p2p_s.append((dst, buf.cpu() if host else buf))
            engine.drop_parked(conv)                      # the KV lives on dst from now on
            self.bytes_sent += buf.numel() * buf.element_size()
            self.sent += 1
        for src, conv in recvs:
            n = their_offer[(src, conv)]
            buf = self._empty(n, torch.device("cpu") if host else None)
            p2p_r.append((src, buf))
            land.append((conv, buf, n))
        self.comm.exchange_p2p(p2p_s, p2p_r)
        out = {}
        for conv, buf, n in land:
            slot = engine.import_kv(conv, n)
            self.unpack(buf.to(self.device) if host else buf, slot)
            out[conv] = n
            self.bytes_recv += buf.numel() * buf.element_size()
            self.received += 1
        return out

    def _device_transfer(self, sends, recvs, mine, their_offer, engine) -> None:
        """RCCL data plane: pack on the compute stream, p2p + unpack on the
        side stream; the host only enqueues."""
        comp = torch.cuda.current_stream(self.device)
        side = self._stream
        p2p_s, p2p_r, land = [], [], []
        for dst, conv in sends:
            slot, n = mine[(dst, conv)]
            buf = self.pack(slot, n)                       # compute stream: after the KV's writers
            engine.drop_parked(conv)                       # later reuse of the slot is stream-ordered after
            p2p_s.append((dst, buf))
            self.bytes_sent += buf.numel() * buf.element_size()
            self.sent += 1
        tail = torch.cuda.Event()
        tail.record(comp)                                  # packs done + every queued forward
        for src, conv in recvs:
            n = their_offer[(src, conv)]
            slot = engine.reserve_import(conv, n)
            buf = self._empty(n)
            p2p_r.append((src, buf))
            land.append((conv, slot, n, buf))
        with torch.cuda.stream(side):
            side.wait_event(tail)
            self.comm.exchange_p2p(p2p_s, p2p_r)           # RCCL: Work.wait orders the side stream
            for conv, slot, n, buf in land:
                self._kv_move(buf, slot, False, side)
            done = torch.cuda.Event()
            done.record(side)
        for _dst, buf in p2p_s:
            buf.record_stream(side)
            self._sending.append((done, buf))
        for conv, slot, n, buf in land:
            buf.record_stream(side)
            self._pending.append((conv, slot, n, done, buf))

    def poll(self, engine) -> Dict[int, int]:
        """Imports whose data landed since the last call: parks each one in
        its reserved slot and returns ``{conv: tokens}`` (non-blocking)."""
        self._sending = [(e, b) for e, b in self._sending if not e.query()]
        if not self._pending:
            return {}
        out, keep = {}, []
        for conv, slot, n, ev, buf in self._pending:
            if ev.query():
                engine.finish_import(conv, slot, n)
                out[conv] = n
                self.bytes_recv += buf.numel() * buf.element_size()
                self.received += 1
            else:
                keep.append((conv, slot, n, ev, buf))
        self._pending = keep
        return out

    def abandon(self) -> List[object]:
        """Evacuation: forget every import in flight (its slot goes back to
        the engine's free list) and return the side-stream events the
        compute stream must wait on before a slot is reused -- a late unpack
        would otherwise write stale KV under a new request's prefill."""
        evs = []
        for _conv, _slot, _n, ev, buf in self._pending:
            if ev is not None and not any(ev is e for e in evs):
                evs.append(ev)
        self._pending = []
        return evs

    def in_flight(self) -> int:
        return len(self._pending)

    def _p2p_on_device(self) -> bool:
        """RCCL moves device tensors; gloo / in-process comms take host ones."""
        try:
            import torch.distributed as dist
            g = getattr(self.comm, "data_group", None)
            if g is None and hasattr(self.comm, "data"):
                g = getattr(self.comm.data, "data_group", None)
            return dist.is_initialized() and dist.get_backend(g) == "nccl"
        except Exception:
            return False
