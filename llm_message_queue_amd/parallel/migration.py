"""Conversation KV/context migration between GPU backends (N11).

Wired into multi-GPU dispatch (``gateway.router``): when the plan places a
conversation's turn on a GPU other than the one holding its KV (home GPU
saturated, parked by the autoscaler, or excluded by an operator -- but still
alive), the router records a migration order (conversation, source, dest) in
its NEXT load vector; every rank reads the same orders from the all-gathered
loads and ``execute`` moves the KV in two point-to-point phases (token-count
headers, then the packed K/V) before the destination admits the turn, which
then prefills only its new tokens.  A dead source (unhealthy) sends nothing:
the turn replays its dialog instead.

When the rebalancer moves a conversation off the GPU that holds its KV cache
(its "KV-residency hint", which the reference approximates with in-process
session affinity, `internal/loadbalancer/load_balancer.go:501-558`), the
source rank packs the conversation's K/V rows of every layer into ONE
contiguous buffer and sends it point-to-point to the destination rank
(``comm.send_tensor`` = RCCL send/recv over the direct xGMI link between the
two GPUs: one link, bandwidth-bound, no ring).  Llama-3-8B KV is 128 KiB per
token, so an 8k-token dialog moves ~1 GiB in ~7 ms at ~150 GB/s.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import torch


class KVMigrator:
    def __init__(self, model, comm):
        """``model`` is a ``LlamaStub`` (owns ``kcache``/``vcache`` lists)."""
        self.model = model
        self.comm = comm
        self.bytes_sent = 0
        self.bytes_recv = 0
        self.sent = 0
        self.received = 0

    def _shape(self, n: int):
        c = self.model.cfg
        return (c.layers, 2, c.kv_heads, n, c.head_dim)

    def pack(self, slot: int, n: int) -> torch.Tensor:
        m = self.model
        if not 0 < n <= m.max_ctx:
            raise ValueError(f"bad token count {n}")
        buf = torch.empty(self._shape(n), dtype=m.kcache[0].dtype, device=m.kcache[0].device)
        for layer in range(m.cfg.layers):
            buf[layer, 0].copy_(m.kcache[layer][slot, :, :n])
            buf[layer, 1].copy_(m.vcache[layer][slot, :, :n])
        return buf

    def unpack(self, buf: torch.Tensor, slot: int) -> None:
        m = self.model
        n = buf.shape[3]
        for layer in range(m.cfg.layers):
            m.kcache[layer][slot, :, :n].copy_(buf[layer, 0])
            m.vcache[layer][slot, :, :n].copy_(buf[layer, 1])

    def send(self, dst: int, slot: int, n: int) -> int:
        buf = self.pack(slot, n)
        self.comm.send_tensor(buf, dst)
        nb = buf.numel() * buf.element_size()
        self.bytes_sent += nb
        return nb

    def recv(self, src: int, slot: int, n: int) -> int:
        m = self.model
        buf = torch.empty(self._shape(n), dtype=m.kcache[0].dtype, device=m.kcache[0].device)
        self.comm.recv_tensor(buf, src)
        self.unpack(buf, slot)
        nb = buf.numel() * buf.element_size()
        self.bytes_recv += nb
        return nb

    def execute(self, orders: Sequence[Tuple[int, int, int]], engine, me: int) -> Dict[int, int]:
        """Run this tick's migration orders ``(conv, src, dst)`` -- the same
        list on every rank, sorted identically, so the per-pair message order
        matches.  Returns ``{conv: tokens}`` imported by this rank (0 tokens:
        the source no longer had the KV; the turn replays)."""
        orders = sorted({(int(c), int(s), int(d)) for c, s, d in orders if s != d}, key=lambda o: (o[1], o[2], o[0]))
        dev = self.model.kcache[0].device
        hdr_dev = dev if self._p2p_on_device() else torch.device("cpu")
        out_items: List[Tuple[int, int, int, int]] = []
        in_items: List[Tuple[int, int, torch.Tensor]] = []
        sends, recvs = [], []
        for conv, src, dst in orders:
            if me == src:
                slot, n = engine.export_kv(conv)
                sends.append((dst, torch.tensor([n], dtype=torch.int64, device=hdr_dev)))
                out_items.append((dst, conv, slot, n))
            elif me == dst:
                h = torch.zeros(1, dtype=torch.int64, device=hdr_dev)
                recvs.append((src, h))
                in_items.append((src, conv, h))
        if not sends and not recvs:
            return {}
        self.comm.exchange_p2p(sends, recvs)                  # phase 1: token counts
        sends, recvs, land = [], [], []
        host = not self._p2p_on_device() and dev.type == "cuda"   # gloo data plane: stage via host
        for dst, conv, slot, n in out_items:
            if n > 0:
                buf = self.pack(slot, n)
                sends.append((dst, buf.cpu() if host else buf))
                engine.drop_parked(conv)                     # the KV lives on dst from now on
                self.bytes_sent += buf.numel() * buf.element_size()
                self.sent += 1
        imported: Dict[int, int] = {}
        for src, conv, h in in_items:
            n = int(h.item())
            imported[conv] = 0
            if n > 0:
                buf = torch.empty(self._shape(n), dtype=self.model.kcache[0].dtype,
                                  device=torch.device("cpu") if host else dev)
                recvs.append((src, buf))
                land.append((conv, buf, n))
        self.comm.exchange_p2p(sends, recvs)                  # phase 2: packed K/V
        for conv, buf, n in land:
            slot = engine.import_kv(conv, n)
            self.unpack(buf.to(dev, non_blocking=False) if host else buf, slot)
            imported[conv] = n
            self.bytes_recv += buf.numel() * buf.element_size()
            self.received += 1
        return imported

    def _p2p_on_device(self) -> bool:
        """RCCL moves device tensors; gloo / in-process comms take host ones."""
        try:
            import torch.distributed as dist
            g = getattr(self.comm, "data_group", None)
            return dist.is_initialized() and dist.get_backend(g) == "nccl"
        except Exception:
            return False
