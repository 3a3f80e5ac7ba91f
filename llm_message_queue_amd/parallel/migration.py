"""Conversation KV/context migration between GPU backends (N11).

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

import torch


class KVMigrator:
    def __init__(self, model, comm):
        """``model`` is a ``LlamaStub`` (owns ``kcache``/``vcache`` lists)."""
        self.model = model
        self.comm = comm
        self.bytes_sent = 0
        self.bytes_recv = 0

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
