"""Node-shared load pages (N9): one 4 KiB page per GPU backend in /dev/shm.

The page is ``hipHostRegister``-ed as mapped memory, so the backend's
``slot_census`` kernel writes ``{seq, active, free, tokens, step}`` straight
into host memory at the end of each step (system-scope stores), and any router
process on the node reads the live in-flight/free-slot counters with a plain
memory load -- no GPU call, no RPC, no TCP.  The reference's equivalent is
``Endpoint.Connections++/--`` in process memory
(`internal/loadbalancer/load_balancer.go:282,306-308`).

Layout (uint32 words): 0 seq | 1 active | 2 free | 3 tokens | 4 step |
5 hbm_used_MiB | 6 hbm_total_MiB | 7 busy_pct | 8 healthy | 9 pid
"""
from __future__ import annotations

import mmap
import os
from typing import Dict, Optional

import numpy as np

PAGE_BYTES = 4096
W_SEQ, W_ACTIVE, W_FREE, W_TOKENS, W_STEP, W_HBM_USED, W_HBM_TOTAL, W_BUSY, W_HEALTHY, W_PID = range(10)


def page_path(job: str, gpu: int) -> str:
    return f"/dev/shm/llmq_{job}_gpu{gpu}.page"


class SlotPage:
    def __init__(self, job: str, gpu: int, create: bool = True):
        self.path = page_path(job, gpu)
        self.gpu = gpu
        flags = os.O_RDWR | (os.O_CREAT if create else 0)
        fd = os.open(self.path, flags, 0o600)
        try:
            if create and os.fstat(fd).st_size < PAGE_BYTES:
                os.ftruncate(fd, PAGE_BYTES)
            self._mm = mmap.mmap(fd, PAGE_BYTES, mmap.MAP_SHARED, mmap.PROT_READ | mmap.PROT_WRITE)
        finally:
            os.close(fd)
        self.words = np.frombuffer(self._mm, dtype=np.uint32, count=PAGE_BYTES // 4)
        if create:
            # a page left by a crashed job of the same name (torchrun's default
            # run id is the same for every launch) must not be read as live load
            self.words[:] = 0
        self.dev_ptr: Optional[int] = None
        self._registered_ptr: Optional[int] = None
        self.owner = create

    def unlink_name(self) -> None:
        """Drop the page's /dev/shm name, keeping the mapping (a serving job
        whose readers all hold the page object: nothing is left behind if the
        process is SIGKILLed)."""
        if self.owner:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass

    def host_ptr(self) -> int:
        return self.words.ctypes.data

    def register_device(self) -> int:
        """Map the page into the GPU's address space (hipHostRegister)."""
        from .. import _native
        ops = _native.require_hipops()
        _h, dev = ops.register_host_page(self.host_ptr(), PAGE_BYTES)
        self._registered_ptr = self.host_ptr()
        self.dev_ptr = int(dev)
        return self.dev_ptr

    def write_host(self, active: int, free: int, tokens: int, step: int) -> None:
        w = self.words
        w[W_ACTIVE] = active
        w[W_FREE] = free
        w[W_TOKENS] = tokens
        w[W_STEP] = step & 0xFFFFFFFF
        w[W_SEQ] = (int(w[W_SEQ]) + 1) & 0xFFFFFFFF

    def set_telemetry(self, hbm_used_mib: int, hbm_total_mib: int, busy_pct: int) -> None:
        self.words[W_HBM_USED] = hbm_used_mib
        self.words[W_HBM_TOTAL] = hbm_total_mib
        self.words[W_BUSY] = busy_pct

    def set_health(self, healthy: bool) -> None:
        self.words[W_HEALTHY] = 1 if healthy else 0
        self.words[W_PID] = os.getpid()

    def active(self) -> int:
        return int(self.words[W_ACTIVE])

    def free(self) -> int:
        return int(self.words[W_FREE])

    def read(self) -> Dict[str, int]:
        w = self.words.copy()
        return {"seq": int(w[W_SEQ]), "active": int(w[W_ACTIVE]), "free": int(w[W_FREE]),
                "tokens": int(w[W_TOKENS]), "step": int(w[W_STEP]),
                "hbm_used_mib": int(w[W_HBM_USED]), "hbm_total_mib": int(w[W_HBM_TOTAL]),
                "busy_pct": int(w[W_BUSY]), "healthy": int(w[W_HEALTHY]), "pid": int(w[W_PID])}

    def close(self, unlink: bool = False) -> None:
        if self._registered_ptr is not None:
            try:
                from .. import _native
                _native.require_hipops().unregister_host_page(self._registered_ptr)
            except Exception:
                pass
            self._registered_ptr = None
        self.words = None
        try:
            self._mm.close()
        except BufferError:
            pass
        if unlink and self.owner:
            try:
                os.unlink(self.path)
            except FileNotFoundError:
                pass
