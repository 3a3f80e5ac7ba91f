"""Host <-> device transfers for the side-stream pipelines (preprocess,
conversation summaries) that must not wait for the backend's forward.

The runtime's async H2D path was measured to queue behind the forward steps
already submitted on the default stream (a ~60 ms stall per preprocess batch
under load).  ``HostLink`` instead stages through host-mapped pinned memory
and moves bytes with the ``copy_bytes`` kernel on the caller's stream, then
waits on an event of that stream only.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from .. import _native


def _a16(n: int) -> int:
    return (n + 15) & ~15


class HostLink:
    def __init__(self, device, stream: torch.cuda.Stream):
        self.k = _native.require_hipops()
        self.device = torch.device(device)
        self.stream = stream
        self._up = None
        self._up_dev = 0
        self._down = None
        self._down_dev = 0

    def _buf(self, which: str, nbytes: int):
        cur = getattr(self, which)
        if cur is None or cur.numel() < nbytes:
            n = max(nbytes, 2 * (cur.numel() if cur is not None else 0), 1 << 16)
            cur = torch.empty(n, dtype=torch.uint8).pin_memory()
            setattr(self, which, cur)
            setattr(self, which + "_dev", self.k.host_device_ptr(cur.data_ptr()))
        return cur, getattr(self, which + "_dev")

    def upload(self, arrays: Sequence[np.ndarray]) -> List[torch.Tensor]:
        """numpy arrays -> new device tensors (same dtype/shape), ordered on ``stream``."""
        arrays = [np.ascontiguousarray(a) for a in arrays]
        offs, tot = [], 0
        for a in arrays:
            offs.append(tot)
            tot += _a16(a.nbytes)
        buf, dev = self._buf("_up", tot)
        bn = buf.numpy()
        out = []
        s = self.stream.cuda_stream
        for a, o in zip(arrays, offs):
            bn[o:o + a.nbytes] = a.view(np.uint8).reshape(-1)
            t = torch.empty(a.shape, dtype=torch.from_numpy(a[:0].reshape(-1)).dtype, device=self.device)
            self.k.copy_bytes(t.data_ptr(), dev + o, a.nbytes, s)
            out.append(t)
        # the staging buffer is reused by the next upload: wait for the copies
        ev = torch.cuda.Event()
        ev.record(self.stream)
        ev.synchronize()
        return out

    def download(self, tensors: Sequence[torch.Tensor]) -> List[np.ndarray]:
        """device tensors -> numpy copies, after everything queued on ``stream``."""
        tensors = [t.contiguous() for t in tensors]
        offs, tot = [], 0
        for t in tensors:
            offs.append(tot)
            tot += _a16(t.numel() * t.element_size())
        buf, dev = self._buf("_down", tot)
        s = self.stream.cuda_stream
        for t, o in zip(tensors, offs):
            self.k.copy_bytes(dev + o, t.data_ptr(), t.numel() * t.element_size(), s)
        ev = torch.cuda.Event()
        ev.record(self.stream)
        ev.synchronize()
        bn = buf.numpy()
        out = []
        for t, o in zip(tensors, offs):
            nb = t.numel() * t.element_size()
            dt = torch.empty(0, dtype=t.dtype).numpy().dtype
            out.append(bn[o:o + nb].view(dt).reshape(tuple(t.shape)).copy())
        return out
