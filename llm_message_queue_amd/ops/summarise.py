"""Context summarisation (N5) on the GPU: ``summarise_project`` (segmented
mean + bf16 MFMA projection + EMA) and ``salient_topk`` kernels.

Used by the conversation StateManager when messages fall out of a
conversation's context window: instead of the reference's drop-oldest
truncation (`internal/conversation/state_manager.go:131-134`) the evicted
messages are embedded with the classifier's ``embed_pool`` kernel and folded
into a fixed-size per-conversation summary vector plus a salient-token list.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from .. import _native

STOP_WORDS = ("the", "a", "an", "and", "or", "to", "of", "in", "on", "for", "is", "are", "was", "it",
              "this", "that", "with", "as", "at", "be", "by", "i", "you", "me", "my", "we", "please",
              "can", "do", "what", "how")


def stop_hashes():
    from ..preprocess.oracle import fnv1a32
    return [fnv1a32(w.encode()) for w in STOP_WORDS]


class Summariser:
    def __init__(self, dim: int = 256, hidden: int = 1024, alpha: float = 0.8, seed: int = 4321,
                 device="cuda"):
        if dim != 256 or hidden != 1024:
            raise ValueError("summarise kernels are built for hidden=1024 -> dim=256")
        self.k = _native.require_hipops()
        self.dim, self.hidden, self.alpha = dim, hidden, float(alpha)
        self.device = torch.device(device)
        if self.device.type == "cuda" and self.device.index is None:
            self.device = torch.device("cuda", torch.cuda.current_device())
        g = torch.Generator(device="cpu").manual_seed(seed)
        self.Pt = (torch.randn(dim, hidden, generator=g) / hidden ** 0.5).to(torch.bfloat16).to(self.device)
        self._stop = torch.tensor(np.array(stop_hashes(), dtype=np.uint32).view(np.int32),
                                  device=self.device)

    def _s(self) -> int:
        return torch.cuda.current_stream(self.device).cuda_stream

    def project(self, pooled: torch.Tensor, seg_off: torch.Tensor, state: torch.Tensor,
                first: torch.Tensor) -> torch.Tensor:
        """state[c] <- first ? P.mean_c : alpha*state[c] + (1-alpha)*P.mean_c (in place)."""
        C = seg_off.numel() - 1
        for t, dt, name in ((pooled, torch.float32, "pooled"), (state, torch.float32, "state"),
                            (seg_off, torch.int32, "seg_off"), (first, torch.int32, "first")):
            if t.dtype != dt or not t.is_contiguous() or t.device != self.device:
                raise ValueError(f"{name}: expected contiguous {dt} on {self.device}")
        if pooled.shape[1] != self.hidden or state.shape != (C, self.dim) or first.numel() != C:
            raise ValueError("summarise shape mismatch")
        self.k.summarise_project(pooled.data_ptr(), seg_off.data_ptr(), C, self.Pt.data_ptr(), self.alpha,
                                 state.data_ptr(), first.data_ptr(), self.hidden, self.dim, self._s())
        return state

    def salient(self, hashes: torch.Tensor, ntok: torch.Tensor, seg_off: torch.Tensor, k: int = 8,
                stop: Optional[torch.Tensor] = None, ntok_stride: int = 1, link=None
                ) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """Top-k salient token hashes per segment, plus a per-segment
        overflow flag (more distinct tokens than the kernel's 2048-entry LDS
        table: that segment's top-k is partial and must be recomputed).
        ``link`` (an ``ops.hostlink.HostLink`` on the current stream) reads the
        result back without waiting for other streams."""
        C = seg_off.numel() - 1
        L = hashes.shape[1]
        stop = self._stop if stop is None else stop
        oh = torch.zeros((C, k), dtype=torch.int32, device=self.device)
        oc = torch.zeros((C, k), dtype=torch.int32, device=self.device)
        ov = torch.zeros(max(C, 1), dtype=torch.int32, device=self.device)
        self.k.salient_topk(hashes.data_ptr(), L, ntok.data_ptr(), ntok_stride, seg_off.data_ptr(), C,
                            stop.data_ptr(), stop.numel(), k, oh.data_ptr(), oc.data_ptr(), ov.data_ptr(), self._s())
        if link is not None:
            h, c, o = link.download([oh, oc, ov])
            return h.view(np.uint32), c, o[:C]
        return oh.cpu().numpy().view(np.uint32), oc.cpu().numpy(), ov.cpu().numpy()[:C]
