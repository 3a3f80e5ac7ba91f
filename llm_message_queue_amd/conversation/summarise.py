"""Summarise-on-evict engine for conversation windows (N5).

GPU path (default on a GPU host): the evicted messages of a batch of
conversations go through ``text_analyze`` + ``embed_pool`` (token hashes and
pooled embeddings, kept on the device), then ``summarise_project`` (segmented
mean, bf16 MFMA projection 1024->256, EMA into the conversation's summary) and
``salient_topk``.  CPU path (CPU-only deployments and tests): the same math in
plain PyTorch fp32 with identically seeded weights.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import numpy as np

from ..preprocess import oracle


class SummaryEngine:
    def __init__(self, cfg=None, *, device: Optional[str] = None, k: int = 8, alpha: float = 0.8, dim: int = 256):
        import torch
        from ..utils.config import PreprocessorConfig
        self.torch = torch
        self.cfg = cfg or PreprocessorConfig()
        self.k = k
        self.alpha = alpha
        self.dim = int(dim)                 # conversation.summary_dim (the kernels are built for 256)
        if device is None:
            device = "cuda" if torch.cuda.is_available() else "cpu"
        self.device = torch.device(device)
        self.gpu = self.device.type == "cuda"
        self._pipe = None
        self._sm = None
        self._cpu_w = None
        self.batches = 0
        self.salient_overflows = 0      # conversations recomputed on the host (kernel table overflow)

    # --------------------------------------------------------------- GPU
    def _gpu_parts(self):
        if self._pipe is None:
            from ..ops.summarise import Summariser
            from ..ops.text import TextPipeline
            self._pipe = TextPipeline(self.cfg, device=str(self.device))
            self._sm = Summariser(dim=self.dim, hidden=self.cfg.hidden_dim, alpha=self.alpha, device=str(self.device))
        return self._pipe, self._sm

    # --------------------------------------------------------------- CPU reference
    def _cpu_parts(self):
        if self._cpu_w is None:
            from ..ops.text import ClassifierWeights
            torch = self.torch
            w = ClassifierWeights(self.cfg.vocab_buckets, self.cfg.embed_dim, self.cfg.hidden_dim, self.cfg.seed,
                                  device="cpu")
            g = torch.Generator(device="cpu").manual_seed(4321)
            Pt = (torch.randn(self.dim, self.cfg.hidden_dim, generator=g) / self.cfg.hidden_dim ** 0.5).to(torch.bfloat16)
            self._cpu_w = (w, Pt)
        return self._cpu_w

    def _pool_cpu(self, contents: Sequence[str]) -> Tuple[np.ndarray, List[List[int]]]:
        torch = self.torch
        w, _ = self._cpu_parts()
        L = self.cfg.max_tokens
        pooled = torch.zeros((len(contents), w.hidden))
        toks = []
        E, W1t, b1 = w.E.float(), w.W1t.float(), w.b1
        for i, c in enumerate(contents):
            h = oracle.token_hashes(oracle.sanitize(c), L)
            toks.append(h)
            if not h:
                continue
            idx = torch.as_tensor([x & (w.vocab - 1) for x in h], dtype=torch.long)
            Hd = E[idx] @ W1t.t() + b1
            Hd = 0.5 * Hd * (1 + torch.tanh(0.7978845608028654 * (Hd + 0.044715 * Hd ** 3)))
            pooled[i] = Hd.mean(0)
        return pooled, toks

    def _link(self, pipe):
        if getattr(self, "_hostlink", None) is None:
            from ..ops.hostlink import HostLink
            self._hostlink = HostLink(self.device, pipe.stream)
        return self._hostlink

    # --------------------------------------------------------------- API
    def summarise(self, groups: Sequence[Tuple[Optional[np.ndarray], Sequence[str]]]
                  ) -> List[Tuple[np.ndarray, List[Tuple[int, int]]]]:
        """``groups[c] = (previous summary or None, evicted contents)`` ->
        ``[(new summary [256] f32, [(token_hash, count), ...])]``."""
        if not groups:
            return []
        self.batches += 1
        torch = self.torch
        contents = [c for _, cs in groups for c in cs]
        counts = [len(cs) for _, cs in groups]
        seg = np.zeros(len(groups) + 1, dtype=np.int32)
        np.cumsum(counts, out=seg[1:])
        C = len(groups)
        state = np.zeros((C, 256), dtype=np.float32)
        first = np.zeros(C, dtype=np.int32)
        for c, (prev, _) in enumerate(groups):
            if prev is None:
                first[c] = 1
            else:
                state[c] = np.asarray(prev, dtype=np.float32)
        if self.gpu:
            pipe, sm = self._gpu_parts()
            from ..preprocess.oracle import default_patterns
            res = pipe.run(contents, default_patterns(), 0, classify=True, keep_device=True)
            link = self._link(pipe)
            with torch.cuda.stream(pipe.stream):
                seg_d, st_d, fi_d, ntok = link.upload([seg, state, first,
                                                       np.ascontiguousarray(res.stats[:, 5], dtype=np.int32)])
                sm.project(res.pooled, seg_d, st_d, fi_d)
                hs, cs, ovf = sm.salient(res.hashes, ntok, seg_d, k=self.k, link=link)
                new_state = link.download([st_d])[0]
            sal = [[(int(h), int(n)) for h, n in zip(hs[c], cs[c]) if n > 0] for c in range(C)]
            for c in np.flatnonzero(ovf):
                # > 2048 distinct tokens overflowed the kernel's LDS table:
                # exact top-k on the host for that conversation
                self.salient_overflows += 1
                a, b = int(seg[c]), int(seg[c + 1])
                toks = [oracle.token_hashes(oracle.sanitize(x), self.cfg.max_tokens) for x in contents[a:b]]
                sal[c] = _topk_host(toks, self.k)
            return [(new_state[c], sal[c]) for c in range(C)]
        # CPU reference
        pooled, toks = self._pool_cpu(contents)
        _, Pt = self._cpu_parts()
        stop = set(_stop_hashes())
        out = []
        for c in range(C):
            a, b = int(seg[c]), int(seg[c + 1])
            mean = pooled[a:b].mean(0).to(torch.bfloat16).float() if b > a else torch.zeros(pooled.shape[1])
            proj = (Pt.float() @ mean).numpy()
            s = proj if first[c] else self.alpha * state[c] + (1 - self.alpha) * proj
            out.append((s.astype(np.float32), _topk_host(toks[a:b], self.k, stop)))
        return out


def _topk_host(toks: Sequence[Sequence[int]], k: int, stop=None) -> List[Tuple[int, int]]:
    """Exact salient top-k: non-stop-word token hashes by (count desc,
    first occurrence asc); hash 0 is folded to 1 as in the kernel."""
    stop = set(_stop_hashes()) if stop is None else stop
    cnt, firstpos = {}, {}
    i = 0
    for msg in toks:
        for t in msg:
            if t in stop:
                i += 1
                continue
            t = t or 1
            cnt[t] = cnt.get(t, 0) + 1
            firstpos.setdefault(t, i)
            i += 1
    return sorted(cnt.items(), key=lambda kv: (-kv[1], firstpos[kv[0]]))[:k]


def _stop_hashes():
    from ..ops.summarise import stop_hashes
    return stop_hashes()
