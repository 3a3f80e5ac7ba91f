"""Backend-stub decode ops: HIP kernels (``_hipops``) and plain-PyTorch fp32
reference implementations of the same math (used by the numerics tests and,
explicitly requested, by CPU-only engine tests -- never as a silent fallback
on a GPU host).

KV cache layout per layer: ``[slots, kv_heads, max_ctx, 128]`` bf16.
"""
from __future__ import annotations

import math
from typing import Optional

import os

import torch

from .. import _native


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _check(t: torch.Tensor, dtype, name: str):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


class HipOps:
    """Thin validated wrappers over the HIP kernels."""

    def __init__(self):
        self.k = _native.require_hipops()

    def rmsnorm(self, x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
        _check(x, torch.bfloat16, "x")
        _check(w, torch.bfloat16, "w")
        T, D = x.shape
        if w.numel() != D:
            raise ValueError("rmsnorm weight size mismatch")
        if residual is not None:
            _check(residual, torch.bfloat16, "residual")
            if residual.shape != x.shape:
                raise ValueError("residual shape mismatch")
        y = out if out is not None else torch.empty_like(x)
        self.k.rmsnorm(x.data_ptr(), residual.data_ptr() if residual is not None else 0, w.data_ptr(),
                       y.data_ptr(), T, D, float(eps), _stream(x))
        return y

    def silu_mul(self, gu: torch.Tensor, out: Optional[torch.Tensor] = None, perm: bool = False) -> torch.Tensor:
        """silu(gate) * up; ``perm``: ``gu`` columns are in the fused GEMM's
        swiglu order (``ops.gemm.swiglu_perm_index``) instead of [gate | up]."""
        _check(gu, torch.bfloat16, "gu")
        T, F2 = gu.shape
        F = F2 // 2
        y = out if out is not None else torch.empty((T, F), dtype=gu.dtype, device=gu.device)
        self.k.silu_mul(gu.data_ptr(), y.data_ptr(), T, F, _stream(gu), perm)
        return y

    def row_rms(self, x: torch.Tensor, eps: float) -> torch.Tensor:
        """1 / sqrt(mean(x^2) + eps) per row (the RMSNorm scale), fp32.  The
        buffer holds ceil(T/256)*256 floats -- the fused GEMMs read whole
        256-row tiles of it with vector loads -- and its first T are the
        scales."""
        from .gemm import row_scale_len
        _check(x, torch.bfloat16, "x")
        T, D = x.shape
        r = torch.empty(row_scale_len(T), dtype=torch.float32, device=x.device)
        self.k.row_rms(x.data_ptr(), r.data_ptr(), T, D, float(eps), _stream(x))
        return r

    def swiglu_rows(self, x, w_perm, r):
        """The MLP up-projection of rmsnorm(x): one GEMM over the raw rows,
        the norm weight folded into ``w_perm``, ``r`` applied per row."""
        from . import gemm as G
        return G.gemm_swiglu(x, w_perm, row_scale=r)

    def qkv_rope_rows(self, x, wqkv, r, pos, slot, cos_t, sin_t, Hq, Hkv, kc, vc, split=True, split_full=None):
        from . import gemm as G
        return G.qkv_rope(x, wqkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc, vc, row_scale=r, split=split,
                          split_full=split_full)

    def greedy_head(self, x, w, fused: bool = True, min_rows: int = 256):
        """Greedy tokens of the LM head (int32 [M]): the hand-written GEMM
        with the argmax epilogue from ``min_rows`` rows (no logits tensor),
        else hipBLASLt + torch.argmax."""
        from . import gemm as G
        if fused and x.shape[0] >= min_rows and G.supported(x.shape[0], w.shape[0], x.shape[1]):
            return G.lm_head_argmax(x, w)
        return torch.argmax(torch.nn.functional.linear(x, w), dim=-1).to(torch.int32)

    def mlp_up(self, x: torch.Tensor, w_gu: torch.Tensor, fused: bool, min_fused_tokens: int) -> torch.Tensor:
        """silu(x·Wgᵀ) * (x·Wuᵀ).  ``fused``: ``w_gu`` is in swiglu order and
        steps of >= ``min_fused_tokens`` rows run the hand-written GEMM with
        the SwiGLU epilogue (one launch, no [T][2F] intermediate); smaller
        steps keep hipBLASLt + the permuted silu_mul."""
        if not fused:
            return self.silu_mul(torch.nn.functional.linear(x, w_gu))
        from . import gemm as G
        if x.shape[0] >= min_fused_tokens and G.supported(x.shape[0], w_gu.shape[0], x.shape[1]):
            return G.gemm_swiglu(x, w_gu)
        return self.silu_mul(torch.nn.functional.linear(x, w_gu), perm=True)

    def rope_kv(self, qkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc, vc, q_out=None):
        _check(qkv, torch.bfloat16, "qkv")
        _check(pos, torch.int32, "pos")
        _check(slot, torch.int32, "slot")
        T = qkv.shape[0]
        if qkv.shape[1] != (Hq + 2 * Hkv) * 128:
            raise ValueError("qkv width mismatch")
        S, hk, max_ctx, hd = kc.shape
        if hk != Hkv or hd != 128 or vc.shape != kc.shape:
            raise ValueError("kv cache shape mismatch")
        q = q_out if q_out is not None else torch.empty((T, Hq * 128), dtype=qkv.dtype, device=qkv.device)
        self.k.rope_kv(qkv.data_ptr(), pos.data_ptr(), slot.data_ptr(), cos_t.data_ptr(), sin_t.data_ptr(), T,
                       Hq, Hkv, max_ctx, S, q.data_ptr(), kc.data_ptr(), vc.data_ptr(), _stream(qkv))
        return q

    def attention(self, q, kc, vc, pos, slot, Hq, Hkv, scale, out=None):
        _check(q, torch.bfloat16, "q")
        T = q.shape[0]
        max_ctx = kc.shape[2]
        o = out if out is not None else torch.empty_like(q)
        self.k.attention(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), pos.data_ptr(), slot.data_ptr(), T, Hq, Hkv,
                         max_ctx, kc.shape[0], float(scale), o.data_ptr(), _stream(q))
        return o


    MIXED_ATTENTION = os.environ.get("LLMQ_ATTN_MIXED", "1") != "0"

    def attention_tiles(self, q, kc, vc, tiles, Hq, Hkv, scale, out=None, n_dec: int = 0, seg_keys: int = 32,
                        mixed: bool = None):
        """Tiled attention; ``tiles`` int32 [n, 4] on the device = (first
        token row, n <= 16, slot, first position).  The first ``n_dec`` tiles
        must be 1-token (decode) tiles: they run on the wave-per-item decode
        kernel, the rest on the MFMA segment kernel (``seg_keys`` keys per
        block: 32 or 64).  ``mixed`` (default on; env LLMQ_ATTN_MIXED=0
        turns it off): a step with both kinds runs them in ONE launch."""
        _check(q, torch.bfloat16, "q")
        if tiles.dtype != torch.int32 or tiles.dim() != 2 or tiles.shape[1] != 4 or not tiles.is_contiguous():
            raise ValueError("tiles must be a contiguous int32 [n, 4] tensor")
        o = out if out is not None else torch.empty_like(q)
        self.k.attention_tiles(q.data_ptr(), kc.data_ptr(), vc.data_ptr(), tiles.data_ptr(), tiles.shape[0],
                               int(n_dec), Hq, Hkv, kc.shape[2], kc.shape[0], q.shape[0], float(scale),
                               o.data_ptr(), _stream(q), int(seg_keys),
                               self.MIXED_ATTENTION if mixed is None else bool(mixed))
        return o


def make_tiles(seg_start, seg_len, seg_slot, seg_pos0, tile: int = 16):
    """Cut segments (runs of consecutive positions of one slot) into
    attention tiles of <= ``tile`` tokens: int32 [n, 4] numpy array."""
    out = []
    for st, n, sl, p0 in zip(seg_start, seg_len, seg_slot, seg_pos0):
        for a in range(0, n, tile):
            out.append((st + a, min(tile, n - a), sl, p0 + a))
    import numpy as _np
    return _np.asarray(out, dtype=_np.int32).reshape(-1, 4)


class RefOps:
    """fp32 PyTorch reference of the same math (bf16 in / bf16 out)."""

    def rmsnorm(self, x, w, eps, residual=None, out=None):
        xf = x.float()
        if residual is not None:
            r = (xf + residual.float()).to(torch.bfloat16)
            residual.copy_(r)
            xf = r.float()
        y = xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps) * w.float()
        y = y.to(torch.bfloat16)
        if out is not None:
            out.copy_(y)
            return out
        return y

    def silu_mul(self, gu, out=None, perm: bool = False):
        F = gu.shape[1] // 2
        if perm:
            from .gemm import swiglu_perm_index
            gu = gu.index_select(1, swiglu_perm_index(F, gu.device).argsort())
        g, u = gu[:, :F].float(), gu[:, F:].float()
        y = (torch.nn.functional.silu(g) * u).to(torch.bfloat16)
        if out is not None:
            out.copy_(y)
            return out
        return y

    def row_rms(self, x, eps):
        xf = x.float()
        return torch.rsqrt(xf.pow(2).mean(-1) + eps)

    def swiglu_rows(self, x, w_perm, r):
        """Reference of ``HipOps.swiglu_rows`` (fp32 math, one bf16 rounding)."""
        from .gemm import swiglu_unpermute
        w = swiglu_unpermute(w_perm).float()
        F = w.shape[0] // 2
        gu = (x.float() * r[:, None]) @ w.t()
        return (torch.nn.functional.silu(gu[:, :F]) * gu[:, F:]).to(torch.bfloat16)

    def qkv_rope_rows(self, x, wqkv, r, pos, slot, cos_t, sin_t, Hq, Hkv, kc, vc, split=True, split_full=None):
        qkv = ((x.float() * r[:, None]) @ wqkv.float().t()).to(torch.bfloat16)
        return self.rope_kv(qkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc, vc)

    def greedy_head(self, x, w, fused: bool = True, min_rows: int = 256):
        return torch.argmax(torch.nn.functional.linear(x, w), dim=-1).to(torch.int32)

    def mlp_up(self, x, w_gu, fused: bool, min_fused_tokens: int):
        """Reference of ``HipOps.mlp_up`` (``w_gu`` in swiglu order if fused)."""
        if fused:
            from .gemm import swiglu_unpermute
            w_gu = swiglu_unpermute(w_gu)
        return self.silu_mul(torch.nn.functional.linear(x, w_gu))

    def rope_kv(self, qkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc, vc, q_out=None):
        T = qkv.shape[0]
        x = qkv.float().view(T, Hq + 2 * Hkv, 128)
        c = cos_t[pos.long()].unsqueeze(1)   # [T,1,64]
        s = sin_t[pos.long()].unsqueeze(1)

        def rot(v):
            a, b = v[..., :64], v[..., 64:]
            return torch.cat([a * c - b * s, b * c + a * s], dim=-1)

        q = rot(x[:, :Hq]).to(torch.bfloat16).reshape(T, Hq * 128)
        k = rot(x[:, Hq:Hq + Hkv]).to(torch.bfloat16)
        v = x[:, Hq + Hkv:].to(torch.bfloat16)
        for t in range(T):
            kc[slot[t], :, pos[t]] = k[t]
            vc[slot[t], :, pos[t]] = v[t]
        if q_out is not None:
            q_out.copy_(q)
            return q_out
        return q

    def attention(self, q, kc, vc, pos, slot, Hq, Hkv, scale, out=None):
        T = q.shape[0]
        G = Hq // Hkv
        res = torch.empty_like(q)
        qf = q.float().view(T, Hq, 128)
        for t in range(T):
            n = int(pos[t]) + 1
            K = kc[slot[t], :, :n].float()       # [Hkv, n, 128]
            V = vc[slot[t], :, :n].float()
            Kx = K.repeat_interleave(G, dim=0)   # [Hq, n, 128]
            Vx = V.repeat_interleave(G, dim=0)
            sc = torch.einsum("hd,hnd->hn", qf[t], Kx) * scale
            p = torch.softmax(sc, dim=-1)
            res[t] = torch.einsum("hn,hnd->hd", p, Vx).reshape(-1).to(torch.bfloat16)
        if out is not None:
            out.copy_(res)
            return out
        return res

    def attention_tiles(self, q, kc, vc, tiles, Hq, Hkv, scale, out=None, n_dec: int = 0, seg_keys: int = 32):
        """Reference: expand tiles to per-token (pos, slot) and reuse ``attention``."""
        t = tiles.cpu().long()
        T = q.shape[0]
        pos = torch.zeros(T, dtype=torch.long)
        slot = torch.zeros(T, dtype=torch.long)
        for r0, n, sl, p0 in t.tolist():
            pos[r0:r0 + n] = torch.arange(p0, p0 + n)
            slot[r0:r0 + n] = sl
        return self.attention(q, kc, vc, pos, slot, Hq, Hkv, scale, out=out)


def rope_tables(max_pos: int, theta: float = 500000.0, device="cpu"):
    inv = 1.0 / (theta ** (torch.arange(0, 64, dtype=torch.float64) / 64.0))
    t = torch.arange(max_pos, dtype=torch.float64)
    f = torch.outer(t, inv)
    return f.cos().float().to(device).contiguous(), f.sin().float().to(device).contiguous()


def get_ops(impl: str):
    if impl == "hip":
        return HipOps()
    if impl == "ref":
        return RefOps()
    raise ValueError(f"unknown op implementation {impl!r}")
