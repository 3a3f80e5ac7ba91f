"""Hand-written gfx950 GEMMs (``csrc/kernels/gemm_kernels.h``).

``gemm_swiglu(x, w_perm)`` computes the Llama MLP's ``silu(x·Wgᵀ) * (x·Wuᵀ)``
in ONE launch: the gate/up product never reaches HBM and the separate
``silu_mul`` pass disappears.  ``w_perm`` is the [2F][K] gate/up weight with
its rows permuted by :func:`swiglu_permute` so that, inside every 256-column
output tile, each wave's 64 columns are 32 gate features followed by the same
32 up features (the kernel's register layout puts g and u of one element in
the same lane).  ``gemm(x, w)`` is the plain ``x·Wᵀ`` on the same kernel,
kept for A/B measurements against hipBLASLt.

CPU / reference path: :func:`swiglu_reference` (fp32 math of the same op).
"""
from __future__ import annotations

import torch

from .. import _native

EPI_STORE = 0
EPI_SWIGLU = 2
TILE_N = 256
SWIGLU_HALF = 32   # per-wave gate/up split (a wave owns 64 output columns)


def swiglu_perm_index(ffn: int, device=None, half: int = None) -> torch.Tensor:
    """Row order of the permuted [2F][K] weight: row r of the permuted
    matrix is row ``idx[r]`` of ``cat([W_gate, W_up])``.  Each wave's
    2*half output columns are ``half`` gate features then the same ``half``
    up features (the kernel: half = 32)."""
    half = half or SWIGLU_HALF
    if ffn % (TILE_N // 2):
        raise ValueError("ffn must be a multiple of 128")
    r = torch.arange(2 * ffn, device=device)
    tn, rem = r // TILE_N, r % TILE_N
    wc, rem2 = rem // (2 * half), rem % (2 * half)
    nh, c = rem2 // half, rem2 % half
    f = tn * (TILE_N // 2) + wc * half + c
    return torch.where(nh == 0, f, ffn + f)


def swiglu_permute(w_gu: torch.Tensor, half: int = None) -> torch.Tensor:
    """[gate; up] (2F x K) -> the fused kernel's row order (contiguous)."""
    ffn = w_gu.shape[0] // 2
    return w_gu.index_select(0, swiglu_perm_index(ffn, w_gu.device, half)).contiguous()


def swiglu_unpermute(w_perm: torch.Tensor, half: int = None) -> torch.Tensor:
    ffn = w_perm.shape[0] // 2
    idx = swiglu_perm_index(ffn, w_perm.device, half)
    out = torch.empty_like(w_perm)
    out.index_copy_(0, idx, w_perm)
    return out


def swiglu_reference(x: torch.Tensor, w_gu: torch.Tensor) -> torch.Tensor:
    """fp32 reference over the UNpermuted [gate; up] weight."""
    ffn = w_gu.shape[0] // 2
    gu = x.float() @ w_gu.float().t()
    return (torch.nn.functional.silu(gu[:, :ffn]) * gu[:, ffn:]).to(x.dtype)


def _check(t: torch.Tensor, name: str):
    if t.dtype != torch.bfloat16:
        raise TypeError(f"{name}: expected bfloat16, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    if t.data_ptr() % 16:
        raise ValueError(f"{name} must be 16-byte aligned")


def supported(M: int, N: int, K: int) -> bool:
    return M > 0 and N % TILE_N == 0 and K % 128 == 0


def _launch(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, epi: int):
    k = _native.require_hipops()
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError("gemm: inner dimensions differ")
    if not supported(M, N, K):
        raise ValueError(f"gemm: unsupported shape M={M} N={N} K={K}")
    k.gemm_bf16(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, epi,
                torch.cuda.current_stream(x.device).cuda_stream)
    return out


def gemm(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """x [M][K] · w[N][K]ᵀ -> [M][N] bf16 on the hand-written kernel."""
    _check(x, "x")
    _check(w, "w")
    y = out if out is not None else torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
    _check(y, "out")
    return _launch(x, w, y, EPI_STORE)


def gemm_swiglu(x: torch.Tensor, w_perm: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """silu(x·Wgᵀ) * (x·Wuᵀ) -> [M][F] bf16, ``w_perm`` from :func:`swiglu_permute`."""
    _check(x, "x")
    _check(w_perm, "w_perm")
    F = w_perm.shape[0] // 2
    y = out if out is not None else torch.empty((x.shape[0], F), dtype=x.dtype, device=x.device)
    _check(y, "out")
    if y.shape != (x.shape[0], F):
        raise ValueError("gemm_swiglu: out shape mismatch")
    return _launch(x, w_perm, y, EPI_SWIGLU)
