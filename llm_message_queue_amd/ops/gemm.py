"""Hand-written gfx950 GEMMs (``csrc/kernels/gemm_kernels.h``).

``gemm_swiglu(x, w_perm)`` computes the Llama MLP's ``silu(x·Wgᵀ) * (x·Wuᵀ)``
in ONE launch: the gate/up product never reaches HBM and the separate
``silu_mul`` pass disappears.  ``w_perm`` is the [2F][K] gate/up weight with
its rows permuted by :func:`swiglu_permute` so that, inside every 256-column
output tile, each wave's 64 columns are 32 gate features followed by the same
32 up features (the kernel's register layout puts g and u of one element in
the same lane).  ``gemm(x, w)`` is the plain ``x·Wᵀ`` on the same kernel,
kept for A/B measurements against hipBLASLt.  ``qkv_rope`` runs the qkv
projection with the RoPE + K/V-cache-write epilogue (replacing F.linear +
``rope_kv``).

CPU / reference path: :func:`swiglu_reference` (fp32 math of the same op).
"""
from __future__ import annotations

import functools

import torch

from .. import _native

EPI_STORE = 0
EPI_SWIGLU = 2
EPI_RESID = 5       # A/B: residual tile read into registers in the epilogue
EPI_RESID_LDS = 6   # residual tile staged into LDS by DMA, added in place (default)
EPI_RESID_PRE = 7   # A/B: ... its first quarter fetched into spare LDS at kernel start
# which residual epilogue ``gemm_residual`` launches (bench.py --resid-epi)
RESID_EPI = EPI_RESID_LDS
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


def row_scale_len(M: int) -> int:
    """Floats a row_scale buffer must hold: the kernel reads whole 256-row
    tiles of it (rows past M are read but never stored)."""
    return (M + 255) // 256 * 256


def _row_scale_ptr(rs, M: int) -> int:
    if rs is None:
        return 0
    if rs.dtype != torch.float32 or not rs.is_contiguous() or rs.numel() < row_scale_len(M):
        raise ValueError("row_scale must be a contiguous float32 tensor of >= ceil(M/256)*256 values "
                         "(ops.llama_ops.HipOps.row_rms pads)")
    if rs.data_ptr() % 16:
        raise ValueError("row_scale must be 16-byte aligned")
    return rs.data_ptr()


def split_all(M: int, N: int, K: int, cus: int):
    """Split-K for a step too small to fill ``cus`` CUs with whole tiles:
    every tile runs as two K-half blocks (returns 0 = the first whole
    tile index) when twice the tiles still fit one wave, else None."""
    tiles = (M + TILE_M - 1) // TILE_M * (N // TILE_N)
    if cus <= 0 or 2 * tiles > cus or K % 256 or K < 512:
        return None
    return 0


def _launch(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, epi: int, group_m: int = 8, row_scale=None,
            split_cus: int = 0):
    k = _native.require_hipops()
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K:
        raise ValueError("gemm: inner dimensions differ")
    if not supported(M, N, K):
        raise ValueError(f"gemm: unsupported shape M={M} N={N} K={K}")
    stream = torch.cuda.current_stream(x.device).cuda_stream
    f = None
    if split_cus:                                      # every tile split, else only a half-empty last wave
        f = split_all(M, N, K, split_cus)
        f = split_plan(M, N, K, split_cus) if f is None else f
    ws = cnt = 0
    if f is not None:
        n_split = (M + TILE_M - 1) // TILE_M * (N // TILE_N) - f
        w_t, c_t = _split_workspace(x.device, stream, n_split, max(split_cus, 2 * n_split))
        ws, cnt = w_t.data_ptr(), c_t.data_ptr()
    k.gemm_bf16(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, epi, stream, group_m,
                _row_scale_ptr(row_scale, M), f or 0, ws, cnt)
    return out


def gemm(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None, row_scale=None,
         split_cus: int = 0) -> torch.Tensor:
    """x [M][K] · w[N][K]ᵀ -> [M][N] bf16 on the hand-written kernel
    (``row_scale`` [M] fp32: output row i is multiplied by row_scale[i];
    ``split_cus``: run split-K when the tiles cannot fill that many CUs,
    :func:`split_all`, or on a half-empty last wave, :func:`split_plan`)."""
    _check(x, "x")
    _check(w, "w")
    y = out if out is not None else torch.empty((x.shape[0], w.shape[0]), dtype=x.dtype, device=x.device)
    _check(y, "out")
    return _launch(x, w, y, EPI_STORE, row_scale=row_scale, split_cus=split_cus)


def gemm_swiglu(x: torch.Tensor, w_perm: torch.Tensor, out: torch.Tensor = None, row_scale=None,
                split_cus: int = 0) -> torch.Tensor:
    """silu(x·Wgᵀ) * (x·Wuᵀ) -> [M][F] bf16, ``w_perm`` from :func:`swiglu_permute`.
    ``row_scale`` [M] fp32 scales row i of both products first: with the
    RMSNorm weight folded into W and row_scale = ``row_rms(x)`` this is the
    MLP of rmsnorm(x) without materialising the normalised rows."""
    _check(x, "x")
    _check(w_perm, "w_perm")
    F = w_perm.shape[0] // 2
    y = out if out is not None else torch.empty((x.shape[0], F), dtype=x.dtype, device=x.device)
    _check(y, "out")
    if y.shape != (x.shape[0], F):
        raise ValueError("gemm_swiglu: out shape mismatch")
    return _launch(x, w_perm, y, EPI_SWIGLU, row_scale=row_scale, split_cus=split_cus)


_RMS_WS = {}


def _rms_workspace(device, stream: int, tiles_m: int, tiles_n: int):
    """Per-(device, stream) scratch of the fused row-scale epilogue: fp32
    row partials [tiles_m * tiles_n * 256] and int tickets [tiles_m] (zero;
    every launch leaves them zero), grown on demand."""
    key = (device.type, device.index, stream)
    ws = _RMS_WS.get(key)
    if ws is None or ws[0].numel() < tiles_m * tiles_n * 256 or ws[1].numel() < tiles_m:
        tm = max(tiles_m, ws[1].numel() if ws else 0)
        ws = (torch.empty(tm * max(tiles_n, 16) * 256, dtype=torch.float32, device=device),
              torch.zeros(tm, dtype=torch.int32, device=device))
        _RMS_WS[key] = ws
    return ws


def gemm_residual_rms(x: torch.Tensor, w: torch.Tensor, res: torch.Tensor, eps: float) -> torch.Tensor:
    """``res += x · wᵀ`` (the LDS-DMA residual epilogue) and, in the same
    launch, the RMSNorm row scale of the updated ``res``: returns fp32
    [row_scale_len(M)] holding ``1 / sqrt(mean(res[r]^2) + eps)`` for rows
    r < M -- ``HipOps.row_rms(res, eps)`` without its separate pass over the
    rows (the next fused GEMM applies it per row).  Sums of squares are
    added in a fixed order, so the result is deterministic; it matches
    ``row_rms`` to fp32 rounding of a different summation order."""
    _check(x, "x")
    _check(w, "w")
    _check(res, "res")
    M, K = x.shape
    N = w.shape[0]
    if res.shape != (M, N):
        raise ValueError("gemm_residual_rms: res shape mismatch")
    stream = torch.cuda.current_stream(x.device).cuda_stream
    tiles_m, tiles_n = (M + TILE_M - 1) // TILE_M, N // TILE_N
    part, ticket = _rms_workspace(x.device, stream, tiles_m, tiles_n)
    scale = torch.empty(row_scale_len(M), dtype=torch.float32, device=x.device)
    _native.require_hipops().gemm_residual_rms(x.data_ptr(), w.data_ptr(), res.data_ptr(), M, N, K, stream,
                                               8, part.data_ptr(), ticket.data_ptr(), scale.data_ptr(),
                                               float(eps))
    return scale


def gemm_residual(x: torch.Tensor, w: torch.Tensor, res: torch.Tensor, split_cus: int = 0) -> torch.Tensor:
    """``res += x · wᵀ`` in place (bf16 ``res`` [M][N]; the fp32 sum is
    rounded once, as hipBLASLt's beta = 1 epilogue) -- the o / down
    projections accumulating into the residual stream.  Pulling the residual
    tile into L2 during the K-loop drain (4 or 8 MFMA phases ahead of the
    epilogue) was measured at +0.0-0.1 % (no gain: the epilogue is not
    waiting on the read; profiles/r3_gemm_resid_prefetch_ab.jsonl), so the
    plain epilogue stays."""
    _check(x, "x")
    _check(w, "w")
    _check(res, "res")
    if res.shape != (x.shape[0], w.shape[0]):
        raise ValueError("gemm_residual: res shape mismatch")
    if split_cus and RESID_EPI != EPI_RESID_LDS:
        split_cus = 0                                  # (split-K is wired for the LDS epilogue only)
    return _launch(x, w, res, RESID_EPI, split_cus=split_cus)


def residual_tiles_ok(M: int, N: int, cus: int, min_fill: float = 0.97) -> bool:
    """Whether the 256x256-tile kernel fills the chip for ``res += x·wᵀ``:
    the last wave of tiles at least ``min_fill`` busy.  On a partial wave
    (e.g. 128 tiles on 256 CUs) hipBLASLt's stream-K kernel splits K across
    the idle CUs and stays ahead (profiles/r2_gemm_resid_ab.jsonl)."""
    if not supported(M, N, 128) or N % TILE_N:
        return False
    tiles = -(-M // TILE_M) * (N // TILE_N)
    waves = -(-tiles // cus)
    return tiles / (waves * cus) >= min_fill


TILE_M = 256
_SPLIT_WS = {}


def split_plan(M: int, N: int, K: int, cus: int):
    """Split-K for the last, partial wave of tiles: returns ``full`` (tiles
    run whole) or None.  The kernel holds one block per CU, so ``tiles`` over
    ``cus`` CUs is ceil(tiles / cus) waves; when the last wave is at most half
    full its tiles run as two blocks over one K-half each (one wave of
    ``cus`` becomes half a wave).  qkv at the serving shape: 16 x 24 = 384
    tiles on 256 CUs -> 256 whole + 128 split."""
    tiles = (M + TILE_M - 1) // TILE_M * (N // TILE_N)
    tail = tiles % cus
    if tiles <= cus or tail == 0 or 2 * tail > cus or K % 256 or K < 512:
        return None
    return tiles - tail


def _split_workspace(device, stream: int, n_split: int, cus: int):
    """fp32 slabs (256 KiB per split tile) + zeroed ticket/ready counters,
    sized for the largest possible tail (cus / 2).  The kernel re-zeroes the
    counters it used, so launches in stream order can share them; the cache
    is keyed by (device, stream) so concurrent streams never do."""
    key = (device.type, device.index, stream)
    ws = _SPLIT_WS.get(key)
    if ws is None or n_split > ws[1].numel() // 2:
        # (grown in stream order: a launch still using the old slabs is ahead
        # on this same stream, and the caching allocator reuses them after it)
        cap = max(cus // 2, n_split, ws[1].numel() // 2 if ws is not None else 0)
        ws = (torch.empty(cap * 512 * 128, dtype=torch.float32, device=device),
              torch.zeros(cap * 2, dtype=torch.int32, device=device))
        _SPLIT_WS[key] = ws
    return ws


@functools.lru_cache(maxsize=None)
def _cu_count_idx(index: int) -> int:
    return torch.cuda.get_device_properties(index).multi_processor_count


# device index -> CUs the serving steps' stream may use, when the chip is
# split into CU partitions (backend.cu_partition): wave / split-K plans are
# sized for the partition, not the whole chip
EFFECTIVE_CUS = {}


def _cu_count(device) -> int:
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return EFFECTIVE_CUS.get(idx) or _cu_count_idx(idx)


def qkv_rope(x: torch.Tensor, wqkv: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor,
             cos_t: torch.Tensor, sin_t: torch.Tensor, Hq: int, Hkv: int,
             kc: torch.Tensor, vc: torch.Tensor, q_out: torch.Tensor = None, row_scale=None,
             split: bool = True, split_full: int = None, group_m: int = 8) -> torch.Tensor:
    """The qkv projection with RoPE + the K/V cache write as its epilogue:
    returns q [T][Hq*128] (rotated) and writes this step's K/V rows into
    ``kc`` / ``vc`` [slots][Hkv][max_ctx][128] -- the same result as
    ``F.linear`` followed by ``HipOps.rope_kv``, without the [T][qkv]
    intermediate or the second launch.  ``row_scale`` as in :func:`gemm_swiglu`
    (applied to q, k and v before the rotation).  ``split``: run a partial
    last wave of tiles split-K (:func:`split_plan`)."""
    _check(x, "x")
    _check(wqkv, "wqkv")
    for t, n in ((kc, "kc"), (vc, "vc")):
        _check(t, n)
    if pos.dtype != torch.int32 or slot.dtype != torch.int32 or not (pos.is_contiguous() and slot.is_contiguous()):
        raise TypeError("pos / slot must be contiguous int32")
    if cos_t.dtype != torch.float32 or sin_t.dtype != torch.float32 or cos_t.shape[1] != 64:
        raise TypeError("cos / sin tables must be float32 [max_ctx][64]")
    T, K = x.shape
    S, hk, max_ctx, hd = kc.shape
    if hk != Hkv or hd != 128 or vc.shape != kc.shape or cos_t.shape[0] < max_ctx:
        raise ValueError("kv cache / rope table shape mismatch")
    if pos.numel() != T or slot.numel() != T:
        raise ValueError("pos / slot length must equal the token count")
    q = q_out if q_out is not None else torch.empty((T, Hq * 128), dtype=x.dtype, device=x.device)
    _check(q, "q_out")
    k = _native.require_hipops()
    N = wqkv.shape[0]
    full, ws, cnt = 0, 0, 0
    stream = torch.cuda.current_stream(x.device).cuda_stream
    if split:
        cus = _cu_count(x.device)
        f = split_plan(T, N, K, cus) if split_full is None else split_full
        if f is not None:
            n_split = (T + TILE_M - 1) // TILE_M * (N // TILE_N) - f
            w_t, c_t = _split_workspace(x.device, stream, n_split, cus)
            full, ws, cnt = f, w_t.data_ptr(), c_t.data_ptr()
    k.gemm_qkv_rope(x.data_ptr(), wqkv.data_ptr(), T, N, K, pos.data_ptr(), slot.data_ptr(),
                    cos_t.data_ptr(), sin_t.data_ptr(), Hq, Hkv, max_ctx, S, q.data_ptr(), kc.data_ptr(),
                    vc.data_ptr(), stream, _row_scale_ptr(row_scale, T), full, ws, cnt, group_m)
    return q


# ---------------------------------------------------------------------- skinny small steps
SKINNY_MAX_M = 64              # the model's gate/up on the skinny kernel up to this many rows
SKINNY_PROJ_MAX_M = 256        # ... and qkv up to this many (profiles/r6_skinny_chunked.jsonl)
SKINNY_RESID_MAX_M = 512       # ... and o / down (into the residual) up to this many (profiles/r6_skinny_mid_m.jsonl)
SKINNY_CHUNKED_MAX_M = 1024    # the kernel itself: 128-row chunks of A up to this many rows
SK_STORE, SK_RESID, SK_SWIGLU = 0, 1, 2
_SKINNY_WS = {}


def skinny_splits(N: int, K: int, cus: int, M: int = 1) -> int:
    """Split-K factor of a skinny GEMM: the fewest K-splits that give at
    least two blocks (128 columns x one 128-row chunk of M) per CU, each
    split a multiple of 128 deep and at least 512."""
    blocks = N // 128 * max(1, -(-M // 128))
    best = 1
    for s in (1, 2, 4, 7, 8, 14, 16):
        if K % (128 * s) or K // s < 512:
            continue
        best = s
        if blocks * s >= 2 * cus:
            break
    return best


def skinny(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor, epi: int, row_scale=None, cus: int = 32,
           splits: int = 0):
    """``out`` (+)= ``x`` [M <= 1024][K] . ``w`` [N][K]^T on the skinny kernel
    (``csrc/kernels/skinny_kernels.h``): SK_STORE (out [M][N]), SK_RESID
    (out += ..., one rounding), SK_SWIGLU (``w`` swiglu-permuted, out [M][N/2]);
    ``row_scale`` multiplies row i of the product first (the folded RMSNorm).
    ``cus``: CUs the launch may use (the split-K factor is sized for them);
    ``splits`` > 0 forces the split-K factor (measurements)."""
    _check(x, "x")
    _check(w, "w")
    _check(out, "out")
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K or not 1 <= M <= SKINNY_CHUNKED_MAX_M or N % 128 or K % 128:
        raise ValueError(f"skinny: unsupported shape M={M} N={N} K={K}")
    want = (M, N // 2) if epi == SK_SWIGLU else (M, N)
    if tuple(out.shape) != want:
        raise ValueError(f"skinny: out shape {tuple(out.shape)} != {want}")
    S = splits or skinny_splits(N, K, cus, M)
    if K % (128 * S):
        raise ValueError(f"skinny: K={K} does not split {S} ways in 128-deep steps")
    stream = torch.cuda.current_stream(x.device).cuda_stream
    key = (x.device.type, x.device.index, stream)
    need = S * M * N
    ws = _SKINNY_WS.get(key)
    if ws is None or ws.numel() < need:
        ws = _SKINNY_WS[key] = torch.empty(max(need, SKINNY_MAX_M * 32768), dtype=torch.float32, device=x.device)
    rs = 0
    if row_scale is not None:
        if row_scale.dtype != torch.float32 or not row_scale.is_contiguous() or row_scale.numel() < M:
            raise ValueError("skinny: row_scale must be contiguous float32 [>= M]")
        rs = row_scale.data_ptr()
    _native.require_hipops().skinny_gemm(x.data_ptr(), w.data_ptr(), out.data_ptr(), M, N, K, epi, rs,
                                         ws.data_ptr(), S, stream)
    return out


_ARGMAX_WS = {}


def lm_head_argmax(x: torch.Tensor, w: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """Greedy next tokens ``argmax_n (x . w[n])`` -> int32 [M] with the argmax
    in the GEMM epilogue: no [M][vocab] logits tensor is written or re-read
    (the LM head of the serving step: ~1k rows x 128k vocab).  Ties resolve
    to the lower index as torch.argmax does; the values compared are the fp32
    accumulators, not bf16-rounded logits.  Scratch [M][N/256] (value, column)
    partials are cached per (device, stream)."""
    _check(x, "x")
    _check(w, "w")
    M, K = x.shape
    N = w.shape[0]
    if w.shape[1] != K or not supported(M, N, K):
        raise ValueError(f"lm_head_argmax: unsupported shape M={M} N={N} K={K}")
    stream = torch.cuda.current_stream(x.device).cuda_stream
    key = (x.device.type, x.device.index, stream)
    need = M * (N // TILE_N)
    ws = _ARGMAX_WS.get(key)
    if ws is None or ws[0].numel() < need:
        n = max(need, 2 * ws[0].numel() if ws is not None else 0)
        ws = _ARGMAX_WS[key] = (torch.empty(n, dtype=torch.float32, device=x.device),
                                torch.empty(n, dtype=torch.int32, device=x.device))
    y = out if out is not None else torch.empty(M, dtype=torch.int32, device=x.device)
    if y.dtype != torch.int32 or y.numel() < M or not y.is_contiguous():
        raise ValueError("lm_head_argmax: out must be contiguous int32 [M]")
    _native.require_hipops().gemm_argmax(x.data_ptr(), w.data_ptr(), M, N, K, ws[0].data_ptr(), ws[1].data_ptr(),
                                         y.data_ptr(), stream)
    return y

