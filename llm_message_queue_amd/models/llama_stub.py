"""Llama-3-8B-shaped backend stub (N12): random-init bf16 weights, one
instance per GPU, serving the gateway's dispatched requests.

The reference never calls its endpoints (`internal/loadbalancer/load_balancer.go:35-49`,
URLs from `internal/scheduler/scheduler.go:299-301`); here each endpoint is a
real GPU worker so load signals (in-flight slots, HBM) are live.

Forward = one continuous-batching step over T tokens (chunked-prefill and
decode tokens mixed).  GEMMs: ``torch.nn.functional.linear`` (hipBLASLt).
The o / down projections accumulate into the residual stream in the GEMM
epilogue (beta = 1).  Everything else: hand-written HIP kernels
(``ops.llama_ops.HipOps``): RMSNorm (optionally fused with the residual add), RoPE + KV-cache write, segment-tiled MFMA GQA attention
over the slot KV cache (prefill chunks and decode tokens), SiLU*up -- and,
with ``fused_mlp`` (default with the HIP ops), the hand-written gfx950 GEMM
with the SwiGLU epilogue for the gate/up projection (``ops.gemm``): the
[T][2F] gate/up product never reaches HBM and the silu_mul pass disappears
(``profiles/r2_gemm_swiglu.md``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch
import torch.nn.functional as F

from ..ops import gemm as G
from ..ops.llama_ops import get_ops, rope_tables


@dataclass
class LlamaConfig:
    vocab: int = 128256
    dim: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    head_dim: int = 128
    ffn: int = 14336
    rope_theta: float = 500000.0
    eps: float = 1e-5

    @classmethod
    def llama3_8b(cls) -> "LlamaConfig":
        return cls()

    @classmethod
    def tiny(cls) -> "LlamaConfig":
        """Smoke/CPU-test size (same kernels, same head_dim=128, GQA 4)."""
        return cls(vocab=1024, dim=2048, layers=2, heads=16, kv_heads=4, ffn=2048)

    @classmethod
    def by_name(cls, name: str) -> "LlamaConfig":
        n = name.lower().replace("_", "-")
        if n in ("llama3-8b", "llama-3-8b", "llama3_8b", "8b"):
            return cls.llama3_8b()
        if n == "tiny":
            return cls.tiny()
        raise ValueError(f"unknown backend model {name!r}")

    def param_count(self) -> int:
        d, f = self.dim, self.ffn
        qkv = d * (self.heads + 2 * self.kv_heads) * self.head_dim
        per = qkv + d * d + 2 * d * f + d * f + 2 * d
        return self.layers * per + 2 * self.vocab * d + d


class LlamaStub:
    def __init__(self, cfg: LlamaConfig, slots: int, max_ctx: int, device="cuda", impl: str = "hip",
                 seed: int = 0, dtype=torch.bfloat16, residual_in_gemm: bool = True, split_qkv: bool = False,
                 fused_mlp: Optional[bool] = None, min_fused_tokens: int = 512,
                 fused_qkv: Optional[bool] = None, min_fused_qkv_tokens: int = 2048, row_scale_norm: bool = True,
                 fused_head: Optional[bool] = None, fused_resid: Optional[bool] = None,
                 fused_rms: Optional[bool] = None,
                 prune_last: bool = True, library_gemm: bool = False):
        if cfg.head_dim != 128:
            raise ValueError("kernels assume head_dim = 128")
        self.cfg = cfg
        self.device = torch.device(device)
        self.ops = get_ops(impl)
        self.impl = impl
        self.slots = slots
        self.max_ctx = max_ctx
        # o / down projections accumulate straight into the residual stream
        # (hipBLASLt beta = 1: res += a @ W^T, one rounding); the following
        # RMSNorm then only reads res -- half its HBM traffic
        # (profiles/r1_gemm_experiments.md).  False: F.linear + fused
        # residual-add RMSNorm.
        self.residual_in_gemm = residual_in_gemm
        # the last layer's o projection and MLP only for the step's sampled
        # rows (see ``hidden``); False: every row, then select (A/B)
        self.prune_last = bool(prune_last)
        # QKV as two GEMMs (q: d x d, kv: 2*kv_heads*hd x d) written into
        # column slices of one qkv buffer: the fused 6144-wide GEMM at
        # T = 4096 is 384 256x256 tiles = 1.5 rounds over 256 CUs; the split
        # pair measured ~15% faster in isolation (bench/qkv_split.py) and cut
        # in-model GEMM time 4.3%, but the serving step did not get shorter
        # (profiles/r1_gemm_experiments.md), so it is off by default.  The
        # weight stays one tensor; its row slices are contiguous views.
        self.split_qkv = split_qkv
        # gate/up weight kept in the fused kernel's swiglu row order (same
        # random draw, rows permuted once at init) so the HIP path runs
        # gemm_swiglu on steps of >= min_fused_tokens rows
        self.fused_mlp = (impl == "hip") if fused_mlp is None else bool(fused_mlp)
        self.min_fused_tokens = int(min_fused_tokens)
        # qkv projection with the RoPE + K/V-cache-write epilogue (ops.gemm.qkv_rope)
        # on steps of >= min_fused_qkv_tokens rows (3.5% faster than hipBLASLt +
        # rope_kv at T = 4041, slower below ~2k rows: profiles/r2_gemm_swiglu.md)
        self.fused_qkv = (impl == "hip" and not split_qkv) if fused_qkv is None else bool(fused_qkv)
        self.min_fused_qkv_tokens = int(min_fused_qkv_tokens)
        # LM head + greedy argmax in one hand-written GEMM (argmax epilogue, no
        # [rows][vocab] logits) when the step samples >= 256 rows
        self.fused_head = (impl == "hip") if fused_head is None else bool(fused_head)
        # o / down projections into the residual on the hand-written kernel
        # (ops.gemm.RESID_EPI: the residual tile staged into LDS by DMA and
        # added in place) when its 256x256 tiles fill whole waves of the chip
        # (the saturated serving step: T ~ 4,040 -> 256 tiles); hipBLASLt's
        # beta = 1 stream-K kernel otherwise (ops.gemm.residual_tiles_ok).
        # Default since round 5: faster than hipBLASLt in isolation (o 94.8 vs
        # 95.3 us, down 299.7 vs 304.3 us at T = 4041,
        # profiles/r5_resid_ab_1gpu.jsonl) and >= it in the serving A/B
        # (profiles/r5_resid_serving_ab_1gpu.jsonl).
        self.fused_resid = (impl == "hip") if fused_resid is None else bool(fused_resid)
        # with the residual GEMM: the RMSNorm row scales of the updated
        # residual rows out of its epilogue (ops.gemm.gemm_residual_rms)
        # instead of a separate row_rms pass.  Off by default: the epilogue's
        # cross-block reduction adds 0.5-7 us to the tail of a single-wave
        # GEMM, more than the 12.8 us row_rms launch it removes saves
        # (profiles/r5_resid_rms_bench.jsonl, profiles/r5_fused_rms_serving_ab_1gpu.jsonl)
        self.fused_rms = False if fused_rms is None else bool(fused_rms)
        # False (the default since round 6): no library GEMM at any row
        # count -- skinny for small steps, 256x256 tiles (split-K where whole
        # tiles leave CUs idle) above, the argmax head at any row count.
        # True: hipBLASLt where it was faster (sub-wave o / down, the head
        # under 256 rows); measured equal within 0.4 % on the bench
        # (profiles/r6_realtime_modes.md).  fused_resid=False keeps the library.
        self.library_gemm = bool(library_gemm) or impl != "hip" or not self.fused_resid
        self._cus = G._cu_count(self.device) if (self.fused_resid and self.device.type == "cuda") else 0
        # fused paths take the raw residual rows + a per-row RMSNorm scale
        # (True) or an rmsnorm'd copy of the rows (False, A/B)
        self.row_scale_norm = bool(row_scale_norm)
        g = torch.Generator(device=self.device).manual_seed(seed)
        std = 0.02

        def w(*shape):
            return (torch.randn(*shape, generator=g, device=self.device, dtype=torch.float32) * std).to(dtype)

        d, hq, hkv, hd = cfg.dim, cfg.heads, cfg.kv_heads, cfg.head_dim
        self.embed = w(cfg.vocab, d)
        self.lm_head = w(cfg.vocab, d)
        self.final_norm = torch.ones(d, dtype=dtype, device=self.device)
        self.layers = []
        for _ in range(cfg.layers):
            L = {
                "attn_norm": torch.ones(d, dtype=dtype, device=self.device),
                "wqkv": w((hq + 2 * hkv) * hd, d),
                "wo": w(d, hq * hd),
                "mlp_norm": torch.ones(d, dtype=dtype, device=self.device),
                "w_gu": w(2 * cfg.ffn, d),
                "w_down": w(d, cfg.ffn),
            }
            # the fused paths read the raw residual rows: the RMSNorm weight
            # moves into the projection's input columns (W' = W diag(g)) and
            # the norm left on the small-step path becomes a unit-weight one
            if self.fused_qkv:
                L["wqkv"], L["attn_norm"] = self._fold_norm(L["wqkv"], L["attn_norm"])
            if self.fused_mlp:
                L["w_gu"], L["mlp_norm"] = self._fold_norm(L["w_gu"], L["mlp_norm"])
            L["w_gu"] = self._gu_layout(L["w_gu"])
            self.layers.append(L)
        # KV cache: per layer [slots, kv_heads, max_ctx, head_dim]
        self.kcache = [torch.zeros((slots, hkv, max_ctx, hd), dtype=dtype, device=self.device)
                       for _ in range(cfg.layers)]
        self.vcache = [torch.zeros((slots, hkv, max_ctx, hd), dtype=dtype, device=self.device)
                       for _ in range(cfg.layers)]
        self.cos, self.sin = rope_tables(max_ctx, cfg.rope_theta, self.device)
        self.scale = 1.0 / math.sqrt(hd)

    @staticmethod
    def _fold_norm(w: torch.Tensor, g: torch.Tensor):
        if not bool((g == 1).all()):
            w = (w.float() * g.float()[None, :]).to(w.dtype)
        return w, torch.ones_like(g)

    def _gu_layout(self, w_gu: torch.Tensor) -> torch.Tensor:
        if not self.fused_mlp:
            return w_gu
        return G.swiglu_permute(w_gu)

    def weight_bytes(self) -> int:
        n = self.embed.numel() + self.lm_head.numel() + self.final_norm.numel()
        for L in self.layers:
            n += sum(t.numel() for t in L.values())
        return n * 2

    def kv_bytes(self) -> int:
        return sum(t.numel() * 2 for t in self.kcache) * 2

    @torch.no_grad()
    def forward(self, tokens: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor,
                sample_idx: torch.Tensor, tiles: Optional[torch.Tensor] = None, n_dec: int = 0,
                small_cus: int = 0) -> torch.Tensor:
        """One step over T tokens; returns greedy next-token ids for the rows
        in ``sample_idx`` (the last token of each request's chunk).
        ``tiles`` (int32 [n, 4], see ``ops.llama_ops.make_tiles``) groups the
        tokens into per-slot segments for the MFMA attention kernel (its first
        ``n_dec`` rows are 1-token decode tiles); without it attention runs
        per token.  ``small_cus`` > 0: a small step confined to that many CUs
        (a realtime micro-forward on its CU partition) -- every GEMM on the
        hand-written kernels whatever the row count (no library kernel, none
        of whose persistent / stream-K grids assume the whole chip), split-K
        where the tiles cannot fill the partition."""
        if self.prune_last and self.residual_in_gemm:
            sel = self.hidden(tokens, pos, slot, tiles=tiles, n_dec=n_dec, rows=sample_idx, small_cus=small_cus)
        else:
            sel = self.hidden(tokens, pos, slot, tiles=tiles, n_dec=n_dec,
                              small_cus=small_cus).index_select(0, sample_idx)
        hand = small_cus or not self.library_gemm
        return self.ops.greedy_head(sel, self.lm_head, self.fused_head, min_rows=1 if hand else 256)

    @torch.no_grad()
    def hidden(self, tokens: torch.Tensor, pos: torch.Tensor, slot: torch.Tensor,
               tiles: Optional[torch.Tensor] = None, n_dec: int = 0,
               rows: Optional[torch.Tensor] = None, small_cus: int = 0) -> torch.Tensor:
        """The 32-layer trunk: final-normed hidden states [T, d] (writes the
        step's K/V into the cache).

        The residual stream ``res`` is updated in place by the o / down GEMMs.
        On steps large enough for the hand-written GEMMs, the RMSNorms before
        the qkv and gate/up projections are never materialised: ``row_rms``
        computes each row's scale, the norm weight is folded into W at init,
        and the GEMM epilogue applies the scale to its accumulator rows.

        ``rows`` (the step's sampled rows): the last layer writes every
        token's K/V and attends for every token as usual, then keeps only
        these rows for its o projection and MLP -- the other rows' outputs of
        that layer feed nothing (no later layer reads them, and the LM head
        reads only the sampled rows), so the result for ``rows`` is the same
        computation.  Returns [len(rows), d] then, else [T, d]."""
        cfg, ops = self.cfg, self.ops
        if not self.residual_in_gemm:
            return self._hidden_residual_norm(tokens, pos, slot, tiles, n_dec)
        res = F.embedding(tokens, self.embed)            # [T, d], updated in place
        T = res.shape[0]
        small = small_cus > 0 and self.impl == "hip"
        nolib = not self.library_gemm and self._cus > 0
        # the skinny kernel (a stream over the weights) for qkv up to
        # SKINNY_PROJ_MAX_M rows; larger steps: the 256x256-tile kernel, split-K
        # (profiles/r6_skinny_chunked.jsonl)
        # (on a micro-forward's CU partition only up to SKINNY_MAX_M: there the
        # split-K tiles were faster for larger steps)
        skinny = (small or nolib) and T <= (G.SKINNY_MAX_M if small else G.SKINNY_PROJ_MAX_M) \
            and self.row_scale_norm and self.fused_mlp
        sk_cus = small_cus if small else self._cus
        rows_qkv = self.fused_qkv and (T >= self.min_fused_qkv_tokens or small or nolib)
        qkv_split = {}
        if small or nolib:
            d = cfg.dim
            f = G.split_all(T, (cfg.heads + 2 * cfg.kv_heads) * cfg.head_dim, d, sk_cus)
            # every tile split when twice the tiles fit one wave; else the
            # default half-empty-last-wave plan (split_plan)
            qkv_split = {"split": True, "split_full": f} if f is not None else {}
        last = len(self.layers) - 1
        if rows is not None and rows.numel() == T:
            rows = None                                  # every row sampled: nothing to drop

        scale = None                                     # row scales of res from the previous down GEMM
        for i, L in enumerate(self.layers):
            if skinny:
                qkv = torch.empty((T, L["wqkv"].shape[0]), dtype=res.dtype, device=res.device)
                G.skinny(res, L["wqkv"], qkv, G.SK_STORE, row_scale=ops.row_rms(res, cfg.eps), cus=sk_cus)
                q = ops.rope_kv(qkv, pos, slot, self.cos, self.sin, cfg.heads, cfg.kv_heads, self.kcache[i],
                                self.vcache[i])
            elif rows_qkv and self.row_scale_norm:
                q = ops.qkv_rope_rows(res, L["wqkv"], scale if scale is not None else ops.row_rms(res, cfg.eps),
                                      pos, slot, self.cos, self.sin, cfg.heads, cfg.kv_heads, self.kcache[i],
                                      self.vcache[i], **qkv_split)
            elif rows_qkv:
                q = G.qkv_rope(ops.rmsnorm(res, L["attn_norm"], cfg.eps), L["wqkv"], pos, slot, self.cos,
                               self.sin, cfg.heads, cfg.kv_heads, self.kcache[i], self.vcache[i])
            else:
                q = self._qkv(ops.rmsnorm(res, L["attn_norm"], cfg.eps), L, i, pos, slot)
            a = self._attend(q, i, pos, slot, tiles, n_dec)
            if i == last and rows is not None:
                if rows.numel() == 0:                    # nothing sampled (a step of unfinished prefill
                    return res[:0]                       # chunks): K/V written, no row kernel gets 0 rows
                res, a = res.index_select(0, rows), a.index_select(0, rows)
            scale = self._mlp_block(res, a, L, want_scale=rows_qkv and self.row_scale_norm and i < last,
                                    small_cus=small_cus if small else 0)
        return ops.rmsnorm(res, self.final_norm, cfg.eps)

    @torch.no_grad()
    def warm_tail(self, sizes) -> int:
        """Run the last layer's o + MLP block (``_mlp_block``) once per row
        count in ``sizes`` on scratch rows: with ``prune_last`` that block
        sees the step's sampled-row count, not its token count, so its GEMM
        shapes get their own warm-up (a first use of a library kernel loads
        its code object)."""
        cfg = self.cfg
        L = self.layers[-1]
        n = 0
        for M in sizes:
            M = int(M)
            res = torch.zeros((M, cfg.dim), dtype=self.embed.dtype, device=self.device)
            a = torch.zeros((M, cfg.heads * cfg.head_dim), dtype=self.embed.dtype, device=self.device)
            self._mlp_block(res, a, L)
            n += 1
        return n

    def _mlp_block(self, res: torch.Tensor, a: torch.Tensor, L: dict, want_scale: bool = False,
                   small_cus: int = 0):
        """res += o(a); res += down(swiglu(norm(res))) -- in place, with the
        fused-path choices made for this block's row count.  Returns the
        RMSNorm row scales of the final ``res`` when ``want_scale`` and the
        down GEMM produced them in its epilogue (``fused_rms``), else None.
        ``small_cus``: a micro-forward's small step on its CU partition --
        the hand-written kernels at any row count, split-K (``forward``)."""
        cfg, ops = self.cfg, self.ops
        M = res.shape[0]
        small = small_cus > 0
        # library-free (``library_gemm`` False): the hand-written kernels at
        # every row count, split-K where whole tiles leave CUs idle
        nolib = not small and not self.library_gemm and self._cus > 0
        cus = small_cus if small else (self._cus if nolib else 0)
        rows_mlp = self.fused_mlp and (M >= self.min_fused_tokens or small or nolib)
        tiles_ok = self._cus > 0 and G.residual_tiles_ok(M, cfg.dim, self._cus)
        resid_o = small or nolib or tiles_ok
        rms = tiles_ok and self.fused_rms and G.RESID_EPI == G.EPI_RESID_LDS and not small

        # skinny: o / down up to SKINNY_RESID_MAX_M rows (past 256 its 128-row
        # chunks still beat 256x256 tiles whose 32-64 tiles leave most CUs
        # idle: profiles/r6_skinny_mid_m.jsonl), gate/up (N = 28,672: enough
        # tiles to fill the chip) only up to SKINNY_MAX_M
        skinny = (small or nolib) and M <= (G.SKINNY_MAX_M if small else G.SKINNY_RESID_MAX_M) \
            and self.row_scale_norm and self.fused_mlp
        skinny_gu = skinny and M <= G.SKINNY_MAX_M

        def into_res(x, wt, scale_out):                  # res += x · wtᵀ (+ its row scales)
            if rms and scale_out:
                return G.gemm_residual_rms(x, wt, res, cfg.eps)
            if skinny:
                G.skinny(x, wt, res, G.SK_RESID, cus=cus)
            elif resid_o:
                G.gemm_residual(x, wt, res, split_cus=cus if (small or not tiles_ok) else 0)
            else:
                res.addmm_(x, wt.t())
            return None

        scale = into_res(a, L["wo"], rows_mlp and self.row_scale_norm)
        if skinny_gu:
            act = torch.empty((M, L["w_gu"].shape[0] // 2), dtype=res.dtype, device=res.device)
            G.skinny(res, L["w_gu"], act, G.SK_SWIGLU, row_scale=ops.row_rms(res, cfg.eps), cus=cus)
        elif rows_mlp and self.row_scale_norm and (small or nolib):
            act = G.gemm_swiglu(res, L["w_gu"], row_scale=scale if scale is not None else ops.row_rms(res, cfg.eps),
                                split_cus=cus)
        elif rows_mlp and self.row_scale_norm:
            act = ops.swiglu_rows(res, L["w_gu"], scale if scale is not None else ops.row_rms(res, cfg.eps))
        elif rows_mlp:
            act = G.gemm_swiglu(ops.rmsnorm(res, L["mlp_norm"], cfg.eps), L["w_gu"])
        else:
            act = ops.mlp_up(ops.rmsnorm(res, L["mlp_norm"], cfg.eps), L["w_gu"], self.fused_mlp,
                             self.min_fused_tokens)
        return into_res(act, L["w_down"], want_scale)

    def _qkv(self, x, L, i, pos, slot):
        """qkv projection (hipBLASLt) + RoPE / KV-cache write of normalised rows."""
        cfg, ops = self.cfg, self.ops
        if self.split_qkv:
            nq = cfg.heads * cfg.head_dim
            qkv = torch.empty((x.shape[0], L["wqkv"].shape[0]), dtype=x.dtype, device=x.device)
            torch.mm(x, L["wqkv"][:nq].t(), out=qkv[:, :nq])
            torch.mm(x, L["wqkv"][nq:].t(), out=qkv[:, nq:])
        else:
            qkv = F.linear(x, L["wqkv"])
        return ops.rope_kv(qkv, pos, slot, self.cos, self.sin, cfg.heads, cfg.kv_heads,
                           self.kcache[i], self.vcache[i])

    def _attend(self, q, i, pos, slot, tiles, n_dec):
        cfg, ops = self.cfg, self.ops
        if tiles is not None:
            return ops.attention_tiles(q, self.kcache[i], self.vcache[i], tiles, cfg.heads, cfg.kv_heads,
                                       self.scale, n_dec=n_dec)
        return ops.attention(q, self.kcache[i], self.vcache[i], pos, slot, cfg.heads, cfg.kv_heads, self.scale)

    def _hidden_residual_norm(self, tokens, pos, slot, tiles, n_dec):
        """residual_in_gemm=False (A/B only): F.linear o / down projections and
        residual-add RMSNorm kernels instead of beta = 1 GEMM epilogues."""
        cfg, ops = self.cfg, self.ops
        h = F.embedding(tokens, self.embed)
        res = h.clone()
        x = ops.rmsnorm(h, self.layers[0]["attn_norm"], cfg.eps)
        out = None
        for i, L in enumerate(self.layers):
            if i > 0:
                x = ops.rmsnorm(out, L["attn_norm"], cfg.eps, residual=res)
            a = self._attend(self._qkv(x, L, i, pos, slot), i, pos, slot, tiles, n_dec)
            x2 = ops.rmsnorm(F.linear(a, L["wo"]), L["mlp_norm"], cfg.eps, residual=res)
            act = ops.mlp_up(x2, L["w_gu"], self.fused_mlp, self.min_fused_tokens)
            out = F.linear(act, L["w_down"])
        return ops.rmsnorm(out, self.final_norm, cfg.eps, residual=res)
