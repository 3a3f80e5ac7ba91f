"""Hand-written gfx950 GEMM (csrc/kernels/gemm_kernels.h, ops/gemm.py).

CPU: the swiglu weight permutation and the model's fused-MLP reference path.
GPU: the kernel against fp32 PyTorch references at T in {1, 37, 300, 4096}
(4096: the serving step), plain and SwiGLU epilogues, the permuted silu_mul,
and a tiny model forward with the fused MLP against the ref ops.
"""
import pytest
import torch

from llm_message_queue_amd.models.llama_stub import LlamaConfig, LlamaStub
from llm_message_queue_amd.ops import gemm as G
from llm_message_queue_amd.ops.llama_ops import RefOps


def test_swiglu_perm_index_is_a_permutation_in_kernel_layout():
    ffn = 512
    idx = G.swiglu_perm_index(ffn)
    assert sorted(idx.tolist()) == list(range(2 * ffn))
    # in every 256-column tile, each wave's 64 columns = 32 gate then the same 32 up
    for r in (0, 31, 32, 63, 64, 255, 256, 300, 1023):
        tn, rem = divmod(r, 256)
        wc, rem2 = divmod(rem, 64)
        nh, c = divmod(rem2, 32)
        f = tn * 128 + wc * 32 + c
        assert idx[r].item() == (f if nh == 0 else ffn + f)


def test_swiglu_permute_roundtrip_and_reference():
    torch.manual_seed(0)
    w = torch.randn(2 * 256, 64)
    wp = G.swiglu_permute(w)
    assert torch.equal(G.swiglu_unpermute(wp), w)
    x = torch.randn(5, 64)
    ref = G.swiglu_reference(x, w).float()
    # emulate the kernel's epilogue over the permuted product
    p = x @ wp.t()
    out = torch.empty(5, 256)
    for f in range(256):
        tn, r = divmod(f, 128)
        wc, c = divmod(r, 32)
        col = tn * 256 + wc * 64 + c
        out[:, f] = torch.nn.functional.silu(p[:, col]) * p[:, col + 32]
    assert torch.allclose(out, ref, atol=1e-5, rtol=1e-5)


def test_ref_silu_mul_perm_matches_unpermuted():
    torch.manual_seed(1)
    F = 256
    gu = torch.randn(7, 2 * F).to(torch.bfloat16)
    idx = G.swiglu_perm_index(F)
    gu_perm = gu.index_select(1, idx)
    ops = RefOps()
    assert torch.equal(ops.silu_mul(gu_perm, perm=True), ops.silu_mul(gu))


def test_fused_mlp_model_matches_unfused_on_ref_ops():
    cfg = LlamaConfig(vocab=512, dim=256, layers=2, heads=2, kv_heads=1, ffn=512)
    a = LlamaStub(cfg, slots=2, max_ctx=16, device="cpu", impl="ref", seed=5, fused_mlp=True)
    b = LlamaStub(cfg, slots=2, max_ctx=16, device="cpu", impl="ref", seed=5, fused_mlp=False)
    assert not torch.equal(a.layers[0]["w_gu"], b.layers[0]["w_gu"])       # stored permuted
    assert torch.equal(G.swiglu_unpermute(a.layers[0]["w_gu"]), b.layers[0]["w_gu"])
    tok = torch.randint(0, cfg.vocab, (12,), generator=torch.Generator().manual_seed(0))
    pos = torch.tensor(list(range(6)) * 2, dtype=torch.int32)
    slot = torch.tensor([0] * 6 + [1] * 6, dtype=torch.int32)
    assert torch.equal(a.hidden(tok, pos, slot), b.hidden(tok, pos, slot))


def test_row_scaled_fused_paths_match_rmsnorm_on_ref_ops():
    """The rows path (row_rms + norm weight folded into W + per-row scale in
    the fused GEMMs) computes the same trunk as rmsnorm -> GEMM, here on the
    fp32 reference ops with a non-trivial norm weight."""
    cfg = LlamaConfig(vocab=512, dim=512, layers=2, heads=4, kv_heads=2, ffn=512)
    a = LlamaStub(cfg, slots=2, max_ctx=16, device="cpu", impl="ref", seed=5, fused_mlp=True, fused_qkv=True,
                  min_fused_tokens=1, min_fused_qkv_tokens=1)
    b = LlamaStub(cfg, slots=2, max_ctx=16, device="cpu", impl="ref", seed=5, fused_mlp=False, fused_qkv=False)
    g = torch.Generator().manual_seed(3)
    for La, Lb in zip(a.layers, b.layers):
        for key in ("attn_norm", "mlp_norm"):
            gw = (1 + 0.2 * torch.randn(cfg.dim, generator=g)).to(torch.bfloat16)
            Lb[key] = gw
        La["wqkv"], _ = LlamaStub._fold_norm(Lb["wqkv"], Lb["attn_norm"])
        wg, _ = LlamaStub._fold_norm(Lb["w_gu"], Lb["mlp_norm"])
        La["w_gu"] = G.swiglu_permute(wg)
    tok = torch.randint(0, cfg.vocab, (12,), generator=torch.Generator().manual_seed(0))
    pos = torch.tensor(list(range(6)) * 2, dtype=torch.int32)
    slot = torch.tensor([0] * 6 + [1] * 6, dtype=torch.int32)
    ha, hb = a.hidden(tok, pos, slot).float(), b.hidden(tok, pos, slot).float()
    assert ((ha - hb).norm() / hb.norm()).item() < 2e-2


def test_gemm_rejects_unsupported_shapes():
    assert G.supported(37, 512, 256)
    assert not G.supported(37, 500, 256)
    assert not G.supported(37, 512, 200)
    assert not G.supported(0, 512, 256)


# ----------------------------------------------------------------------------- GPU
DEV = "cuda"


def _rand(T, K, N, seed=0):
    g = torch.Generator(device=DEV).manual_seed(seed)
    x = torch.randn(T, K, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, generator=g, device=DEV) * 0.02).to(torch.bfloat16)
    return x, w


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 37, 300, 4096])
def test_gemm_plain_matches_fp32(T):
    x, w = _rand(T, 4096, 1024, seed=T)
    ref = x.float() @ w.float().t()
    out = G.gemm(x, w).float()
    err = (out - ref).abs().max().item()
    assert err <= 0.01 * ref.abs().max().item() + 1e-3, err


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 37, 300, 4096])
def test_gemm_swiglu_matches_fp32(T):
    x, w = _rand(T, 4096, 2 * 1536, seed=100 + T)
    ref = G.swiglu_reference(x, w).float()
    out = G.gemm_swiglu(x, G.swiglu_permute(w)).float()
    err = (out - ref).abs().max().item()
    # one bf16 rounding of the output (the unfused path rounds g and u too)
    assert err <= 0.01 * ref.abs().max().item() + 1e-3, err
    assert torch.isfinite(out).all()


@pytest.mark.gpu
def test_gemm_swiglu_rows_past_m_untouched():
    """M not a multiple of 256: rows >= M of a larger output buffer stay as
    they were (loads clamp, stores mask)."""
    x, w = _rand(300, 512, 512, seed=7)
    big = torch.full((512, 256), 7.0, dtype=torch.bfloat16, device=DEV)
    G.gemm_swiglu(x, G.swiglu_permute(w), out=big[:300])
    assert (big[300:] == 7.0).all()
    ref = G.swiglu_reference(x, w).float()
    assert (big[:300].float() - ref).abs().max().item() <= 0.01 * ref.abs().max().item() + 1e-3


@pytest.mark.gpu
def test_silu_mul_perm_matches_ref():
    from llm_message_queue_amd.ops.llama_ops import HipOps
    F = 1024
    g = torch.Generator(device=DEV).manual_seed(3)
    gu = torch.randn(37, 2 * F, generator=g, device=DEV).to(torch.bfloat16)
    gu_perm = gu.index_select(1, G.swiglu_perm_index(F, DEV))
    hip = HipOps().silu_mul(gu_perm, perm=True).float()
    ref = RefOps().silu_mul(gu).float()
    assert (hip - ref).abs().max().item() < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize("T", [37, 600, 2400])
def test_tiny_model_fused_mlp_matches_ref(T):
    """The HIP model with the fused MLP (GEMM+SwiGLU for T >= 512, permuted
    silu_mul below) and the fused qkv+RoPE GEMM (T >= 2048) against the
    fp32-reference ops on the same weights."""
    cfg = LlamaConfig.tiny()
    hip = LlamaStub(cfg, slots=4, max_ctx=1024, device=DEV, impl="hip", seed=3, min_fused_tokens=512,
                    min_fused_qkv_tokens=2048)
    ref = LlamaStub(cfg, slots=4, max_ctx=1024, device=DEV, impl="ref", seed=3, residual_in_gemm=True)
    assert hip.fused_mlp and hip.fused_qkv and not ref.fused_mlp and not ref.fused_qkv
    n = T // 4
    tok = torch.randint(0, cfg.vocab, (4 * n,), device=DEV)
    pos = torch.arange(n, device=DEV, dtype=torch.int32).repeat(4)
    slot = torch.arange(4, device=DEV, dtype=torch.int32).repeat_interleave(n)
    ha = hip.hidden(tok, pos, slot).float()
    hb = ref.hidden(tok, pos, slot).float()
    rel = (ha - hb).norm() / hb.norm()
    assert rel < 2e-2, rel.item()


@pytest.mark.gpu
@pytest.mark.parametrize("T", [37, 300, 4096])
def test_qkv_rope_matches_linear_plus_rope_kv(T):
    """The qkv GEMM with the RoPE/KV epilogue == F.linear + the rope_kv
    kernel (q rows, and the K/V cache rows written at (slot, pos)); cache
    cells no token addresses stay zero."""
    from llm_message_queue_amd.ops.llama_ops import HipOps, rope_tables
    Hq, Hkv, max_ctx, S, d = 8, 2, 64, 96, 512
    g = torch.Generator(device=DEV).manual_seed(T)
    x = torch.randn(T, d, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn((Hq + 2 * Hkv) * 128, d, generator=g, device=DEV) * 0.05).to(torch.bfloat16)
    cos_t, sin_t = rope_tables(max_ctx, 500000.0, DEV)
    cell = torch.randperm(S * max_ctx, generator=g, device=DEV)[:T]
    slot, pos = (cell // max_ctx).to(torch.int32), (cell % max_ctx).to(torch.int32)
    kc1 = torch.zeros(S, Hkv, max_ctx, 128, dtype=torch.bfloat16, device=DEV)
    vc1, kc2, vc2 = torch.zeros_like(kc1), torch.zeros_like(kc1), torch.zeros_like(kc1)
    q1 = HipOps().rope_kv(torch.nn.functional.linear(x, w), pos, slot, cos_t, sin_t, Hq, Hkv, kc1, vc1)
    q2 = G.qkv_rope(x, w, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2)
    tol = 0.02 * q1.float().abs().max().item()
    assert (q1.float() - q2.float()).abs().max().item() <= tol
    assert (kc1.float() - kc2.float()).abs().max().item() <= tol
    assert (vc1.float() - vc2.float()).abs().max().item() <= tol
    untouched = torch.ones(S, max_ctx, dtype=torch.bool, device=DEV)
    untouched[slot.long(), pos.long()] = False
    assert (kc2.permute(0, 2, 1, 3)[untouched] == 0).all()


@pytest.mark.gpu
def test_serving_shapes_match_fp32():
    """The exact serving shapes of the 8B stub at a step of 4,041 tokens
    (M not a multiple of 256): gate/up + SwiGLU (N = 28672, K = 4096) and the
    qkv + RoPE epilogue (32 / 8 heads) against fp32 references."""
    from llm_message_queue_amd.ops.llama_ops import rope_tables
    T, d, ffn = 4041, 4096, 14336
    x, w = _rand(T, d, 2 * ffn, seed=77)
    ref = G.swiglu_reference(x, w).float()
    out = G.gemm_swiglu(x, G.swiglu_permute(w)).float()
    assert (out - ref).abs().max().item() <= 0.01 * ref.abs().max().item() + 1e-3
    del w, out, ref
    Hq, Hkv, max_ctx, S = 32, 8, 64, 128
    wqkv = (torch.randn((Hq + 2 * Hkv) * 128, d, generator=torch.Generator(device=DEV).manual_seed(5),
                        device=DEV) * 0.02).to(torch.bfloat16)
    cos_t, sin_t = rope_tables(max_ctx, 500000.0, DEV)
    cell = torch.randperm(S * max_ctx, device=DEV)[:T]
    slot, pos = (cell // max_ctx).to(torch.int32), (cell % max_ctx).to(torch.int32)
    kc1 = torch.zeros(S, Hkv, max_ctx, 128, dtype=torch.bfloat16, device=DEV)
    vc1, kc2, vc2 = torch.zeros_like(kc1), torch.zeros_like(kc1), torch.zeros_like(kc1)
    qkv_ref = (x.float() @ wqkv.float().t()).to(torch.bfloat16)
    from llm_message_queue_amd.ops.llama_ops import HipOps
    # reference: an fp32-accumulated product rounded to bf16, then the rope_kv kernel
    q1 = HipOps().rope_kv(qkv_ref, pos, slot, cos_t, sin_t, Hq, Hkv, kc1, vc1)
    q2 = G.qkv_rope(x, wqkv, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2)
    tol = 0.02 * q1.float().abs().max().item()
    assert (q1.float() - q2.float()).abs().max().item() <= tol
    assert (kc1.float() - kc2.float()).abs().max().item() <= tol
    assert (vc1.float() - vc2.float()).abs().max().item() <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("epi", ["regs", "lds", "pre"])
@pytest.mark.parametrize("T,K", [(1, 512), (37, 4096), (300, 1024), (4041, 4096), (4041, 14336)])
def test_gemm_residual_matches_fp32(T, K, epi):
    """res += x·wᵀ in place (the o / down projections; "regs" = GM_EPI_RESID,
    the residual tile through registers; "lds" = GM_EPI_RESID_LDS, staged by
    DMA): against the fp32 sum rounded once; rows past M of a larger buffer
    untouched."""
    N = 4096 if T == 4041 else 1024
    x, w = _rand(T, K, N, seed=300 + T)
    g = torch.Generator(device=DEV).manual_seed(T)
    big = torch.full((T + 19, N), 3.0, dtype=torch.bfloat16, device=DEV)
    big[:T] = torch.randn(T, N, generator=g, device=DEV).to(torch.bfloat16)
    res0 = big[:T].float().clone()
    ref = res0 + x.float() @ w.float().t()
    G._launch(x, w, big[:T], {"regs": G.EPI_RESID, "lds": G.EPI_RESID_LDS, "pre": G.EPI_RESID_PRE}[epi])
    err = (big[:T].float() - ref).abs().max().item()
    assert err <= 0.01 * ref.abs().max().item() + 1e-3, err
    assert (big[T:] == 3.0).all()
    if T == 4041 and K == 4096:                      # same single rounding as hipBLASLt's beta = 1
        r2 = res0.to(torch.bfloat16)
        r2.addmm_(x, w.t())
        d = (big[:T].float() - r2.float()).abs()
        assert d.max().item() <= 0.01 * ref.abs().max().item() + 1e-3
        assert (d == 0).float().mean().item() > 0.9, "residual epilogue should round like beta = 1"


@pytest.mark.gpu
@pytest.mark.parametrize("T,K", [(37, 4096), (300, 1024), (4041, 4096), (4096, 14336)])
def test_gemm_residual_rms_matches_row_rms(T, K):
    """The residual GEMM with the fused RMSNorm row scale: ``res`` exactly as
    the plain LDS epilogue leaves it, and the scales equal ``row_rms`` of the
    updated rows (fp32, a different summation order); twice in a row (the
    tickets the last block re-zeroes), bit-identical."""
    from llm_message_queue_amd.ops.llama_ops import HipOps
    N = 4096
    x, w = _rand(T, K, N, seed=700 + T)
    g = torch.Generator(device=DEV).manual_seed(T + 1)
    res0 = torch.randn(T, N, generator=g, device=DEV).to(torch.bfloat16)
    r_plain = res0.clone()
    G._launch(x, w, r_plain, G.EPI_RESID_LDS)
    scales = []
    for _ in range(2):
        r_rms = res0.clone()
        sc = G.gemm_residual_rms(x, w, r_rms, 1e-5)
        torch.cuda.synchronize()
        assert torch.equal(r_rms, r_plain)
        scales.append(sc[:T].clone())
    assert torch.equal(scales[0], scales[1])
    ref = HipOps().row_rms(r_plain, 1e-5)[:T]
    assert torch.allclose(scales[0], ref, rtol=1e-5, atol=0), (scales[0] - ref).abs().max().item()
    exact = r_plain.float().pow(2).mean(-1).add(1e-5).rsqrt()
    assert torch.allclose(scales[0], exact, rtol=1e-4, atol=0)


@pytest.mark.gpu
def test_8b_model_fused_rms_matches_row_rms_path():
    """The model with the row scales from the residual GEMM's epilogue
    (``fused_rms``, an A/B option) against the separate row_rms pass (the
    default): same hidden states to bf16 noise at a full-chip step, and
    row_rms runs only for layer 0's qkv."""
    from llm_message_queue_amd.ops import llama_ops
    cfg = LlamaConfig(layers=3)
    a = LlamaStub(cfg, slots=64, max_ctx=128, device=DEV, impl="hip", seed=6, fused_rms=True)
    b = LlamaStub(cfg, slots=64, max_ctx=128, device=DEV, impl="hip", seed=6)
    assert a.fused_rms and not b.fused_rms
    T = 4041
    if not G.residual_tiles_ok(T, cfg.dim, a._cus):
        pytest.skip(f"{a._cus} CUs: T = {T} is not a whole wave of tiles here")
    calls = []
    orig = llama_ops.HipOps.row_rms
    llama_ops.HipOps.row_rms = lambda self, *x: (calls.append(1), orig(self, *x))[1]
    try:
        tok = torch.randint(0, cfg.vocab, (T,), device=DEV)
        pos = (torch.arange(T, device=DEV, dtype=torch.int32) % 64)
        slot = (torch.arange(T, device=DEV, dtype=torch.int32) // 64)
        ha = a.hidden(tok, pos, slot).float()
        n_fused = len(calls)
        hb = b.hidden(tok, pos, slot).float()
    finally:
        llama_ops.HipOps.row_rms = orig
    assert n_fused == 1 and len(calls) - n_fused == 2 * cfg.layers
    rel = ((ha - hb).norm() / hb.norm()).item()
    assert rel < 1e-2, rel


@pytest.mark.gpu
def test_8b_model_residual_gemm_matches_hipblaslt_path():
    """At a full-chip step (T = 4041 -> 256 tiles of o / down) the model's
    o / down projections run on the residual GEMM epilogue (the default
    since round 5); hidden states equal the hipBLASLt beta = 1 path to bf16
    noise (2 layers, 8B dims)."""
    cfg = LlamaConfig(layers=2)
    a = LlamaStub(cfg, slots=64, max_ctx=128, device=DEV, impl="hip", seed=5)
    b = LlamaStub(cfg, slots=64, max_ctx=128, device=DEV, impl="hip", seed=5, fused_resid=False)
    assert G.RESID_EPI == G.EPI_RESID_LDS
    T = 4041
    assert a.fused_resid and a._cus > 0 and not b.fused_resid
    if not G.residual_tiles_ok(T, cfg.dim, a._cus):
        pytest.skip(f"{a._cus} CUs: T = {T} is not a whole wave of tiles here")
    called = []
    orig, orig_rms = G.gemm_residual, G.gemm_residual_rms
    G.gemm_residual = lambda *x, **kw: (called.append(1), orig(*x, **kw))[1]
    G.gemm_residual_rms = lambda *x: (called.append(1), orig_rms(*x))[1]      # (with the row scales)
    try:
        tok = torch.randint(0, cfg.vocab, (T,), device=DEV)
        pos = (torch.arange(T, device=DEV, dtype=torch.int32) % 64)
        slot = (torch.arange(T, device=DEV, dtype=torch.int32) // 64)
        ha = a.hidden(tok, pos, slot).float()
        hb = b.hidden(tok, pos, slot).float()
    finally:
        G.gemm_residual, G.gemm_residual_rms = orig, orig_rms
    assert len(called) == 2 * cfg.layers
    rel = ((ha - hb).norm() / hb.norm()).item()
    assert rel < 1e-2, rel


def test_residual_tiles_ok_wants_whole_waves():
    assert G.residual_tiles_ok(4041, 4096, 256)                 # 16 x 16 = 256 tiles: one full wave
    assert G.residual_tiles_ok(3841, 4096, 256)                 # 16 x 16 tiles (the last M-tile holds 1 row)
    assert not G.residual_tiles_ok(3840, 4096, 256)             # 15 x 16 = 240 tiles: 94 % of the chip
    assert not G.residual_tiles_ok(2048, 4096, 256)             # 128 tiles: half the chip
    assert G.residual_tiles_ok(8192, 4096, 256)                 # two full waves
    assert not G.residual_tiles_ok(4041, 4000, 256)             # N not a multiple of 256
    assert not G.residual_tiles_ok(0, 4096, 256)


def test_split_plan_only_splits_a_half_empty_last_wave():
    assert G.split_plan(4041, 6144, 4096, 256) == 256          # 384 tiles: 256 whole + 128 split
    assert G.split_plan(2600, 6144, 4096, 256) == 256          # 264 tiles: 8 split
    assert G.split_plan(2048, 6144, 4096, 256) is None         # 192 tiles: one wave already
    assert G.split_plan(4096, 8192, 4096, 256) is None         # 512 tiles: two full waves
    assert G.split_plan(5000, 6144, 4096, 256) is None         # 480 tiles: tail 224 > half
    assert G.split_plan(4041, 6144, 384, 256) is None          # K too short to halve


@pytest.mark.gpu
@pytest.mark.parametrize("T", [2600, 4041])
def test_qkv_rope_split_k_tail_matches_unsplit(T):
    """The split-K last wave (two blocks per tile over one K-half each,
    fp32 handoff through a workspace) == the unsplit kernel, over repeated
    launches (the counters are re-zeroed by the kernel itself)."""
    from llm_message_queue_amd.ops.llama_ops import rope_tables
    d, Hq, Hkv, max_ctx, S = 4096, 32, 8, 64, 128
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    if G.split_plan(T, (Hq + 2 * Hkv) * 128, d, cus) is None:
        pytest.skip(f"no split on {cus} CUs")
    g = torch.Generator(device=DEV).manual_seed(T)
    x = torch.randn(T, d, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn((Hq + 2 * Hkv) * 128, d, generator=g, device=DEV) * 0.02).to(torch.bfloat16)
    cos_t, sin_t = rope_tables(max_ctx, 500000.0, DEV)
    cell = torch.randperm(S * max_ctx, generator=g, device=DEV)[:T]
    slot, pos = (cell // max_ctx).to(torch.int32), (cell % max_ctx).to(torch.int32)
    kc1 = torch.zeros(S, Hkv, max_ctx, 128, dtype=torch.bfloat16, device=DEV)
    vc1 = torch.zeros_like(kc1)
    q1 = G.qkv_rope(x, w, pos, slot, cos_t, sin_t, Hq, Hkv, kc1, vc1, split=False)
    for it in range(3):
        kc2, vc2 = torch.zeros_like(kc1), torch.zeros_like(kc1)
        q2 = G.qkv_rope(x, w, pos, slot, cos_t, sin_t, Hq, Hkv, kc2, vc2, split=True)
        tol = 0.01 * q1.float().abs().max().item()
        assert (q1.float() - q2.float()).abs().max().item() <= tol, it
        assert (kc1.float() - kc2.float()).abs().max().item() <= tol, it
        assert (vc1.float() - vc2.float()).abs().max().item() <= tol, it
    _, cnt = G._SPLIT_WS[("cuda", 0, torch.cuda.current_stream().cuda_stream)]
    assert int(cnt.abs().sum()) == 0                             # left zeroed for the next launch


@pytest.mark.gpu
def test_row_rms_and_row_scaled_swiglu_match_rmsnorm_path():
    from llm_message_queue_amd.ops.llama_ops import HipOps
    ops = HipOps()
    x, w = _rand(300, 4096, 2 * 1024, seed=21)
    x = (x.float() * 3.0).to(torch.bfloat16)
    r = ops.row_rms(x, 1e-5)
    assert r.numel() == 512                                    # padded to whole 256-row tiles
    ref_r = torch.rsqrt(x.float().pow(2).mean(-1) + 1e-5)
    assert torch.allclose(r[:300], ref_r, rtol=1e-4, atol=1e-6)
    ones = torch.ones(4096, dtype=torch.bfloat16, device=DEV)
    ref = G.swiglu_reference(ops.rmsnorm(x, ones, 1e-5), w).float()
    out = G.gemm_swiglu(x, G.swiglu_permute(w), row_scale=r).float()
    assert (out - ref).abs().max().item() <= 0.02 * ref.abs().max().item() + 1e-3


@pytest.mark.gpu
@pytest.mark.parametrize("M", [256, 300, 1000])
def test_lm_head_argmax_matches_fp32_argmax(M):
    """LM head with the argmax epilogue == argmax of the fp32 logits (a
    mismatch is only allowed between near-tied logits)."""
    V, d = 128256, 4096
    g = torch.Generator(device=DEV).manual_seed(M)
    x = torch.randn(M, d, generator=g, device=DEV).to(torch.bfloat16)
    w = (torch.randn(V, d, generator=g, device=DEV) * 0.02).to(torch.bfloat16)
    got = G.lm_head_argmax(x, w).long()
    ref = torch.empty(M, V, device=DEV)
    for i in range(0, M, 128):                                   # fp32 logits in row chunks
        ref[i:i + 128] = x[i:i + 128].float() @ w.float().t()
    exp = ref.argmax(1)
    bad = (got != exp).nonzero().flatten()
    assert bad.numel() <= max(1, M // 100), bad.numel()
    for i in bad.tolist():
        gap = (ref[i, exp[i]] - ref[i, got[i]]).item()
        assert 0 <= gap <= 1e-3 * ref[i].abs().max().item(), (i, gap)


@pytest.mark.gpu
def test_lm_head_argmax_ties_pick_the_lowest_column():
    V, d = 128256, 256
    x = torch.zeros(256, d, device=DEV)
    w = torch.zeros(V, d, device=DEV)
    x[0, 0] = 1.0
    w[[300, 1000, 70000], 0] = 2.0                               # tie across tiles
    x[1, 1] = 1.0
    w[[515, 513, 77777], 1] = 3.0                                # tie inside one tile (513, 515) and across
    x[2, 2] = -1.0
    w[:, 2] = 1.0
    w[12345, 2] = -5.0                                           # single maximum, negative logits
    got = G.lm_head_argmax(x.to(torch.bfloat16), w.to(torch.bfloat16)).tolist()
    assert got[0] == 300 and got[1] == 513 and got[2] == 12345
    assert all(t == 0 for t in got[3:])                          # all-zero rows: every logit ties at 0


@pytest.mark.gpu
def test_tiny_model_fused_head_matches_fp32_argmax():
    """The model's fused head returns the argmax of the fp32 logits of its
    hidden states (the unfused path argmaxes bf16-rounded logits, which tie
    often at this model's logit scale -- it is not the reference here)."""
    from llm_message_queue_amd.models.llama_stub import LlamaConfig, LlamaStub
    cfg = LlamaConfig.tiny()
    a = LlamaStub(cfg, slots=5, max_ctx=64, device=DEV, impl="hip", seed=3, fused_head=True)
    T = 300                                                      # distinct (slot, pos) cells
    tok = torch.randint(0, cfg.vocab, (T,), device=DEV)
    pos = (torch.arange(T, device=DEV) % 64).to(torch.int32)
    slot = (torch.arange(T, device=DEV) // 64).to(torch.int32)
    samp = torch.arange(T, device=DEV)
    xf = a.hidden(tok, pos, slot)
    ref = (xf.float() @ a.lm_head.float().t())
    got = a.ops.greedy_head(xf, a.lm_head, True).long()
    exp = ref.argmax(1)
    for i in (got != exp).nonzero().flatten().tolist():
        gap = (ref[i, exp[i]] - ref[i, got[i]]).item()
        assert 0 <= gap <= 1e-3 * ref[i].abs().max().item(), (i, gap)
    # forward() (hidden + the fused head) gives the same tokens: the trunk is deterministic
    assert torch.equal(a.forward(tok, pos, slot, samp).long(), got)


# ---------------------------------------------------------------------- split-K for small steps (micro partition)
def test_split_all_plans_only_when_twice_the_tiles_fit():
    assert G.split_all(37, 4096, 4096, 32) == 0              # 16 tiles -> 32 K-half blocks on 32 CUs
    assert G.split_all(37, 6144, 4096, 32) is None           # 24 tiles: 48 blocks would not fit one wave
    assert G.split_all(300, 4096, 14336, 64) == 0            # 32 tiles on 64 CUs
    assert G.split_all(37, 4096, 384, 32) is None            # K too short to halve in whole 128-deep steps
    assert G.split_all(37, 4096, 4096, 0) is None


@pytest.mark.gpu
@pytest.mark.parametrize("T,K", [(1, 4096), (37, 4096), (64, 14336), (300, 4096)])
def test_split_k_store_swiglu_residual_match_fp32(T, K):
    """Every tile split over two K-half blocks (the micro partition's small
    steps): store, SwiGLU (with row scales) and the residual epilogue equal
    the fp32 reference of the whole product."""
    x, w = _rand(T, K, 4096, seed=11 * T + K)
    ref = x.float() @ w.float().t()
    out = G.gemm(x, w, split_cus=256).float()
    assert (out - ref).abs().max().item() <= 0.01 * ref.abs().max().item() + 1e-3
    res = torch.randn(T, 4096, device=DEV).to(torch.bfloat16)
    want = res.float() + ref
    got = G.gemm_residual(x, w, res.clone(), split_cus=256).float()
    assert (got - want).abs().max().item() <= 0.01 * want.abs().max().item() + 1e-2
    xs, ws = _rand(T, K, 2 * 1024, seed=7 * T + K)
    r = torch.rand(G.row_scale_len(T), device=DEV) + 0.5
    sref = G.swiglu_reference((xs.float() * r[:T, None]).to(torch.bfloat16), ws).float()
    sout = G.gemm_swiglu(xs, G.swiglu_permute(ws), row_scale=r, split_cus=256).float()
    assert (sout - sref).abs().max().item() <= 0.02 * sref.abs().max().item() + 1e-3


@pytest.mark.gpu
def test_small_step_forward_matches_the_serving_path():
    """The 8B-shaped stub's small-step mode (hand-written kernels at any row
    count, split-K, argmax head) gives the same greedy ids as the serving
    path (library GEMMs at these row counts) -- the micro-forwards' numerics."""
    from llm_message_queue_amd.models.llama_stub import LlamaConfig, LlamaStub
    cfg = LlamaConfig(vocab=32000, dim=4096, layers=2, heads=32, kv_heads=8, ffn=14336)
    m = LlamaStub(cfg, slots=8, max_ctx=64, device=DEV, impl="hip", seed=5, library_gemm=True)
    T = 40
    tok = torch.randint(0, cfg.vocab, (T,), device=DEV)
    pos = torch.arange(T, device=DEV, dtype=torch.int32) % 20
    slot = (torch.arange(T, device=DEV, dtype=torch.int32) // 20)
    samp = torch.tensor([19, 39], device=DEV, dtype=torch.long)
    a = m.hidden(tok, pos, slot, rows=samp).float()
    m2 = LlamaStub(cfg, slots=8, max_ctx=64, device=DEV, impl="hip", seed=5)
    b = m2.hidden(tok, pos, slot, rows=samp, small_cus=32).float()
    assert (a - b).abs().max().item() <= 0.03 * a.abs().max().item()
    # the small step's head: the argmax epilogue at 2 rows = argmax of the fp32 logits
    sel = b.to(torch.bfloat16)
    ids = m2.ops.greedy_head(sel, m2.lm_head, True, min_rows=1)
    assert ids.tolist() == torch.argmax(sel.float() @ m2.lm_head.float().t(), dim=-1).tolist()


@pytest.mark.gpu
@pytest.mark.parametrize("M", [1, 17, 40, 64, 65, 128, 129, 200, 256, 300, 640, 1000])
@pytest.mark.parametrize("N,K", [(4096, 4096), (1024, 14336), (6144, 512)])
def test_skinny_gemm_matches_fp32(M, N, K):
    """The skinny kernel (M <= 64 in one block; up to 256 rows in 128-row
    chunks of A; split-K partials summed in order): store and residual
    epilogues with a row scale, equal to the fp32 reference."""
    x, w = _rand(M, K, N, seed=3 * M + N + K)
    r = torch.rand(M, device=DEV) + 0.5
    ref = (x.float() * r[:, None]) @ w.float().t()
    out = torch.empty(M, N, dtype=torch.bfloat16, device=DEV)
    G.skinny(x, w, out, G.SK_STORE, row_scale=r, cus=32)
    assert (out.float() - ref).abs().max().item() <= 0.01 * ref.abs().max().item() + 1e-3
    res = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    want = res.float() + x.float() @ w.float().t()
    got = res.clone()
    G.skinny(x, w, got, G.SK_RESID, cus=32)
    assert (got.float() - want).abs().max().item() <= 0.01 * want.abs().max().item() + 1e-2
    again = res.clone()
    G.skinny(x, w, again, G.SK_RESID, cus=32)
    assert torch.equal(got, again)                            # deterministic (partials summed in order)


@pytest.mark.gpu
@pytest.mark.parametrize("M", [3, 64, 160])
def test_skinny_swiglu_matches_fp32(M):
    x, w = _rand(M, 4096, 2 * 1536, seed=40 + M)
    r = torch.rand(M, device=DEV) + 0.5
    ref = G.swiglu_reference((x.float() * r[:, None]).to(torch.bfloat16), w).float()
    out = torch.empty(M, 1536, dtype=torch.bfloat16, device=DEV)
    G.skinny(x, G.swiglu_permute(w), out, G.SK_SWIGLU, row_scale=r, cus=32)
    assert (out.float() - ref).abs().max().item() <= 0.02 * ref.abs().max().item() + 1e-3


def test_split_cus_falls_back_to_the_tail_plan():
    """``split_cus`` splits every tile when twice the tiles fit one wave, else
    only a half-empty last wave (what the library-free path relies on)."""
    assert G.split_all(300, 4096, 4096, 224) == 0            # 32 tiles -> 64 blocks
    assert G.split_all(3000, 4096, 4096, 224) is None        # 192 tiles: whole
    assert G.split_plan(3000, 4096, 4096, 224) is None       # one 86 % wave
    assert G.split_plan(4041, 4096, 14336, 224) == 224       # 256 tiles: 224 whole + 32 split


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 37, 300, 900, 3000, 4041])
@pytest.mark.parametrize("K", [4096, 14336])
def test_library_free_residual_matches_fp32(T, K):
    """o / down into the residual on the hand-written kernels at every row
    count the serving steps produce: the skinny kernel
    for T <= 64, 256x256 tiles with split-K otherwise -- each equal to the
    fp32 ``res + x·wᵀ`` and to hipBLASLt's beta = 1 ``addmm_`` within one
    bf16 rounding of the output."""
    cus = G._cu_count(DEV)
    x, w = _rand(T, K, 4096, seed=T + K)
    res = torch.randn(T, 4096, device=DEV).to(torch.bfloat16)
    want = res.float() + x.float() @ w.float().t()
    got = res.clone()
    if T <= G.SKINNY_MAX_M:
        G.skinny(x, w, got, G.SK_RESID, cus=cus)
    else:
        G.gemm_residual(x, w, got, split_cus=cus)
    tol = 0.01 * want.abs().max().item() + 1e-2
    assert (got.float() - want).abs().max().item() <= tol
    lib = res.clone().addmm_(x, w.t())
    assert (got.float() - lib.float()).abs().max().item() <= tol


@pytest.mark.gpu
@pytest.mark.parametrize("T", [1, 40, 165, 256, 300, 512, 513, 900])
def test_library_free_model_matches_the_default_routing(T):
    """``library_gemm=False`` (no hipBLASLt call in the forward) gives the
    same hidden rows as the default routing to bf16 tolerance and the same
    greedy ids."""
    from llm_message_queue_amd.models.llama_stub import LlamaConfig, LlamaStub
    cfg = LlamaConfig(vocab=32000, dim=4096, layers=2, heads=32, kv_heads=8, ffn=14336)
    tok = torch.randint(0, cfg.vocab, (T,), device=DEV)
    pos = torch.arange(T, device=DEV, dtype=torch.int32) % 64
    slot = (torch.arange(T, device=DEV, dtype=torch.int32) // 64)
    samp = torch.arange(min(T, 63), T, 64, device=DEV, dtype=torch.long)
    if samp.numel() == 0:
        samp = torch.tensor([T - 1], device=DEV, dtype=torch.long)
    out = []
    for lib in (True, False):
        m = LlamaStub(cfg, slots=16, max_ctx=64, device=DEV, impl="hip", seed=5, library_gemm=lib)
        out.append((m.hidden(tok, pos, slot, rows=samp).float(),
                    m.forward(tok, pos, slot, sample_idx=samp).tolist()))
    a, b = out[0][0], out[1][0]
    assert (a - b).abs().max().item() <= 0.03 * a.abs().max().item()
    # greedy ids agree wherever the top-2 logit gap exceeds the routing's difference
    W = m.lm_head.float()
    la, lb = a.to(torch.bfloat16).float() @ W.t(), b.to(torch.bfloat16).float() @ W.t()
    top = torch.topk(la, 2, dim=-1).values
    clear = ((top[:, 0] - top[:, 1]) > 2 * (la - lb).abs().max(dim=-1).values).tolist()
    for i, (x, y) in enumerate(zip(out[0][1], out[1][1])):
        assert x == y or not clear[i]
