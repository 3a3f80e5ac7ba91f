// Decode-path kernels of the Llama-3-8B-shaped backend stub (N12): fused
// residual-add + RMSNorm, SiLU*up, RoPE + paged KV write, and a unified
// prefill/decode GQA attention over the slot KV cache.  The big GEMMs with
// fused epilogues (qkv + RoPE/KV write, gate/up + SwiGLU, LM head + argmax)
// are the hand-written MFMA kernels of gemm_kernels.h; the o / down
// projections stay on hipBLASLt's beta = 1 residual GEMM.
//
// Unified attention: every token of a step (prefill chunk tokens and decode
// tokens alike) carries (slot, pos); its K/V are written to the slot's cache
// at `pos` BEFORE attention, and the token then attends to cache[0..pos].
// Causality is therefore by construction and one kernel serves chunked
// prefill and decode.  KV cache layout per layer: [slot][kv_head][max_ctx][128]
// so one (slot, kv head)'s keys are contiguous.
//
// Attention tiling (gfx950): one 256-thread workgroup per (token, kv head);
// its 4 waves are the GQA group's 4 query heads.  K and V are staged 64 keys
// at a time into LDS (register-staged 16-B loads, rows padded to 272 B so the
// per-lane row reads of the QK^T dot products are bank-conflict free), shared
// by the 4 heads; softmax is online (running max/sum per wave).

#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "summarise_kernels.h"

namespace llmq {

typedef __attribute__((ext_vector_type(8))) unsigned short u16x8;

__device__ __forceinline__ float bf(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}

// y = rmsnorm(x (+ residual)) * w.  If `res` is non-null: res <- x + res (the
// new residual stream) and the norm is taken of that sum.  D = NPASS * 2048
// (one 256-thread block per row, 8 bf16 per thread per pass); NPASS is a
// template parameter so every pass's 16-B loads are issued before the first
// is consumed (D = 4096 for the 8B model: 2 loads in flight per thread).
template <int NPASS>
__global__ void __launch_bounds__(256)
rmsnorm_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
               uint16_t* __restrict__ y, int D, float eps) {
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  constexpr int npass = NPASS;
  float v[NPASS][8];
  float ss = 0.f;
#pragma unroll
  for (int p = 0; p < npass; ++p) {
    const int col = p * 2048 + tid * 8;
    const u16x8 xv = *reinterpret_cast<const u16x8*>(x + (int64_t)row * D + col);
    u16x8 rv;
    if (res) rv = *reinterpret_cast<const u16x8*>(res + (int64_t)row * D + col);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float a = bf(xv[k]);
      if (res) a += bf(rv[k]);
      v[p][k] = a;
    }
    if (res) {
      u16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o[k] = f32_to_bf16_rne(v[p][k]);
      *reinterpret_cast<u16x8*>(res + (int64_t)row * D + col) = o;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[p][k] = bf(o[k]);  // norm of the rounded residual
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) ss += v[p][k] * v[p][k];
  }
  __shared__ float red[4];
  ss = wave_sum(ss);
  if ((tid & 63) == 0) red[tid >> 6] = ss;
  __syncthreads();
  const float tot = red[0] + red[1] + red[2] + red[3];
  const float inv = rsqrtf(tot / (float)D + eps);
#pragma unroll
  for (int p = 0; p < npass; ++p) {
    const int col = p * 2048 + tid * 8;
    const u16x8 wv = *reinterpret_cast<const u16x8*>(w + col);
    u16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = f32_to_bf16_rne(v[p][k] * inv * bf(wv[k]));
    *reinterpret_cast<u16x8*>(y + (int64_t)row * D + col) = o;
  }
}

// r[t] = 1 / sqrt(mean(x[t]^2) + eps): the RMSNorm scale only (one wave per
// row, 4 rows per block).  The fused GEMMs apply it to their accumulator rows
// with the norm weight folded into W, so the normalised activations are never
// written (ops/gemm.py row_scale).
__global__ void __launch_bounds__(256)
row_rms_kernel(const uint16_t* __restrict__ x, float* __restrict__ r, int T, int D, float eps) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= T) return;
  const int lane = threadIdx.x & 63;
  const uint16_t* xr = x + (int64_t)row * D;
  float ss = 0.f;
  for (int c = lane * 8; c < D; c += 512) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(xr + c);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float a = bf(v[k]);
      ss += a * a;
    }
  }
  ss = wave_sum(ss);
  if (lane == 0) r[row] = rsqrtf(ss / (float)D + eps);
}

// out[t, i] = silu(gu[t, i]) * gu[t, F + i], 8 elements per thread.
__global__ void __launch_bounds__(256)
silu_mul_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out, int T, int F, int perm) {
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  const int64_t total = (int64_t)T * F;
  if (idx >= total) return;
  const int64_t t = idx / F;
  const int64_t i = idx % F;
  // perm: gu columns in the fused GEMM's swiglu order (ops/gemm.py
  // swiglu_perm_index, half = 32): feature i sits at column
  // (i/128)*256 + ((i%128)/32)*64 + i%32, its up value 32 columns later.
  const int64_t gc = perm ? (i >> 7) * 256 + ((i & 127) >> 5) * 64 + (i & 31) : i;
  const int64_t uc = perm ? gc + 32 : F + i;
  const u16x8 g = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + gc);
  const u16x8 u = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + uc);
  u16x8 o;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const float a = bf(g[k]);
    const float s = a / (1.0f + __expf(-a));
    o[k] = f32_to_bf16_rne(s * bf(u[k]));
  }
  *reinterpret_cast<u16x8*>(out + idx) = o;
}

// RoPE (rotate-half, Llama-3) on q and k of the fused qkv projection, then
// write k/v into this layer's cache at (slot, pos).  One block per token;
// thread t takes rotary pairs 4j..4j+3 (j = t & 15) of head slot t >> 4, so a
// head is 16 threads x 8-B accesses (two coalesced 128-B halves: dims i and
// i + 64) and a block covers 16 heads per pass.
__global__ void __launch_bounds__(256)
rope_kv_kernel(const uint16_t* __restrict__ qkv, const int32_t* __restrict__ pos,
               const int32_t* __restrict__ slot, const float* __restrict__ cos_t,
               const float* __restrict__ sin_t, int Hq, int Hkv, int max_ctx, int n_slots,
               uint16_t* __restrict__ q_out, uint16_t* __restrict__ kc, uint16_t* __restrict__ vc) {
  const int t = blockIdx.x;
  const int tid = threadIdx.x;
  const int j = tid & 15;            // pairs 4j .. 4j+3
  const int hs = tid >> 4;           // head slot 0..15
  const int p = pos[t];
  const int s = slot[t];
  // a corrupt descriptor must not become a wild KV-cache write (GPU fault):
  // out-of-range (slot, pos) rows are dropped
  if ((unsigned)s >= (unsigned)n_slots || (unsigned)p >= (unsigned)max_ctx) return;
  const float4 c = *reinterpret_cast<const float4*>(cos_t + (int64_t)p * 64 + 4 * j);
  const float4 sn = *reinterpret_cast<const float4*>(sin_t + (int64_t)p * 64 + 4 * j);
  const float cc[4] = {c.x, c.y, c.z, c.w}, ss[4] = {sn.x, sn.y, sn.z, sn.w};
  const int64_t row = (int64_t)t * (Hq + 2 * Hkv) * 128;
  auto rot = [&](uint2 lo, uint2 hi, uint2* olo, uint2* ohi) {
    const uint16_t* a = reinterpret_cast<const uint16_t*>(&lo);
    const uint16_t* b = reinterpret_cast<const uint16_t*>(&hi);
    uint16_t* oa = reinterpret_cast<uint16_t*>(olo);
    uint16_t* ob = reinterpret_cast<uint16_t*>(ohi);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float x0 = bf(a[k]), x1 = bf(b[k]);
      oa[k] = f32_to_bf16_rne(x0 * cc[k] - x1 * ss[k]);
      ob[k] = f32_to_bf16_rne(x1 * cc[k] + x0 * ss[k]);
    }
  };
  for (int h = hs; h < Hq; h += 16) {
    const uint2 lo = *reinterpret_cast<const uint2*>(qkv + row + h * 128 + 4 * j);
    const uint2 hi = *reinterpret_cast<const uint2*>(qkv + row + h * 128 + 64 + 4 * j);
    uint2 olo, ohi;
    rot(lo, hi, &olo, &ohi);
    uint16_t* dst = q_out + (int64_t)t * Hq * 128 + h * 128;
    *reinterpret_cast<uint2*>(dst + 4 * j) = olo;
    *reinterpret_cast<uint2*>(dst + 64 + 4 * j) = ohi;
  }
  for (int h = hs; h < Hkv; h += 16) {
    const int64_t kb = row + (int64_t)(Hq + h) * 128;
    const int64_t vb = row + (int64_t)(Hq + Hkv + h) * 128;
    const uint2 lo = *reinterpret_cast<const uint2*>(qkv + kb + 4 * j);
    const uint2 hi = *reinterpret_cast<const uint2*>(qkv + kb + 64 + 4 * j);
    uint2 olo, ohi;
    rot(lo, hi, &olo, &ohi);
    const int64_t dst = (((int64_t)s * Hkv + h) * max_ctx + p) * 128;
    *reinterpret_cast<uint2*>(kc + dst + 4 * j) = olo;
    *reinterpret_cast<uint2*>(kc + dst + 64 + 4 * j) = ohi;
    *reinterpret_cast<uint2*>(vc + dst + 4 * j) = *reinterpret_cast<const uint2*>(qkv + vb + 4 * j);
    *reinterpret_cast<uint2*>(vc + dst + 64 + 4 * j) = *reinterpret_cast<const uint2*>(qkv + vb + 64 + 4 * j);
  }
}

constexpr int AT_KEYS = 64;
constexpr int AT_ROW = 136;  // 128 bf16 + 8 pad (272 B rows)

__global__ void __launch_bounds__(256)
attention_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                 const uint16_t* __restrict__ vc, const int32_t* __restrict__ pos,
                 const int32_t* __restrict__ slot, int Hq, int Hkv, int max_ctx, int n_slots, float scale,
                 uint16_t* __restrict__ out) {
  __shared__ __align__(16) uint16_t Ks[AT_KEYS * AT_ROW];
  __shared__ __align__(16) uint16_t Vs[AT_KEYS * AT_ROW];
  __shared__ __align__(16) float qs[4][128];
  __shared__ float ps[4][AT_KEYS];
  const int t = blockIdx.x / Hkv;
  const int g = blockIdx.x % Hkv;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int group = Hq / Hkv;      // 4 for Llama-3-8B
  const int h = g * group + wv;
  const int ctx = pos[t] + 1;
  const int s = slot[t];
  if ((unsigned)s >= (unsigned)n_slots || ctx < 1 || ctx > max_ctx) return;   // whole block: no barrier skipped
  const int64_t kvbase = ((int64_t)s * Hkv + g) * max_ctx * 128;

  if (wv < group) {
    qs[wv][lane] = bf(q[((int64_t)t * Hq + h) * 128 + lane]) * scale;
    qs[wv][lane + 64] = bf(q[((int64_t)t * Hq + h) * 128 + lane + 64]) * scale;
  }
  float m = -3.0e38f, l = 0.f, acc0 = 0.f, acc1 = 0.f;

  for (int k0 = 0; k0 < ctx; k0 += AT_KEYS) {
    __syncthreads();
    // stage 64 keys x 128 dims of K and V: 1024 16-B chunks each, 4 per thread
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = tid + r * 256;
      const int key = c >> 4, ch = c & 15;
      uint4 kv = make_uint4(0u, 0u, 0u, 0u), vv = make_uint4(0u, 0u, 0u, 0u);
      if (k0 + key < ctx) {
        kv = *reinterpret_cast<const uint4*>(kc + kvbase + (int64_t)(k0 + key) * 128 + ch * 8);
        vv = *reinterpret_cast<const uint4*>(vc + kvbase + (int64_t)(k0 + key) * 128 + ch * 8);
      }
      *reinterpret_cast<uint4*>(Ks + key * AT_ROW + ch * 8) = kv;
      *reinterpret_cast<uint4*>(Vs + key * AT_ROW + ch * 8) = vv;
    }
    __syncthreads();
    if (wv >= group) continue;
    // scores: lane j = key k0 + j
    float sc = 0.f;
#pragma unroll
    for (int ch = 0; ch < 16; ++ch) {
      const u16x8 kk = *reinterpret_cast<const u16x8*>(Ks + lane * AT_ROW + ch * 8);
      const float4 qa = *reinterpret_cast<const float4*>(&qs[wv][ch * 8]);
      const float4 qb = *reinterpret_cast<const float4*>(&qs[wv][ch * 8 + 4]);
      sc += qa.x * bf(kk[0]) + qa.y * bf(kk[1]) + qa.z * bf(kk[2]) + qa.w * bf(kk[3]) +
            qb.x * bf(kk[4]) + qb.y * bf(kk[5]) + qb.z * bf(kk[6]) + qb.w * bf(kk[7]);
    }
    const bool live = (k0 + lane) < ctx;
    sc = live ? sc : -3.0e38f;
    const float mn = fmaxf(m, wave_max(sc));
    const float pj = live ? __expf(sc - mn) : 0.f;
    const float corr = __expf(m - mn);
    l = l * corr + wave_sum(pj);
    acc0 *= corr;
    acc1 *= corr;
    m = mn;
    ps[wv][lane] = pj;
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    const int nk = min(AT_KEYS, ctx - k0);
    for (int j = 0; j < nk; ++j) {
      const float p = ps[wv][j];
      const uint32_t v2 = *reinterpret_cast<const uint32_t*>(Vs + j * AT_ROW + lane * 2);
      acc0 += p * bf((uint16_t)(v2 & 0xFFFFu));
      acc1 += p * bf((uint16_t)(v2 >> 16));
    }
  }
  if (wv < group) {
    const float inv = 1.0f / l;
    uint32_t o = (uint32_t)f32_to_bf16_rne(acc0 * inv) | ((uint32_t)f32_to_bf16_rne(acc1 * inv) << 16);
    *reinterpret_cast<uint32_t*>(out + ((int64_t)t * Hq + h) * 128 + lane * 2) = o;
  }
}

// ---------------------------------------------------------------------------
// Segment-tiled MFMA attention (the serving path).  A step's tokens come in
// SEGMENTS: a run of consecutive positions of one slot (a prefill chunk; a
// decode token is a segment of 1).  The engine cuts segments into tiles of
// <= 16 tokens: tiles[i] = {first token row, n, slot, first position}.
//
// One 256-thread workgroup per (tile, kv head); wave w = query head g*4+w of
// the GQA group, so every wave owns a 16-token x 128 Q block (A operand, kept
// in registers) and the 4 waves share the K/V block staged in LDS -- K/V of a
// slot are read ONCE per tile instead of once per token (a 12-token prefill
// chunk reads its context 12x less than the per-token kernel above).
//   S = Q K^T : v_mfma_f32_16x16x32_bf16, 4 key tiles x 4 k-steps per 64 keys;
//               K rows staged with 16-B chunks XOR-swizzled by (key & 15) so
//               the B-fragment reads (16 keys, one chunk each) hit 16 banks;
//   softmax   : online, causal mask key <= pos0 + row, exp2 with the scale
//               folded into log2(e); row max/sum reduced over the 16 lanes
//               that hold a row (C layout: lane = (row quad fq, key fr));
//   O += P V  : P goes through a per-wave LDS tile (C layout -> A layout),
//               V is staged TRANSPOSED (Vt[dim][key], 2 keys packed per
//               dword write) so B fragments are 16-B reads; 8 dim tiles x
//               2 k-steps per 64 keys, O in 32 accumulator VGPRs.
//
// XCD mapping: blockIdx = tile * Hkv + g and workgroups are dealt round-robin
// to the 8 XCDs, so with Hkv = 8 every tile's kv head g runs on XCD g: the
// tiles of one prefill chunk (which re-read each other's K/V rows) share that
// XCD's L2 by construction, with no remap needed.
//
// KEYS (32 or 64) is the key block per iteration.  Serving prompts are short
// (<= 32 tokens), so the 32-key block does no masked MFMA work on them and
// halves the LDS and score registers: more workgroups resident per CU, and
// this latency-bound kernel runs in fewer rounds.  Long dialog contexts loop
// over more blocks.
// LDS elements (bf16) of one segment-attention block: K tile | V^T tile |
// per-wave P tiles; after the key loop the same bytes stage the output tiles
template <int KEYS>
constexpr int seg_lds_elems() { return KEYS * 128 + 128 * (KEYS + 8) + 4 * 16 * (KEYS + 8); }

template <int KEYS>
__device__ __forceinline__ void attention_seg_block(int bid, uint16_t* __restrict__ smem,
                                                    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                    const uint16_t* __restrict__ vc, const int32_t* __restrict__ tiles,
                                                    int Hq, int Hkv, int max_ctx, int n_slots, int T,
                                                    float scale_log2, uint16_t* __restrict__ out) {
  static_assert(KEYS == 32 || KEYS == 64, "key block");
  constexpr int SA_KEYS = KEYS;
  constexpr int SA_VROW = KEYS + 8;   // Vt row: KEYS keys + 8 pad
  constexpr int SA_PROW = KEYS + 8;   // P row
  constexpr int NJ = KEYS / 16;       // 16-key score tiles per block
  constexpr int NKS = KEYS / 32;      // 32-key PV k-steps per block
  constexpr int SA_OROW = 136;                        // O staging row: 128 dims + 8 pad
  static_assert(seg_lds_elems<KEYS>() >= 4 * 16 * SA_OROW, "output staging must fit");
  uint16_t* Ks = smem;
  uint16_t* Vt = smem + SA_KEYS * 128;
  const int tile = bid / Hkv;
  const int g = bid % Hkv;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int tok0 = tiles[tile * 4 + 0];
  const int n = tiles[tile * 4 + 1];
  const int s = tiles[tile * 4 + 2];
  const int pos0 = tiles[tile * 4 + 3];
  // block-uniform descriptor check (before any barrier): a corrupt tile is skipped, never dereferenced
  if ((unsigned)s >= (unsigned)n_slots || n < 1 || n > 16 || pos0 < 0 || pos0 + n > max_ctx || tok0 < 0 ||
      tok0 + n > T)
    return;
  const int h = g * 4 + wv;
  const int ctx = pos0 + n;
  const int64_t kvbase = ((int64_t)s * Hkv + g) * max_ctx * 128;

  // Q fragments (A operand): row = token fr of the tile, dims ks*32 + fq*8 .. +7
  bf16x8 qf[4];
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    qf[ks] = bf16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (fr < n) qf[ks] = *reinterpret_cast<const bf16x8*>(q + ((int64_t)(tok0 + fr) * Hq + h) * 128 + ks * 32 + fq * 8);
  }
  f32x4 o[8];
#pragma unroll
  for (int nt = 0; nt < 8; ++nt) o[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrow[4] = {-3.0e38f, -3.0e38f, -3.0e38f, -3.0e38f};
  float lrow[4] = {0.f, 0.f, 0.f, 0.f};
  uint16_t* P = smem + SA_KEYS * 128 + 128 * SA_VROW + wv * 16 * SA_PROW;

  for (int k0 = 0; k0 < ctx; k0 += SA_KEYS) {
    __syncthreads();
    // K: KEYS keys x 16 chunks of 16 B staged by DMA (buffer_load ... lds:
    // no VGPRs, issued before the V loads so both share one round trip).
    // Wave wv's j-th instruction fills LDS chunks [(wv NKI + j) 64, +64) of
    // Ks, lane l chunk P: key P / 16 at swizzled slot P % 16 = ch ^ (key &
    // 15), i.e. source chunk ch = (P % 16) ^ (key & 15).  Keys >= ctx read 0
    // off the buffer descriptor (num_records ends at key ctx).  The round-4
    // form loaded into registers under a per-key predicate, which compiled
    // to a load -> vmcnt(0) -> store chain (profiles/r5_attn_ab.jsonl).
    {
      constexpr int NKI = KEYS * 16 / 256;
      const __amdgpu_buffer_rsrc_t krs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(kc + kvbase + (int64_t)k0 * 128), 0, (uint32_t)(ctx - k0) * 256u, 0x00020000);
#pragma unroll
      for (int j = 0; j < NKI; ++j) {
        const int P = (wv * NKI + j) * 64 + lane;
        const int key = P >> 4, ch = (P & 15) ^ (key & 15);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            krs, (__attribute__((address_space(3))) void*)(Ks + (wv * NKI + j) * 64 * 8), 16,
            (uint32_t)(key * 256 + ch * 16), 0, 0, 0);
      }
    }
    // V^T: item = (key pair kp, chunk ch); two keys per dword store.  The
    // rows come through a buffer descriptor ending at key ctx: unconditional
    // loads (keys >= ctx read 0), all in flight together with the K DMA
    {
      const __amdgpu_buffer_rsrc_t vrs = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(vc + kvbase + (int64_t)k0 * 128), 0, (uint32_t)(ctx - k0) * 256u, 0x00020000);
      typedef unsigned int vu32x4 __attribute__((ext_vector_type(4)));
      vu32x4 va[KEYS / 32], vb[KEYS / 32];
#pragma unroll
      for (int r = 0; r < KEYS / 32; ++r) {
        const int c = tid + r * 256;
        const int kp = c % (KEYS / 2), ch = c / (KEYS / 2);
        va[r] = __builtin_bit_cast(vu32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, (2 * kp) * 256 + ch * 16, 0, 0));
        vb[r] = __builtin_bit_cast(vu32x4, __builtin_amdgcn_raw_buffer_load_b128(vrs, (2 * kp + 1) * 256 + ch * 16, 0, 0));
      }
#pragma unroll
      for (int r = 0; r < KEYS / 32; ++r) {
        const int c = tid + r * 256;
        const int kp = c % (KEYS / 2), ch = c / (KEYS / 2);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t a = va[r][i], b = vb[r][i];
          *reinterpret_cast<uint32_t*>(Vt + (ch * 8 + 2 * i) * SA_VROW + 2 * kp) = (a & 0xFFFFu) | (b << 16);
          *reinterpret_cast<uint32_t*>(Vt + (ch * 8 + 2 * i + 1) * SA_VROW + 2 * kp) = (a >> 16) | (b & 0xFFFF0000u);
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0): this wave's K DMA has landed
    __syncthreads();

    // ---- S = Q K^T (C layout: sc[j][k] = S[row 4fq+k][key k0 + 16j + fr])
    f32x4 sc[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      sc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (j * 16 + fr) * 128 + (((ks * 4 + fq) ^ fr) * 8));
        sc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf, sc[j], 0, 0, 0);
      }
    }
    // ---- online softmax over this block (rows 4fq+k live in the 16 lanes of quad fq)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int row = 4 * fq + k;
      const int lim = (row < n) ? pos0 + row : -1;       // causal: key <= position
      float mx = -3.0e38f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int key = k0 + j * 16 + fr;
        const float v = (key <= lim) ? sc[j][k] * scale_log2 : -3.0e38f;
        sc[j][k] = v;
        mx = fmaxf(mx, v);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
      const float mn = fmaxf(mrow[k], mx);
      const float corr = exp2f(mrow[k] - mn);
      float sum = 0.f;
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int key = k0 + j * 16 + fr;
        const float p = (key <= lim) ? exp2f(sc[j][k] - mn) : 0.f;
        sum += p;
        P[row * SA_PROW + j * 16 + fr] = f32_to_bf16_rne(p);
      }
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 64);
      lrow[k] = lrow[k] * corr + sum;
      mrow[k] = mn;
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) o[nt][k] *= corr;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // this wave's P stores landed (lgkmcnt 0)
    __builtin_amdgcn_wave_barrier();
    // ---- O += P V
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      const bf16x8 pf = *reinterpret_cast<const bf16x8*>(P + fr * SA_PROW + ks * 32 + fq * 8);
#pragma unroll
      for (int nt = 0; nt < 8; ++nt) {
        const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vt + (nt * 16 + fr) * SA_VROW + ks * 32 + fq * 8);
        o[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, o[nt], 0, 0, 0);
      }
    }
  }
  // ---- epilogue: o[nt][k] = O[row 4fq+k][dim 16nt + fr] -> LDS (row-major,
  // 272-B rows: the 4 row-quads of a store land 16 banks apart) -> 16-B
  // global stores of whole row chunks (4 per lane instead of 32 2-byte ones)
  __syncthreads();                                    // every wave is done with K / V^T / P
  uint16_t* Os = smem + wv * 16 * SA_OROW;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int row = 4 * fq + k;
    const float inv = row < n ? 1.0f / lrow[k] : 0.f;
#pragma unroll
    for (int nt = 0; nt < 8; ++nt) Os[row * SA_OROW + nt * 16 + fr] = f32_to_bf16_rne(o[nt][k] * inv);
  }
  __builtin_amdgcn_s_waitcnt(0xC07F);                 // this wave's O stores landed (lgkmcnt 0)
  __builtin_amdgcn_wave_barrier();
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int c = lane + 64 * r;                      // 16 rows x 16 chunks of 8 dims
    const int row = c >> 4, ch = c & 15;
    if (row < n)
      *reinterpret_cast<uint4*>(out + ((int64_t)(tok0 + row) * Hq + h) * 128 + ch * 8) =
          *reinterpret_cast<const uint4*>(Os + row * SA_OROW + ch * 8);
  }
}

template <int KEYS>
__global__ void __launch_bounds__(256, KEYS == 32 ? 4 : 3)
attention_seg_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                     const uint16_t* __restrict__ vc, const int32_t* __restrict__ tiles, int Hq, int Hkv,
                     int max_ctx, int n_slots, int T, float scale_log2, uint16_t* __restrict__ out) {
  __shared__ __align__(16) uint16_t smem[seg_lds_elems<KEYS>()];
  attention_seg_block<KEYS>(blockIdx.x, smem, q, kc, vc, tiles, Hq, Hkv, max_ctx, n_slots, T, scale_log2, out);
}

// ---------------------------------------------------------------------------
// Decode attention (1-token tiles): one WAVE per (token, kv head), the GQA
// group's 4 query heads handled together by that wave, 4 independent items
// per 256-thread workgroup (no block barrier).  A decode token attends a
// short context (tens to hundreds of keys) that no other token of the step
// shares, so the kernel is latency-bound and is laid out to shorten the
// dependent chain per wave:
//   * scores: 8 keys per pass, 8 lanes per key, each lane 16 dims of the K
//     row (two 16-B loads; the 8 lanes of a key read its 256-B row) against
//     the 4 heads' q slices held in registers as bf16 pairs,
//     v_dot2c_f32_bf16 (fp32 accumulate); the 8 partial dots are combined
//     with 3 xor-shuffles.  A 26-key context is 4 passes of 2 loads + 32 dot2
//     per lane (a lane-per-key layout idles 60% of the lanes on it);
//   * online softmax over the 64-key block with lane = key (wave max/sum);
//   * P.V: the two half-waves take even / odd keys, each lane 4 dims (one
//     8-B load per key; a half-wave reads a 256-B V row), so the serial key
//     loop is half as long; the halves are summed with one xor-32 shuffle.
// LDS: 1 KiB of scores/probabilities per wave.
__device__ __forceinline__ void attention_dec_block(int bid, float (*__restrict__ ps)[4][64],
                                                    const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                                                    const uint16_t* __restrict__ vc, const int32_t* __restrict__ tiles,
                                                    int n_items, int Hq, int Hkv, int max_ctx, int n_slots, int T,
                                                    float scale_log2, uint16_t* __restrict__ out) {
  typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int item = bid * 4 + wv;
  if (item >= n_items) return;                 // whole wave; no block barrier below
  const int tile = item / Hkv;
  const int g = item % Hkv;
  const int row = tiles[tile * 4 + 0];
  const int s = tiles[tile * 4 + 2];
  const int ctx = tiles[tile * 4 + 3] + 1;
  if ((unsigned)s >= (unsigned)n_slots || ctx < 1 || ctx > max_ctx || (unsigned)row >= (unsigned)T) return;
  const int64_t kvbase = ((int64_t)s * Hkv + g) * max_ctx * 128;
  const int part = lane & 7, ksub = lane >> 3;         // score layout: 8 keys x 8 dim-parts of 16
  uint32_t qv[4][8];                                   // q of head h, dims [part*16, +16), bf16 pairs
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    const uint4* src = reinterpret_cast<const uint4*>(q + ((int64_t)row * Hq + g * 4 + h) * 128 + part * 16);
    const uint4 a = src[0], b = src[1];
    qv[h][0] = a.x; qv[h][1] = a.y; qv[h][2] = a.z; qv[h][3] = a.w;
    qv[h][4] = b.x; qv[h][5] = b.y; qv[h][6] = b.z; qv[h][7] = b.w;
  }
  float m[4], l[4], acc[4][4];
#pragma unroll
  for (int h = 0; h < 4; ++h) {
    m[h] = -3.0e38f;
    l[h] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[h][i] = 0.f;
  }
  const int kh = lane >> 5, dp = lane & 31;            // P.V layout: key parity x 4-dim slices
  for (int k0 = 0; k0 < ctx; k0 += 64) {
    const int nk = min(64, ctx - k0);
    // ---- scores of keys k0 .. k0+nk-1 (pre-scaled by scale*log2e) -> ps.
    // The K rows of 32 keys (4 passes) are loaded before any is used: one
    // memory round trip per 32 keys instead of one per 8
    for (int kb0 = 0; kb0 < nk; kb0 += 32) {
      uint4 ka[4], kb[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int key = kb0 + u * 8 + ksub;
        if (key < nk) {
          const uint4* kr = reinterpret_cast<const uint4*>(kc + kvbase + (int64_t)(k0 + key) * 128 + part * 16);
          ka[u] = kr[0];
          kb[u] = kr[1];
        } else {
          ka[u] = make_uint4(0u, 0u, 0u, 0u);
          kb[u] = ka[u];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (kb0 + u * 8 >= nk) break;                // wave-uniform
        const int key = kb0 + u * 8 + ksub;
        float d[4] = {0.f, 0.f, 0.f, 0.f};
        if (key < nk) {
          const uint32_t kw[8] = {ka[u].x, ka[u].y, ka[u].z, ka[u].w, kb[u].x, kb[u].y, kb[u].z, kb[u].w};
#pragma unroll
          for (int h = 0; h < 4; ++h)
#pragma unroll
            for (int i = 0; i < 8; ++i)
              d[h] = __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, qv[h][i]),
                                                     __builtin_bit_cast(bf16x2_t, kw[i]), d[h], false);
        }
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          d[h] += __shfl_xor(d[h], 1, 64);
          d[h] += __shfl_xor(d[h], 2, 64);
          d[h] += __shfl_xor(d[h], 4, 64);
        }
        if (part == 0 && key < nk) {
#pragma unroll
          for (int h = 0; h < 4; ++h) ps[wv][h][key] = d[h] * scale_log2;
        }
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    // ---- online softmax over the block, lane = key
    const bool live = lane < nk;
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const float v = live ? ps[wv][h][lane] : -3.0e38f;
      const float mn = fmaxf(m[h], wave_max(v));
      const float p = live ? exp2f(v - mn) : 0.f;
      const float corr = exp2f(m[h] - mn);
      l[h] = l[h] * corr + wave_sum(p);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[h][i] *= corr;
      m[h] = mn;
      ps[wv][h][lane] = p;
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_wave_barrier();
    // ---- O += P V (half-wave kh takes keys of parity kh); the V rows of 16
    // keys are loaded before the first is used (same key order per lane)
    const uint16_t* vr = vc + kvbase + (int64_t)k0 * 128 + dp * 4;
    for (int j0 = 0; j0 < nk; j0 += 16) {
      uint2 vv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + kh + 2 * u;
        vv[u] = j < nk ? *reinterpret_cast<const uint2*>(vr + (int64_t)j * 128) : make_uint2(0u, 0u);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int j = j0 + kh + 2 * u;
        if (j >= nk) break;
        const uint2 v2 = vv[u];
        const float v0 = bf((uint16_t)(v2.x & 0xFFFFu)), v1 = bf((uint16_t)(v2.x >> 16));
        const float v2f = bf((uint16_t)(v2.y & 0xFFFFu)), v3 = bf((uint16_t)(v2.y >> 16));
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          const float p = ps[wv][h][j];
          acc[h][0] += p * v0;
          acc[h][1] += p * v1;
          acc[h][2] += p * v2f;
          acc[h][3] += p * v3;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();          // ps is rewritten by the next block
  }
#pragma unroll
  for (int h = 0; h < 4; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[h][i] += __shfl_xor(acc[h][i], 32, 64);
  if (kh == 0) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const float inv = 1.0f / l[h];
      uint2 o;
      o.x = (uint32_t)f32_to_bf16_rne(acc[h][0] * inv) | ((uint32_t)f32_to_bf16_rne(acc[h][1] * inv) << 16);
      o.y = (uint32_t)f32_to_bf16_rne(acc[h][2] * inv) | ((uint32_t)f32_to_bf16_rne(acc[h][3] * inv) << 16);
      *reinterpret_cast<uint2*>(out + ((int64_t)row * Hq + g * 4 + h) * 128 + dp * 4) = o;
    }
  }
}

__global__ void __launch_bounds__(256)
attention_dec_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                     const uint16_t* __restrict__ vc, const int32_t* __restrict__ tiles, int n_items, int Hq,
                     int Hkv, int max_ctx, int n_slots, int T, float scale_log2, uint16_t* __restrict__ out) {
  __shared__ float ps[4][4][64];
  attention_dec_block(blockIdx.x, ps, q, kc, vc, tiles, n_items, Hq, Hkv, max_ctx, n_slots, T, scale_log2, out);
}

// Both kinds of tiles of a step in ONE launch: blocks [0, n_seg_blocks) run
// segment (prefill-chunk) tiles, the rest decode items.  Each kernel alone is
// latency-bound and leaves most of the chip idle for part of its run; in one
// grid the decode blocks fill the CUs behind the segment blocks instead of
// waiting for the segment kernel's last block (stream order).  The LDS array
// is the segment block's; a decode block uses its first 4 KiB.
template <int KEYS>
__global__ void __launch_bounds__(256, KEYS == 32 ? 4 : 3)
attention_mixed_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                       const uint16_t* __restrict__ vc, const int32_t* __restrict__ tiles, int n_dec_tiles,
                       int n_seg_blocks, int Hq, int Hkv, int max_ctx, int n_slots, int T, float scale_log2,
                       uint16_t* __restrict__ out) {
  static_assert(seg_lds_elems<KEYS>() * 2 >= 4 * 4 * 64 * 4, "decode scores must fit");
  __shared__ __align__(16) uint16_t smem[seg_lds_elems<KEYS>()];
  const int bid = blockIdx.x;
  if (bid < n_seg_blocks)
    attention_seg_block<KEYS>(bid, smem, q, kc, vc, tiles + 4 * n_dec_tiles, Hq, Hkv, max_ctx, n_slots, T,
                              scale_log2, out);
  else
    attention_dec_block(bid - n_seg_blocks, reinterpret_cast<float (*)[4][64]>(smem), q, kc, vc, tiles,
                        n_dec_tiles * Hkv, Hq, Hkv, max_ctx, n_slots, T, scale_log2, out);
}

// Byte copy between device memory and host-mapped pinned memory, run as a
// kernel on the caller's stream.  Used for the preprocess pipeline's
// host<->device traffic: the runtime's async H2D path was measured to queue
// behind the backend's in-flight forward on the other stream (a 60 ms stall
// per ingest batch); a kernel on the high-priority side stream is not.
__global__ void __launch_bounds__(256)
copy_bytes_kernel(uint8_t* __restrict__ dst, const uint8_t* __restrict__ src, int64_t n16, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride)
    reinterpret_cast<uint4*>(dst)[i] = reinterpret_cast<const uint4*>(src)[i];
  if (blockIdx.x == 0)
    for (int64_t i = n16 * 16 + threadIdx.x; i < n; i += 256) dst[i] = src[i];
  __threadfence_system();   // host-mapped destination: visible once the stream's event completes
}

// N9: device-side slot census -> host-mapped load page (zero-copy for the
// router).  page layout (uint32): [0]=seq, [1]=active slots, [2]=free slots,
// [3]=tokens this step, [4]=step id lo.  Stores are system-scope so a host
// reader polling the page sees them without a device synchronisation.
__global__ void __launch_bounds__(256)
slot_census_kernel(const int32_t* __restrict__ slot_state, int S, int tokens, uint32_t step,
                   uint32_t* page) {
  __shared__ int red[4];
  int n = 0;
  for (int i = threadIdx.x; i < S; i += 256) n += slot_state[i] != 0;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) n += __shfl_xor(n, off, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int act = red[0] + red[1] + red[2] + red[3];
    __hip_atomic_store(page + 1, (uint32_t)act, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(page + 2, (uint32_t)(S - act), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(page + 3, (uint32_t)tokens, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(page + 4, step, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_fetch_add(page + 0, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace llmq
