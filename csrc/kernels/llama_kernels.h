// Decode-path kernels of the Llama-3-8B-shaped backend stub (N12): fused
// residual-add + RMSNorm, SiLU*up, RoPE + paged KV write, and a unified
// prefill/decode GQA attention over the slot KV cache.  The GEMMs stay on
// hipBLASLt through torch.matmul.
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
// new residual stream) and the norm is taken of that sum.  D % 2048 == 0
// (one 256-thread block per row, 8 bf16 per thread per pass).
__global__ void __launch_bounds__(256)
rmsnorm_kernel(const uint16_t* __restrict__ x, uint16_t* __restrict__ res, const uint16_t* __restrict__ w,
               uint16_t* __restrict__ y, int D, float eps) {
  const int row = blockIdx.x;
  const int tid = threadIdx.x;
  const int npass = D / 2048;
  float v[4][8];
  float ss = 0.f;
  for (int p = 0; p < npass && p < 4; ++p) {
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
  for (int p = 0; p < npass && p < 4; ++p) {
    const int col = p * 2048 + tid * 8;
    const u16x8 wv = *reinterpret_cast<const u16x8*>(w + col);
    u16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = f32_to_bf16_rne(v[p][k] * inv * bf(wv[k]));
    *reinterpret_cast<u16x8*>(y + (int64_t)row * D + col) = o;
  }
}

// out[t, i] = silu(gu[t, i]) * gu[t, F + i], 8 elements per thread.
__global__ void __launch_bounds__(256)
silu_mul_kernel(const uint16_t* __restrict__ gu, uint16_t* __restrict__ out, int T, int F) {
  const int64_t idx = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 8;
  const int64_t total = (int64_t)T * F;
  if (idx >= total) return;
  const int64_t t = idx / F;
  const int64_t i = idx % F;
  const u16x8 g = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + i);
  const u16x8 u = *reinterpret_cast<const u16x8*>(gu + t * 2 * F + F + i);
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
// thread i handles rotary pair i (0..63) of heads tid/64, tid/64+4, ...
__global__ void __launch_bounds__(256)
rope_kv_kernel(const uint16_t* __restrict__ qkv, const int32_t* __restrict__ pos,
               const int32_t* __restrict__ slot, const float* __restrict__ cos_t,
               const float* __restrict__ sin_t, int Hq, int Hkv, int max_ctx,
               uint16_t* __restrict__ q_out, uint16_t* __restrict__ kc, uint16_t* __restrict__ vc) {
  const int t = blockIdx.x;
  const int tid = threadIdx.x;
  const int i = tid & 63;            // rotary pair index (dims i and i + 64)
  const int hg = tid >> 6;           // 4 head groups
  const int p = pos[t];
  const int s = slot[t];
  const float c = cos_t[(int64_t)p * 64 + i];
  const float sn = sin_t[(int64_t)p * 64 + i];
  const int64_t row = (int64_t)t * (Hq + 2 * Hkv) * 128;
  for (int h = hg; h < Hq; h += 4) {
    const float x0 = bf(qkv[row + h * 128 + i]);
    const float x1 = bf(qkv[row + h * 128 + i + 64]);
    q_out[(int64_t)t * Hq * 128 + h * 128 + i] = f32_to_bf16_rne(x0 * c - x1 * sn);
    q_out[(int64_t)t * Hq * 128 + h * 128 + i + 64] = f32_to_bf16_rne(x1 * c + x0 * sn);
  }
  for (int h = hg; h < Hkv; h += 4) {
    const int64_t kb = row + (int64_t)(Hq + h) * 128;
    const int64_t vb = row + (int64_t)(Hq + Hkv + h) * 128;
    const float x0 = bf(qkv[kb + i]);
    const float x1 = bf(qkv[kb + i + 64]);
    const int64_t dst = (((int64_t)s * Hkv + h) * max_ctx + p) * 128;
    kc[dst + i] = f32_to_bf16_rne(x0 * c - x1 * sn);
    kc[dst + i + 64] = f32_to_bf16_rne(x1 * c + x0 * sn);
    vc[dst + i] = qkv[vb + i];
    vc[dst + i + 64] = qkv[vb + i + 64];
  }
}

constexpr int AT_KEYS = 64;
constexpr int AT_ROW = 136;  // 128 bf16 + 8 pad (272 B rows)

__global__ void __launch_bounds__(256)
attention_kernel(const uint16_t* __restrict__ q, const uint16_t* __restrict__ kc,
                 const uint16_t* __restrict__ vc, const int32_t* __restrict__ pos,
                 const int32_t* __restrict__ slot, int Hq, int Hkv, int max_ctx, float scale,
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
