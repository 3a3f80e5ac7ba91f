// context_summarise (N5): summarise-on-evict for conversation windows.
//
// Reference behaviour being replaced: drop-oldest truncation beyond
// MaxContextLength (`internal/conversation/state_manager.go:131-134`) and
// plain string concatenation of completed contents
// (`internal/statemanager/manager.go:133-135`).  Here evicted messages are
// folded into a fixed-size per-conversation summary state:
//
//   mean_c = mean over the conversation's evicted messages of pooled[m]   (H)
//   proj_c = mean_c . P                     (bf16 MFMA, H=1024 -> DS=256)
//   s_c    = alpha * s_c + (1 - alpha) * proj_c          (EMA, f32, in place)
//
// plus a salient-token list: the top-k token hashes of the evicted messages
// by frequency (stop words excluded), ties broken by first occurrence.
//
// summarise_project_kernel: one workgroup = 16 conversations x 256 outputs;
// the 16 mean rows are built in LDS as bf16 (32 KiB, chunk-swizzled like
// embed_pool's A tile) and each wave computes 64 output columns with
// v_mfma_f32_16x16x32_bf16 over K = 1024 (32 k-steps); P is stored
// transposed (Pt[DS][H]) so B fragments are 16 contiguous bytes.

#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "classify_kernels.h"

namespace llmq {

constexpr int SM_ROWS = 16;
constexpr int SM_H = 1024;
constexpr int SM_DS = 256;

__device__ __forceinline__ uint16_t f32_to_bf16_rne(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7F800000u) == 0x7F800000u) return (uint16_t)((u >> 16) | ((u & 0xFFFFu) ? 0x40u : 0u));
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

__global__ void __launch_bounds__(256)
summarise_project_kernel(const float* __restrict__ pooled, const int32_t* __restrict__ seg_off, int C,
                         const uint16_t* __restrict__ Pt, float alpha, float* __restrict__ state,
                         int32_t* __restrict__ first_flag) {
  __shared__ __align__(16) uint16_t Am[SM_ROWS * SM_H];  // 32 KiB
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int c0 = blockIdx.x * SM_ROWS;

  // ---- segment means -> bf16 rows (chunk ^ (row & 15) swizzle, 8 bf16 per chunk)
  for (int idx = tid; idx < SM_ROWS * (SM_H / 8); idx += 256) {
    const int r = idx / (SM_H / 8);
    const int ch = idx % (SM_H / 8);
    const int c = c0 + r;
    float v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (c < C) {
      const int a = seg_off[c], b = seg_off[c + 1];
      for (int m = a; m < b; ++m) {
        const float4 x0 = *reinterpret_cast<const float4*>(pooled + (int64_t)m * SM_H + ch * 8);
        const float4 x1 = *reinterpret_cast<const float4*>(pooled + (int64_t)m * SM_H + ch * 8 + 4);
        v[0] += x0.x; v[1] += x0.y; v[2] += x0.z; v[3] += x0.w;
        v[4] += x1.x; v[5] += x1.y; v[6] += x1.z; v[7] += x1.w;
      }
      const float inv = (b > a) ? 1.0f / (float)(b - a) : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] *= inv;
    }
    uint16_t* dst = Am + r * SM_H + ((ch ^ (r & 15)) * 8);
#pragma unroll
    for (int k = 0; k < 8; ++k) dst[k] = f32_to_bf16_rne(v[k]);
  }
  __syncthreads();

  const int fr = lane & 15, fq = lane >> 4;
  f32x4 acc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int ks = 0; ks < SM_H / 32; ++ks) {
    const int ch = ks * 4 + fq;
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(Am + fr * SM_H + ((ch ^ fr) * 8));
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wv * 64 + j * 16 + fr;
      const bf16x8 b = *reinterpret_cast<const bf16x8*>(Pt + (int64_t)col * SM_H + ks * 32 + fq * 8);
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc[j], 0, 0, 0);
    }
  }
  // ---- EMA update: C map row = 4*fq + k, col = fr
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = wv * 64 + j * 16 + fr;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + fq * 4 + k;
      if (c < C) {
        float* s = state + (int64_t)c * SM_DS + col;
        // a conversation's first summary takes the projection as-is
        *s = first_flag[c] ? acc[j][k] : alpha * (*s) + (1.0f - alpha) * acc[j][k];
      }
    }
  }
}

// Top-k salient token hashes per conversation (one workgroup each).
// tokens of message m: hashes[m*L .. m*L + ntok[m*stride]).
constexpr int SAL_TABLE = 2048;
__global__ void __launch_bounds__(256)
salient_topk_kernel(const uint32_t* __restrict__ hashes, int L, const int32_t* __restrict__ ntok,
                    int stride, const int32_t* __restrict__ seg_off, const uint32_t* __restrict__ stop,
                    int nstop, int K, uint32_t* __restrict__ out_hash, int32_t* __restrict__ out_cnt,
                    int32_t* __restrict__ out_overflow) {
  __shared__ uint32_t key[SAL_TABLE];
  __shared__ int overflow;  // a token found no table slot (> SAL_TABLE distinct): result is partial
  __shared__ int32_t cnt[SAL_TABLE];
  __shared__ int32_t first[SAL_TABLE];
  __shared__ uint64_t best_s[4];
  __shared__ int32_t best_i[4];
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  for (int i = tid; i < SAL_TABLE; i += 256) { key[i] = 0u; cnt[i] = 0; first[i] = 0x7FFFFFFF; }
  if (tid == 0) overflow = 0;
  __syncthreads();
  const int a = seg_off[c], b = seg_off[c + 1];
  int ord = 0;  // running token order across the conversation's messages
  for (int m = a; m < b; ++m) {
    const int n = ntok[(int64_t)m * stride];
    for (int t = tid; t < n; t += 256) {
      uint32_t h = hashes[(int64_t)m * L + t];
      bool is_stop = false;
      for (int s = 0; s < nstop; ++s) is_stop |= (stop[s] == h);
      if (is_stop) continue;
      if (h == 0u) h = 1u;  // 0 marks an empty slot
      uint32_t slot = (h * 2654435761u) & (SAL_TABLE - 1);
      bool placed = false;
      for (int probe = 0; probe < SAL_TABLE; ++probe) {
        const uint32_t prev = atomicCAS(&key[slot], 0u, h);
        if (prev == 0u || prev == h) {
          atomicAdd(&cnt[slot], 1);
          atomicMin(&first[slot], ord + t);
          placed = true;
          break;
        }
        slot = (slot + 1) & (SAL_TABLE - 1);
      }
      if (!placed) overflow = 1;  // benign race: every writer stores 1
    }
    ord += n;
  }
  __syncthreads();
  // K rounds of block argmax over (count desc, first asc)
  for (int k = 0; k < K; ++k) {
    uint64_t bs = 0ull;
    int bi = -1;
    for (int i = tid; i < SAL_TABLE; i += 256) {
      if (cnt[i] > 0) {
        const uint64_t s = ((uint64_t)(uint32_t)cnt[i] << 32) | (uint32_t)(0x7FFFFFFF - first[i]);
        if (s > bs) { bs = s; bi = i; }
      }
    }
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t os = __shfl_xor(bs, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      if (os > bs) { bs = os; bi = oi; }
    }
    if ((tid & 63) == 0) { best_s[tid >> 6] = bs; best_i[tid >> 6] = bi; }
    __syncthreads();
    if (tid == 0) {
      uint64_t s = best_s[0];
      int i = best_i[0];
      for (int w = 1; w < 4; ++w)
        if (best_s[w] > s) { s = best_s[w]; i = best_i[w]; }
      if (i >= 0 && s > 0ull) {
        out_hash[(int64_t)c * K + k] = key[i];
        out_cnt[(int64_t)c * K + k] = cnt[i];
        cnt[i] = 0;
      } else {
        out_hash[(int64_t)c * K + k] = 0u;
        out_cnt[(int64_t)c * K + k] = 0;
      }
    }
    __syncthreads();
  }
  // the host recomputes a flagged conversation exactly (never a silently
  // truncated top-k)
  if (tid == 0) out_overflow[c] = overflow;
}

}  // namespace llmq
