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
// summarise_project_kernel (round 5; profiles/r5_preprocess_kernels_pmc.md):
// one workgroup = 16 conversations x 64 output columns (grid.y = DS / 64),
// its 4 waves split K = 1024 into quarters.  The round-4 form (one block per
// 16 conversations, every lane a serial chain of 8 x n_msgs dependent loads,
// then 32 k-steps each waiting on its own B load, 2-byte LDS stores) took a
// flat 43 us at 16..256 conversations with 60 % LDS bank conflicts:
//   * all 32 B fragments of a wave's 8 k-steps x 4 column tiles are issued at
//     kernel entry (Pt is 512 KiB, L2-resident), overlapping the mean pass;
//   * the mean pass walks the 16 conversations' messages -- one contiguous
//     run of pooled rows -- as ONE flat loop, 16 messages per round with the
//     16 float4 loads in flight together; conversation boundaries are uniform
//     (every lane handles the same message), and a finished row's mean goes
//     to LDS as 4 packed bf16 (8-byte stores, chunk-swizzled), so the
//     summation order per element is the old one (m ascending) and the means
//     are bit-identical;
//   * v_mfma_f32_16x16x32_bf16 over the wave's 8 k-steps, then the four
//     K-quarter partials meet in LDS (stride-68 rows, conflict-free) and the
//     EMA update is a float4 per thread.
// P is stored transposed (Pt[DS][H]) so B fragments are 16 contiguous bytes.

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

constexpr int SM_NB = 64;                 // output columns per block
constexpr int SM_KQ = SM_H / 4;           // K per wave
constexpr int SM_RED = SM_NB + 4;         // reduction row stride (floats)
constexpr int SM_MEAN_UNROLL = 16;       // message rows in flight per lane in the mean pass

__global__ void __launch_bounds__(256)
summarise_project_kernel(const float* __restrict__ pooled, const int32_t* __restrict__ seg_off, int C,
                         const uint16_t* __restrict__ Pt, float alpha, float* __restrict__ state,
                         int32_t* __restrict__ first_flag) {
  __shared__ __align__(16) uint16_t Am[4][SM_ROWS * SM_KQ];       // per wave: 16 rows x its K quarter (8 KiB)
  __shared__ __align__(16) float red[4][SM_ROWS * SM_RED];        // K-quarter partials (17 KiB)
  __shared__ int32_t bnd[SM_ROWS + 1];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  const int c0 = blockIdx.x * SM_ROWS;
  const int n0 = blockIdx.y * SM_NB;
  const int kq = wv * SM_KQ;
  const int fr = lane & 15, fq = lane >> 4;

  // B fragments of all 8 k-steps x 4 column tiles, in flight during the means
  bf16x8 bfr[SM_KQ / 32][4];
#pragma unroll
  for (int ks = 0; ks < SM_KQ / 32; ++ks)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfr[ks][j] = *reinterpret_cast<const bf16x8*>(Pt + (int64_t)(n0 + j * 16 + fr) * SM_H + kq + ks * 32 + fq * 8);

  if (tid <= SM_ROWS) bnd[tid] = seg_off[min(c0 + tid, C)];
  __syncthreads();

  // ---- segment means of this wave's K quarter: lane = 4 columns
  uint16_t* A = Am[wv];
  const int col4 = lane * 4;
  int r = 0;                                         // current row (uniform)
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  auto flush = [&](int row) {                        // mean of row -> bf16 into the swizzled tile
    const int n = bnd[row + 1] - bnd[row];
    const float inv = n > 0 ? 1.0f / (float)n : 0.f;
    const uint32_t lo = (uint32_t)f32_to_bf16_rne(acc.x * inv) | ((uint32_t)f32_to_bf16_rne(acc.y * inv) << 16);
    const uint32_t hi = (uint32_t)f32_to_bf16_rne(acc.z * inv) | ((uint32_t)f32_to_bf16_rne(acc.w * inv) << 16);
    const int ch = (col4 >> 3) ^ (row & 15);         // 16-byte chunk, swizzled
    *reinterpret_cast<uint2*>(A + row * SM_KQ + ch * 8 + (col4 & 7)) = make_uint2(lo, hi);
    acc = make_float4(0.f, 0.f, 0.f, 0.f);
  };
  const int M0 = bnd[0], M1 = bnd[SM_ROWS];
  for (int m = M0; m < M1; m += SM_MEAN_UNROLL) {
    float4 x[SM_MEAN_UNROLL];
    // unconditional loads (rows past M1 re-read row M1 - 1 and are not
    // used): a predicated form compiled to a load -> vmcnt(0) chain
#pragma unroll
    for (int u = 0; u < SM_MEAN_UNROLL; ++u)
      x[u] = *reinterpret_cast<const float4*>(pooled + (int64_t)min(m + u, M1 - 1) * SM_H + kq + col4);
#pragma unroll
    for (int u = 0; u < SM_MEAN_UNROLL; ++u) {
      if (m + u >= M1) break;                        // uniform
      while (m + u >= bnd[r + 1]) flush(r++);        // uniform: rows ending before message m + u
      acc.x += x[u].x; acc.y += x[u].y; acc.z += x[u].z; acc.w += x[u].w;
    }
  }
  while (r < SM_ROWS) flush(r++);                    // the last row, empty rows, rows past C
  __builtin_amdgcn_s_waitcnt(0xC07F);                // lgkmcnt(0): the tile is written
  __builtin_amdgcn_wave_barrier();

  // ---- this wave's K quarter: 8 k-steps x 4 column tiles
  f32x4 pacc[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) pacc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < SM_KQ / 32; ++ks) {
    const int ch = ks * 4 + fq;
    const bf16x8 a = *reinterpret_cast<const bf16x8*>(A + fr * SM_KQ + ((ch ^ fr) * 8));
#pragma unroll
    for (int j = 0; j < 4; ++j) pacc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, bfr[ks][j], pacc[j], 0, 0, 0);
  }
  // C map: row 4 fq + k, column j * 16 + fr
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k) red[wv][(fq * 4 + k) * SM_RED + j * 16 + fr] = pacc[j][k];
  __syncthreads();

  // ---- K-quarter sum + EMA: thread = 4 columns of one row
  const int row = tid >> 4, cc = (tid & 15) * 4;
  const int c = c0 + row;
  if (c < C) {
    float4 p = *reinterpret_cast<const float4*>(&red[0][row * SM_RED + cc]);
#pragma unroll
    for (int w = 1; w < 4; ++w) {
      const float4 q = *reinterpret_cast<const float4*>(&red[w][row * SM_RED + cc]);
      p.x += q.x; p.y += q.y; p.z += q.z; p.w += q.w;
    }
    float4* sp = reinterpret_cast<float4*>(state + (int64_t)c * SM_DS + n0 + cc);
    if (first_flag[c]) {                             // a conversation's first summary takes the projection
      *sp = p;
    } else {
      const float4 o = *sp;
      const float b = 1.0f - alpha;
      *sp = make_float4(alpha * o.x + b * p.x, alpha * o.y + b * p.y, alpha * o.z + b * p.z, alpha * o.w + b * p.w);
    }
  }
}

// One round of a wave argmax over the lanes' NV scores each: returns the
// winner's score ws (0: nothing left) and index_of(its slot) in wi; the
// owner lane retires it.  Scores are unique, so exactly one lane owns it.
template <int NV, typename F>
__device__ __forceinline__ void sal_wave_pick(uint64_t (&v)[NV], F index_of, int lane, uint64_t& ws, int& wi) {
  uint64_t bs = 0ull;
  int be = -1;
#pragma unroll
  for (int e = 0; e < NV; ++e)
    if (v[e] > bs) { bs = v[e]; be = e; }
  uint64_t gs = bs;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const uint64_t o = __shfl_xor(gs, off, 64);
    if (o > gs) gs = o;
  }
  ws = gs;
  wi = -1;
  if (gs == 0ull) return;                              // uniform
  const uint64_t mine = __ballot(be >= 0 && bs == gs);
  const int owner = (int)__builtin_ctzll(mine);
  const int idx = be >= 0 ? index_of(be) : -1;
  wi = __shfl(idx, owner, 64);
  if (lane == owner) {
#pragma unroll
    for (int e = 0; e < NV; ++e)
      if (e == be) v[e] = 0ull;
  }
}

// Top-k salient token hashes per conversation (one workgroup each).
// tokens of message m: hashes[m*L .. m*L + ntok[m*stride]).
constexpr int SAL_TABLE = 2048;
constexpr int SAL_MAX_STOP = 128;
__global__ void __launch_bounds__(256)
salient_topk_kernel(const uint32_t* __restrict__ hashes, int L, const int32_t* __restrict__ ntok,
                    int stride, const int32_t* __restrict__ seg_off, const uint32_t* __restrict__ stop,
                    int nstop, int K, uint32_t* __restrict__ out_hash, int32_t* __restrict__ out_cnt,
                    int32_t* __restrict__ out_overflow) {
  __shared__ uint32_t key[SAL_TABLE];
  __shared__ int overflow;  // a token found no table slot (> SAL_TABLE distinct): result is partial
  __shared__ int32_t cnt[SAL_TABLE];
  __shared__ int32_t first[SAL_TABLE];
  const int tid = threadIdx.x;
  const int c = blockIdx.x;
  for (int i = tid; i < SAL_TABLE; i += 256) { key[i] = 0u; cnt[i] = 0; first[i] = 0x7FFFFFFF; }
  if (tid == 0) overflow = 0;
  __syncthreads();
  const int a = seg_off[c], b = seg_off[c + 1];
  // stop-word hashes in LDS (the list is ~30 words; a longer one stays global)
  __shared__ uint32_t sstop[SAL_MAX_STOP];
  const bool stop_lds = nstop <= SAL_MAX_STOP;
  if (stop_lds && tid < nstop) sstop[tid] = stop[tid];
  const uint32_t* stp = stop_lds ? sstop : stop;
  auto insert = [&](uint32_t h, int ord) {
    bool is_stop = false;
    for (int s = 0; s < nstop; ++s) is_stop |= (stp[s] == h);
    if (is_stop) return;
    if (h == 0u) h = 1u;  // 0 marks an empty slot
    uint32_t slot = (h * 2654435761u) & (SAL_TABLE - 1);
    for (int probe = 0; probe < SAL_TABLE; ++probe) {
      const uint32_t prev = atomicCAS(&key[slot], 0u, h);
      if (prev == 0u || prev == h) {
        atomicAdd(&cnt[slot], 1);
        atomicMin(&first[slot], ord);
        return;
      }
      slot = (slot + 1) & (SAL_TABLE - 1);
    }
    overflow = 1;  // no table slot left: benign race, every writer stores 1
  };
  const int nm = b - a;
  if (nm <= 256) {
    // every token of the conversation at once: an exclusive scan of the
    // messages' token counts, then thread j takes flat tokens j, j + 256, ...
    // (its message by binary search; the flat index IS the token's order).
    // Round 4 walked the messages one after another -- a dependent
    // ntok -> hash -> insert chain per message, a flat ~26 us.
    __shared__ int32_t moff[257];
    __shared__ int32_t wsum[4];
    const int lane = tid & 63, wv = tid >> 6;
    const int v = tid < nm ? ntok[(int64_t)(a + tid) * stride] : 0;
    int x = v;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int y = __shfl_up(x, off, 64);
      if (lane >= off) x += y;
    }
    if (lane == 63) wsum[wv] = x;
    __syncthreads();  // (also publishes sstop)
    int pre = 0;
    for (int k = 0; k < wv; ++k) pre += wsum[k];
    moff[tid] = pre + x - v;
    if (tid == 255) moff[256] = pre + x;
    __syncthreads();
    const int total = moff[256];
    for (int j = tid; j < total; j += 256) {
      int lo = 0, hi = nm - 1;  // largest k with moff[k] <= j
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (moff[mid] <= j) lo = mid; else hi = mid - 1;
      }
      insert(hashes[(int64_t)(a + lo) * L + (j - moff[lo])], j);
    }
  } else {
    __syncthreads();  // sstop
    int ord = 0;  // running token order across the conversation's messages
    for (int m = a; m < b; ++m) {
      const int n = ntok[(int64_t)m * stride];
      for (int t = tid; t < n; t += 256) insert(hashes[(int64_t)m * L + t], ord + t);
      ord += n;
    }
  }
  __syncthreads();
  // ---- selection by (count desc, first occurrence asc); scores are unique
  // (distinct tokens have distinct first positions).  Round 4 ran K rounds of
  // a block-wide argmax, two barriers each (a flat ~26 us); here each wave
  // takes the top K of its 512 table entries from registers with shuffles
  // alone, then wave 0 merges the 4 K candidates the same way: 2 barriers.
  __shared__ uint64_t cand_s[4][64];
  __shared__ int32_t cand_i[4][64];
  const int lane = tid & 63, wv = tid >> 6;
  constexpr int PER = SAL_TABLE / 256;               // entries per lane
  uint64_t sc[PER];
#pragma unroll
  for (int e = 0; e < PER; ++e) {
    const int i = wv * (SAL_TABLE / 4) + e * 64 + lane;
    sc[e] = cnt[i] > 0 ? (((uint64_t)(uint32_t)cnt[i] << 32) | (uint32_t)(0x7FFFFFFF - first[i])) : 0ull;
  }
  for (int k = 0; k < K; ++k) {
    uint64_t ws;
    int wi;
    sal_wave_pick(sc, [&](int e) { return wv * (SAL_TABLE / 4) + e * 64 + lane; }, lane, ws, wi);
    if (lane == 0) { cand_s[wv][k] = ws; cand_i[wv][k] = wi; }
    if (ws == 0ull) {
      for (int kk = k + 1 + lane; kk < K; kk += 64) { cand_s[wv][kk] = 0ull; cand_i[wv][kk] = -1; }
      break;
    }
  }
  __syncthreads();
  if (wv == 0) {
    uint64_t cs[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) cs[q] = lane < K ? cand_s[q][lane] : 0ull;   // candidate (wave q, rank lane)
    for (int k = 0; k < K; ++k) {
      uint64_t ws;
      int wi;
      sal_wave_pick(cs, [&](int q) { return cand_i[q][lane]; }, lane, ws, wi);
      if (lane == 0) {
        if (ws != 0ull && wi >= 0) {
          out_hash[(int64_t)c * K + k] = key[wi];
          out_cnt[(int64_t)c * K + k] = (int32_t)(ws >> 32);
        } else {
          out_hash[(int64_t)c * K + k] = 0u;
          out_cnt[(int64_t)c * K + k] = 0;
        }
      }
    }
  }
  // the host recomputes a flagged conversation exactly (never a silently
  // truncated top-k)
  if (tid == 0) out_overflow[c] = overflow;
}

}  // namespace llmq
