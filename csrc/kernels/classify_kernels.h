// embed_pool: hashed-token embedding gather -> bf16 MFMA GEMM -> GELU ->
// masked mean-pool per message (N4), plus the tiny classifier head.
//
// A NEW capability relative to the reference (which only has keyword regexes,
// `internal/preprocessor/preprocessor.go:117-168`): a random-init priority /
// sentiment / question classifier whose hot path is a gather + GEMM on the
// matrix cores.
//
// Shapes: token rows are the batch's tokens compacted message-major
// (row_off = exclusive scan of ntok), X[row] = E[hash & (V-1)] (D = 256 bf16),
// Hid = GELU(X . W1^T + b1) (H = 1024), pooled[msg] = mean over the message's
// rows.  W1 is stored transposed, W1t[H][D], so a B fragment is 16 contiguous
// bytes of one W1t row.
//
// Tiling (gfx950): one 256-thread workgroup (4 waves) per (64-row tile,
// 256-column chunk of H) -- H / 256 blocks per tile, so the few tiles of a
// serving micro-batch still spread over many CUs (the kernel is latency-bound
// there: 57 -> 18 us at 64 messages, profiles/r3_embed_pool_ab.md).
//   * the 64 x 256 bf16 A tile (32 KiB) is gathered ONCE into LDS with 16-byte
//     register-staged loads (for row gathers from a ~32 MiB table an LDS-DMA
//     global_load_lds with per-lane source rows reads at the same rate, per
//     the MI355X microarchitecture measurements, so the simpler form stays); its 16-byte chunks are XOR-swizzled (chunk ^ (row & 15)) so the
//     v_mfma_f32_16x16x32_bf16 A-fragment reads (16 rows x one chunk per lane
//     group) are bank-conflict free for every ds_read_b128 lane group;
//   * 64 columns per wave = 4x4 16x16 accumulators, K = 256 = 8 MFMA
//     k-steps; the 32 B fragments of all 8 k-steps are loaded from L2 at once
//     (W1t is 512 KiB, resident): one round trip per block, not one per k-step;
//   * epilogue in registers: bias + tanh-GELU on the C fragments, then per
//     message segment of the tile (starts found by one ballot) each lane sums
//     its rows, two xor-shuffles join the four row-quads of a column, and the
//     mean sum/ntok is written -- a plain store when the message lies wholly
//     inside the tile, an f32 atomic add otherwise (pooled is zeroed before
//     the launch).  No LDS slab: the 32 KiB A tile is the block's LDS.
// Grid: ceil(rows_upper / 64) tiles x H / 256 chunks; tiles past the
// device-side row total exit immediately (rows_upper is a host bound from
// byte lengths).

#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmq {

typedef __attribute__((ext_vector_type(8))) short bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int EP_TM = 64;      // rows per tile
constexpr int EP_D = 256;      // embedding dim (K)
constexpr int EP_NCHUNK = 256; // columns per sweep step
constexpr int EP_CHUNKS_PER_ROW = EP_D / 8;  // 16-byte chunks per A row
constexpr uint32_t EP_NO_ROW = 0xFFFFFFFFu;

__device__ __forceinline__ float bf16_to_f32(uint16_t b) {
  return __uint_as_float(((uint32_t)b) << 16);
}

__device__ __forceinline__ float gelu_tanh(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float y = k0 * (x + k1 * x * x * x);
  // tanh(y) = 1 - 2 / (exp(2y) + 1)
  const float t = 1.0f - 2.0f / (__expf(2.0f * y) + 1.0f);
  return 0.5f * x * (1.0f + t);
}

// Exclusive scan of ntok (stats[:, ST_NTOK], row stride `stride`) into
// row_off[0..B]; single workgroup of 1024 threads.
__global__ void __launch_bounds__(1024)
scan_rows_kernel(const int32_t* __restrict__ ntok, int stride, int B, int32_t* __restrict__ row_off) {
  __shared__ int32_t part[1024];
  __shared__ int32_t carry;
  const int t = threadIdx.x;
  if (t == 0) carry = 0;
  __syncthreads();
  for (int base = 0; base < B; base += 1024) {
    const int i = base + t;
    const int v = (i < B) ? ntok[(int64_t)i * stride] : 0;
    part[t] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      const int x = (t >= off) ? part[t - off] : 0;
      __syncthreads();
      part[t] += x;
      __syncthreads();
    }
    if (i < B) row_off[i] = carry + part[t] - v;
    __syncthreads();
    if (t == 1023) carry += part[1023];
    __syncthreads();
  }
  if (t == 0) row_off[B] = carry;
}

__global__ void __launch_bounds__(256)
embed_pool_kernel(const uint32_t* __restrict__ hashes, int L, const int32_t* __restrict__ row_off,
                  int B, const uint16_t* __restrict__ E, uint32_t vmask,
                  const uint16_t* __restrict__ W1t, const float* __restrict__ b1, int H,
                  float* __restrict__ pooled, const int32_t* __restrict__ ntok_src, int ntok_stride) {
  extern __shared__ __align__(16) uint8_t smem[];
  uint16_t* At = reinterpret_cast<uint16_t*>(smem);                       // 64 x 256 bf16 (32 KiB)
  int32_t* rmsg = reinterpret_cast<int32_t*>(smem + EP_TM * EP_D * 2);
  int32_t* rinfo = rmsg + EP_TM;  // [0]=rows in tile, [1]=segments, [2..]=segment starts (+ end)
  int32_t* seg = rinfo + 2;
  __shared__ uint32_t rbucket[EP_TM];   // row -> embedding bucket (EP_NO_ROW: past the tile's rows)

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wv = tid >> 6;
  // row_off: the global scan, or (ntok_src != nullptr) this block's own
  // exclusive scan of the B token counts in LDS -- every block redoes the
  // few-hundred-element scan instead of a separate single-block launch
  const int32_t* ro = row_off;
  // row offsets of messages mlo .. mlo + wn in LDS: the whole scan (in-block
  // path) or a 65-entry window from the tile's first message (global path)
  int32_t* win = rinfo + 2 * EP_TM;
  int mlo = 0, wn = B;
  if (ntok_src) {
    __shared__ int32_t wtot[4];
    int32_t* roff = rinfo + 2 * EP_TM;                                      // [B + 1] ints
    int carry = 0;
    for (int base = 0; base < B; base += 256) {
      const int i = base + tid;
      const int v = i < B ? ntok_src[(int64_t)i * ntok_stride] : 0;
      int x = v;
#pragma unroll
      for (int off = 1; off < 64; off <<= 1) {
        const int y = __shfl_up(x, off, 64);
        if (lane >= off) x += y;
      }
      if (lane == 63) wtot[wv] = x;
      __syncthreads();
      int wpre = 0;
      for (int k = 0; k < wv; ++k) wpre += wtot[k];
      if (i < B) roff[i] = carry + wpre + x - v;
      carry += wtot[0] + wtot[1] + wtot[2] + wtot[3];
      __syncthreads();                                                      // wtot reuse
    }
    if (tid == 0) roff[B] = carry;
    __syncthreads();
    ro = roff;
  }
  const int total = ro[B];
  // one block per (64-row tile, 256-column chunk of H): a small batch (a few
  // tiles) still spreads over H / 256 times as many CUs -- the kernel is
  // latency-bound there; each block gathers its tile's rows (L2-resident)
  const int nchunk = H / EP_NCHUNK;
  const int tile0 = (blockIdx.x / nchunk) * EP_TM;
  const int chunk0 = (blockIdx.x % nchunk) * EP_NCHUNK;
  if (tile0 >= total) return;  // uniform across the block
  const int rows = min(EP_TM, total - tile0);

  const int fr = lane & 15;   // fragment row / col within a 16x16 tile
  const int fq = lane >> 4;   // k-quarter (A/B), row-quad (C)
  const int wc0 = chunk0 + wv * 64;  // this wave's 64 output columns
  // all 8 k-steps' B fragments issued at once (128 VGPRs), before the row
  // search and the gather: their L2 round trip overlaps that dependent chain
  // (hash load -> embedding row load) instead of following it
  bf16x8 bfall[EP_D / 32][4];
#pragma unroll
  for (int ks = 0; ks < EP_D / 32; ++ks)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      bfall[ks][j] = *reinterpret_cast<const bf16x8*>(W1t + (int64_t)(wc0 + j * 16 + fr) * EP_D + ks * 32 + fq * 8);

  if (!ntok_src) {
    // global row_off (large batches): wave 0 finds the tile's first message
    // mlo (largest m with row_off[m] <= tile0) by a 64-ary search -- ceil(log64
    // B) dependent L2 round trips instead of log2 B per row -- and the block
    // keeps row_off[mlo .. mlo + 64] in LDS for the per-row searches and the
    // gather / pooling offsets
    __shared__ int s_mlo;
    if (wv == 0) {
      int lo = 0, hi = B - 1;                          // answer in [lo, hi]; row_off[lo] <= tile0
      while (lo < hi) {
        const int step = (hi - lo + 63) >> 6;          // 64 probes lo + step .. lo + 64 step
        const int c = lo + (lane + 1) * step;
        const bool ok = c <= hi && ro[c] <= tile0;     // a prefix of the lanes (row_off is sorted)
        lo += __popcll(__ballot(ok)) * step;
        hi = min(hi, lo + step - 1);
      }
      if (lane == 0) s_mlo = lo;
    }
    __syncthreads();
    mlo = s_mlo;
    wn = min(EP_TM, B - mlo);
    if (tid <= wn) win[tid] = ro[mlo + tid];           // mlo + wn <= B: row_off has B + 1 entries
    __syncthreads();
  }
  // row_off[m]: from the LDS window when m is inside it
  auto rofs = [&](int m) -> int {
    const int k = m - mlo;
    return (k >= 0 && k <= wn) ? win[k] : ro[m];
  };

  // ---- row -> (message, token) by binary search over row_off
  if (tid < EP_TM) {
    int m = -1;
    const int g = tile0 + tid;
    if (tid < rows) {
      if (mlo + wn == B || win[wn] > g) {              // inside the window
        int lo = 0, hi = wn - 1;
        while (lo < hi) {  // largest k with row_off[mlo + k] <= g
          const int mid = (lo + hi + 1) >> 1;
          if (win[mid] <= g) lo = mid; else hi = mid - 1;
        }
        m = mlo + lo;
      } else {                                         // past it (zero-token messages): global search
        int lo = mlo + wn, hi = B - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (ro[mid] <= g) lo = mid; else hi = mid - 1;
        }
        m = lo;
      }
    }
    rmsg[tid] = m;
  }
  if (tid == 0) rinfo[0] = rows;
  __syncthreads();
  // ---- message segments of the tile (rows are message-major): starts by ballot
  if (tid < EP_TM) {
    const bool start = tid < rows && (tid == 0 || rmsg[tid] != rmsg[tid - 1]);
    const uint64_t mask = __ballot(start);
    if (start) seg[__popcll(mask & ((1ull << tid) - 1ull))] = tid;
    if (tid == 0) {
      rinfo[1] = __popcll(mask);
      seg[__popcll(mask)] = rows;
    }
    // the row's embedding bucket: its ONE hash load, done once per row here
    // (the gather below used to reload it per 16-byte chunk, inside a loop
    // the compiler ran as 8 serial window -> hash -> row load chains: the
    // ~20 us floor at serving batch sizes, profiles/r5_preprocess_kernels_pmc.md)
    const int m = rmsg[tid];
    rbucket[tid] = m >= 0 ? (hashes[(int64_t)m * L + (tile0 + tid - rofs(m))] & vmask) : EP_NO_ROW;
  }
  __syncthreads();

  // ---- gather the A tile: 64 rows x 32 chunks of 16 B, swizzled chunk ^ (row & 15);
  // all 8 loads of a thread in flight (unconditional: a missing row reads row 0)
  {
    constexpr int PER = EP_TM * EP_CHUNKS_PER_ROW / 256;
    uint4 v[PER];
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + u * 256;
      const uint32_t bk = rbucket[c / EP_CHUNKS_PER_ROW];
      v[u] = *reinterpret_cast<const uint4*>(E + (int64_t)(bk == EP_NO_ROW ? 0u : bk) * EP_D +
                                             (c % EP_CHUNKS_PER_ROW) * 8);
    }
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const int c = tid + u * 256;
      const int r = c / EP_CHUNKS_PER_ROW, ch = c % EP_CHUNKS_PER_ROW;
      const uint4 x = rbucket[r] == EP_NO_ROW ? make_uint4(0u, 0u, 0u, 0u) : v[u];
      *reinterpret_cast<uint4*>(At + r * EP_D + ((ch ^ (r & 15)) * 8)) = x;
    }
  }
  __syncthreads();

  {
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

#pragma unroll
    for (int ks = 0; ks < EP_D / 32; ++ks) {
      const bf16x8* bfrag = bfall[ks];
      bf16x8 afrag[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = i * 16 + fr;
        const int ch = ks * 4 + fq;
        afrag[i] = *reinterpret_cast<const bf16x8*>(At + r * EP_D + ((ch ^ (r & 15)) * 8));
      }
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afrag[i], bfrag[j], acc[i][j], 0, 0, 0);
    }

    // ---- epilogue: bias + GELU in registers, then the segmented mean over
    // rows straight from the C fragments (lane: rows i*16 + 4fq + k, column
    // j*16 + fr): per message segment each lane sums its rows inside it, the
    // four row-quads of a column meet by two xor-shuffles, and lanes fq == 0
    // write -- no LDS slab (2 blocks per CU instead of 1)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float bias = b1[wc0 + j * 16 + fr];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) acc[i][j][k] = gelu_tanh(acc[i][j][k] + bias);
    }
    const int nseg = rinfo[1];
    for (int sg = 0; sg < nseg; ++sg) {                 // uniform: every lane runs the shuffles
      const int r0 = seg[sg], r1 = seg[sg + 1];
      const int cur = rmsg[r0];
      float sum[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int r = i * 16 + fq * 4 + k;
          const bool in = r >= r0 && r < r1;
#pragma unroll
          for (int j = 0; j < 4; ++j) sum[j] += in ? acc[i][j][k] : 0.f;
        }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        sum[j] += __shfl_xor(sum[j], 16, 64);
        sum[j] += __shfl_xor(sum[j], 32, 64);
      }
      if (fq == 0) {
        const int a = rofs(cur), b = rofs(cur + 1);
        const float inv = 1.0f / (float)(b - a);
        const bool whole = a >= tile0 && b <= tile0 + rows;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float* dst = pooled + (int64_t)cur * H + wc0 + j * 16 + fr;
          if (whole) *dst = sum[j] * inv; else atomicAdd(dst, sum[j] * inv);
        }
      }
    }
  }
}

// Optional readback into host-mapped memory (int32 offsets into dst): stats
// rows at 0, predictions at o_pred, the first `cap` token hashes at o_ph.
struct ClassifyReadback {
  int32_t* dst;                 // nullptr: no readback
  const int32_t* stats;
  const uint32_t* hashes;
  int stat_cols, L, cap;
  int64_t o_pred, o_ph;
};

// logits[b, 0:8] = pooled[b] . W2 + b2 ; pred[b] = 1 + argmax(logits[b, 0:4])
// One wave per CH_MSGS messages; lane l covers hidden units l, l+64, ...: each
// W2 row (8 floats) is loaded once per wave and used for all its messages
// (W2 is 32 KiB: one read per message made the kernel L2-bound at large
// batches).  Per message the summation order is the one-message-per-wave
// order, so the results are unchanged.
// CH_MSGS = 1 below ~1k messages: a serving micro-batch has few waves, and
// the latency of one wave's chain, not L2 traffic, sets the time there
// (profiles/r3_embed_pool_ab.md: 64 messages 9.5 us at 1 vs 14.4 us at 4).
constexpr int CH_UNROLL = 4;   // hidden units per lane per load round (H % (64 * CH_UNROLL) == 0)

template <int CH_MSGS>
__global__ void __launch_bounds__(256)
classify_head_kernel(const float* __restrict__ pooled, int B, int H, const float* __restrict__ W2,
                     const float* __restrict__ b2, float* __restrict__ logits, int32_t* __restrict__ pred,
                     const ClassifyReadback rb) {
  const int lane = threadIdx.x & 63;
  const int b0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * CH_MSGS;
  if (b0 >= B) return;                                  // whole wave
  const int nm = min(CH_MSGS, B - b0);
  if (rb.dst) {         // the batch's readback rides along: stats rows + prompt hashes of these messages
    for (int m = 0; m < nm; ++m) {
      const int b = b0 + m;
      if (lane < rb.stat_cols) rb.dst[(int64_t)b * rb.stat_cols + lane] = rb.stats[(int64_t)b * rb.stat_cols + lane];
      for (int c = lane; c < rb.cap; c += 64)
        rb.dst[rb.o_ph + (int64_t)b * rb.cap + c] = (int32_t)rb.hashes[(int64_t)b * rb.L + c];
    }
  }
  float part[CH_MSGS][8];
#pragma unroll
  for (int m = 0; m < CH_MSGS; ++m)
#pragma unroll
    for (int o = 0; o < 8; ++o) part[m][o] = 0.f;
  // CH_UNROLL hidden units per lane per round, every load of the round in
  // flight together and unconditional (rows past nm re-read row nm - 1; their
  // partials are never written): the round-4 loop waited on each round's
  // loads, 16 dependent round trips per wave at H = 1024
  // (profiles/r5_preprocess_kernels_pmc.md).  Per message the summation
  // order over h is unchanged.
  for (int h0 = lane; h0 < H; h0 += 64 * CH_UNROLL) {
    float4 wa[CH_UNROLL], wb[CH_UNROLL];
    float x[CH_UNROLL][CH_MSGS];
#pragma unroll
    for (int u = 0; u < CH_UNROLL; ++u) {
      const int h = h0 + u * 64;
      wa[u] = *reinterpret_cast<const float4*>(W2 + (int64_t)h * 8);
      wb[u] = *reinterpret_cast<const float4*>(W2 + (int64_t)h * 8 + 4);
#pragma unroll
      for (int m = 0; m < CH_MSGS; ++m) x[u][m] = pooled[(int64_t)(b0 + min(m, nm - 1)) * H + h];
    }
#pragma unroll
    for (int u = 0; u < CH_UNROLL; ++u)
#pragma unroll
      for (int m = 0; m < CH_MSGS; ++m) {
        const float xv = x[u][m];
        part[m][0] += xv * wa[u].x; part[m][1] += xv * wa[u].y; part[m][2] += xv * wa[u].z;
        part[m][3] += xv * wa[u].w; part[m][4] += xv * wb[u].x; part[m][5] += xv * wb[u].y;
        part[m][6] += xv * wb[u].z; part[m][7] += xv * wb[u].w;
      }
  }
#pragma unroll
  for (int m = 0; m < CH_MSGS; ++m)
#pragma unroll
    for (int o = 0; o < 8; ++o) {
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) part[m][o] += __shfl_xor(part[m][o], off, 64);
    }
  if (lane < nm) {                                      // lane m writes message b0 + m
#pragma unroll
    for (int m = 0; m < CH_MSGS; ++m) {
      if (m != lane) continue;
      const int b = b0 + m;
      int best = 0;
      float bv = -3.4e38f;
#pragma unroll
      for (int o = 0; o < 8; ++o) {
        const float v = part[m][o] + b2[o];
        logits[(int64_t)b * 8 + o] = v;
        if (o < 4 && v > bv) { bv = v; best = o; }
      }
      pred[b] = best + 1;
      if (rb.dst) rb.dst[rb.o_pred + b] = best + 1;
    }
  }
  if (rb.dst) __threadfence_system();   // host-mapped: visible once the stream's event completes
}

}  // namespace llmq
