// Skinny GEMMs for small steps (M <= 64 rows, up to 256 in 64-row chunks): C = A[M][K] . W[N][K]^T with
// the realtime micro-forwards' epilogues (store, residual add, SwiGLU over the
// permuted gate/up weight, optional per-row RMSNorm scale).
//
// Why a second GEMM: at M <= 64 the 256x256-tile kernel (gemm_kernels.h)
// computes 4x the useful MFMA work per tile and a 16-tile N = 4096 product
// leaves most CUs of even a 32-CU partition idle, so a micro-forward ran at
// ~0.42 TB/s of weight traffic (profiles/r6_realtime_modes.md).  A small step
// is a stream over the weights: this kernel reads every weight byte once with
// 64 contiguous bytes a lane (256 B a weight row per four lanes), keeps the
// whole M in one block (MT 16-row MFMA fragments), keeps two 128-deep steps
// of weight loads in flight behind the one it computes, and splits K when
// the column blocks alone cannot fill the CUs.
//
// Layout.  A block = 4 waves = 128 output columns x a K range; wave w owns
// columns [32w, 32w + 32) as two 16-column fragments.  K is walked 128 at a
// time in a PERMUTED order: MFMA step s4 of lane (fr, fq) takes the K chunk
// (fq * 4 + s4) * 8 for BOTH operands, so each lane's weight read for the
// 128-deep step is one contiguous 64-byte run and the sum over K is unchanged
// (the same permutation on both sides).  A[0:M][k:k+128] is staged in LDS
// (double buffered, rows padded by 16 B) and read as MFMA A fragments; the
// weight fragments come straight from global memory into a ring of three
// register stages, two 128-deep steps ahead.
//
// Split-K partials are written to ws[S][M][N] fp32 and summed in split
// order by the finalize kernel (deterministic: no atomics), which applies
// the row scale and the epilogue and writes bf16.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace llmq {

typedef __attribute__((ext_vector_type(8))) short sk_bf16x8;
typedef __attribute__((ext_vector_type(4))) float sk_f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int sk_u32x4;

constexpr int SK_NB = 128;          // output columns per block
constexpr int SK_KS = 128;          // K per pipeline step
constexpr int SK_LDA = SK_KS + 8;   // LDS row stride of the A tile (elements)

enum { SK_EPI_STORE = 0, SK_EPI_RESID = 1, SK_EPI_SWIGLU = 2 };

// M > 64 (up to SK_MAX_M): blockIdx.x also selects one of nm 128-row chunks
// of A (MT = 8; a chunk's A rows staged in two 64-row groups).  Every chunk re-reads its column block's weights, so the nm
// chunks of a column block run on one XCD back to back (block b -> XCD b % 8:
// chunk fastest within the XCD's share) and the repeats come from its L2.
constexpr int SK_MAX_M = 1024;           // up to 8 chunks (o / down at mid-size steps)

template <int MT>
__global__ void __launch_bounds__(256)
skinny_partial_kernel(const uint16_t* __restrict__ A, const uint16_t* __restrict__ W, float* __restrict__ ws,
                      int M, int N, int K, int kc, int nm) {
  __shared__ __align__(16) uint16_t As[2][MT * 16][SK_LDA];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int fr = lane & 15, fq = lane >> 4;
  const int ncb = N / SK_NB;
  int cb = blockIdx.x, mc = 0;
  if (nm > 1) {
    if ((ncb & 7) == 0) {
      const int b = blockIdx.x, idx = b >> 3;
      cb = (idx / nm) * 8 + (b & 7);
      mc = idx % nm;
    } else {
      cb = blockIdx.x / nm;
      mc = blockIdx.x % nm;
    }
  }
  const int m0 = mc * (MT * 16);
  const int Ml = min(M - m0, MT * 16);             // rows of this chunk
  const int n0 = cb * SK_NB + w * 32;
  const int kb = blockIdx.y * kc;
  const int nsteps = kc / SK_KS;
  // weight rows of this lane's two fragments; K offset of its 64-byte run
  const uint16_t* wp0 = W + (size_t)(n0 + fr) * K + kb + fq * 32;
  const uint16_t* wp1 = wp0 + (size_t)16 * K;
  // A staging: thread t -> row g * 64 + t / 4 of each 64-row group g,
  // chunks (t % 4) * 4 .. + 3 (16 B each)
  constexpr int RG = (MT * 16 + 63) / 64;
  const int arow = tid >> 2, acb = (tid & 3) * 4;
  bool a_on[RG], a_live[RG];
  const uint16_t* ap[RG];
#pragma unroll
  for (int g = 0; g < RG; ++g) {
    const int r = g * 64 + arow;
    a_on[g] = r < MT * 16;
    a_live[g] = a_on[g] && r < Ml;
    ap[g] = A + (size_t)(m0 + (a_live[g] ? r : 0)) * K + kb + acb * 8;
  }

  sk_f32x4 acc[MT][2];
#pragma unroll
  for (int m = 0; m < MT; ++m) {
    acc[m][0] = sk_f32x4{0.f, 0.f, 0.f, 0.f};
    acc[m][1] = sk_f32x4{0.f, 0.f, 0.f, 0.f};
  }
  // weight fragments in a ring of three register stages: step k computes
  // from stage k % 3 while steps k + 1 and k + 2 are in flight (64 B a lane
  // a fragment a step: enough bytes outstanding per CU to stream the weights
  // at the partition's bandwidth); the stage index is compile-time below
  sk_u32x4 wb[3][2][4];
  sk_u32x4 ab[RG][4];
  auto load_w = [&](auto stc, int step) {
    constexpr int ST = decltype(stc)::value;
    const int ko = step * SK_KS;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      wb[ST][0][i] = *reinterpret_cast<const sk_u32x4*>(wp0 + ko + 8 * i);
      wb[ST][1][i] = *reinterpret_cast<const sk_u32x4*>(wp1 + ko + 8 * i);
    }
  };
  auto load_a = [&](int step) {
    const int ko = step * SK_KS;
#pragma unroll
    for (int g = 0; g < RG; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        ab[g][i] = a_live[g] ? *reinterpret_cast<const sk_u32x4*>(ap[g] + ko + 8 * i) : sk_u32x4{0u, 0u, 0u, 0u};
  };
  auto store_a = [&](int buf) {
#pragma unroll
    for (int g = 0; g < RG; ++g) {
      if (a_on[g]) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
          *reinterpret_cast<sk_u32x4*>(&As[buf][g * 64 + arow][(acb + i) * 8]) = ab[g][i];
      }
    }
  };
  // one 128-deep step from register stage CUR (= step % 3) and A buffer
  // step % 2; the weights of step + 2 and the A tile of step + 1 load meanwhile
  auto run_step = [&](auto curc, int step) {
    constexpr int CUR = decltype(curc)::value;
    if (step + 2 < nsteps) load_w(std::integral_constant<int, (CUR + 2) % 3>{}, step + 2);
    const bool more = step + 1 < nsteps;
    if (more) load_a(step + 1);
    const int abuf = step & 1;
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      const sk_bf16x8 b0 = __builtin_bit_cast(sk_bf16x8, wb[CUR][0][s4]);
      const sk_bf16x8 b1 = __builtin_bit_cast(sk_bf16x8, wb[CUR][1][s4]);
#pragma unroll
      for (int m = 0; m < MT; ++m) {
        const sk_bf16x8 a = *reinterpret_cast<const sk_bf16x8*>(&As[abuf][m * 16 + fr][(fq * 4 + s4) * 8]);
        acc[m][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b0, acc[m][0], 0, 0, 0);
        acc[m][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b1, acc[m][1], 0, 0, 0);
      }
    }
    if (more) store_a(abuf ^ 1);
    __syncthreads();
  };

  load_a(0);
  load_w(std::integral_constant<int, 0>{}, 0);
  if (nsteps > 1) load_w(std::integral_constant<int, 1>{}, 1);
  store_a(0);
  __syncthreads();
  for (int step = 0; step < nsteps; step += 3) {
    run_step(std::integral_constant<int, 0>{}, step);
    if (step + 1 < nsteps) run_step(std::integral_constant<int, 1>{}, step + 1);
    if (step + 2 < nsteps) run_step(std::integral_constant<int, 2>{}, step + 2);
  }
  // partials: lane -> column n0 + j * 16 + fr, rows m * 16 + fq * 4 + e
  float* out = ws + (size_t)blockIdx.y * M * N;
#pragma unroll
  for (int m = 0; m < MT; ++m)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = m * 16 + fq * 4 + e;
        if (row < Ml) out[(size_t)(m0 + row) * N + n0 + j * 16 + fr] = acc[m][j][e];
      }
}

__device__ __forceinline__ uint16_t sk_f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// One thread = 4 consecutive output columns of one row: the S split partials
// summed in split order, times the row scale, then the epilogue.
//   STORE:  C[row][c]  = sum                          (C: [M][N])
//   RESID:  C[row][c] += sum, one bf16 rounding       (C: [M][N])
//   SWIGLU: C[row][f]  = silu(g) * u over the swiglu-permuted columns of W
//           (gate f at 256 t + 64 wc + c, up 32 columns later; C: [M][N / 2])
template <int EPI>
__global__ void __launch_bounds__(256)
skinny_finalize_kernel(const float* __restrict__ ws, int S, int M, int N, const float* __restrict__ rs,
                       uint16_t* __restrict__ C) {
  const int Nout = EPI == SK_EPI_SWIGLU ? N / 2 : N;
  const int per_row = Nout / 4;
  const int gid = blockIdx.x * 256 + threadIdx.x;
  if (gid >= M * per_row) return;
  const int row = gid / per_row, c4 = (gid % per_row) * 4;
  const float scale = rs ? rs[row] : 1.f;
  if constexpr (EPI == SK_EPI_SWIGLU) {
    const int t = c4 / 128, wc = (c4 % 128) / 32, c = c4 % 32;
    const int gcol = t * 256 + wc * 64 + c;
    sk_f32x4 g = sk_f32x4{0.f, 0.f, 0.f, 0.f}, u = g;
    for (int s = 0; s < S; ++s) {
      const float* p = ws + ((size_t)s * M + row) * N;
      g += *reinterpret_cast<const sk_f32x4*>(p + gcol);
      u += *reinterpret_cast<const sk_f32x4*>(p + gcol + 32);
    }
    uint16_t o[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float ge = g[e] * scale, ue = u[e] * scale;
      o[e] = sk_f2bf(ge / (1.f + __expf(-ge)) * ue);
    }
    *reinterpret_cast<uint2*>(C + (size_t)row * Nout + c4) =
        make_uint2((uint32_t)o[0] | ((uint32_t)o[1] << 16), (uint32_t)o[2] | ((uint32_t)o[3] << 16));
  } else {
    sk_f32x4 v = sk_f32x4{0.f, 0.f, 0.f, 0.f};
    for (int s = 0; s < S; ++s) v += *reinterpret_cast<const sk_f32x4*>(ws + ((size_t)s * M + row) * N + c4);
    uint2* cp = reinterpret_cast<uint2*>(C + (size_t)row * N + c4);
    float r[4] = {v[0] * scale, v[1] * scale, v[2] * scale, v[3] * scale};
    if constexpr (EPI == SK_EPI_RESID) {
      const uint2 cr = *cp;
      r[0] += __uint_as_float(cr.x << 16);
      r[1] += __uint_as_float(cr.x & 0xffff0000u);
      r[2] += __uint_as_float(cr.y << 16);
      r[3] += __uint_as_float(cr.y & 0xffff0000u);
    }
    *cp = make_uint2((uint32_t)sk_f2bf(r[0]) | ((uint32_t)sk_f2bf(r[1]) << 16),
                     (uint32_t)sk_f2bf(r[2]) | ((uint32_t)sk_f2bf(r[3]) << 16));
  }
}

}  // namespace llmq
