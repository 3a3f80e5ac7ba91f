// Hand-written gfx950 bf16 GEMM for the backend's MLP: C = A · Wᵀ with
// A [M][K] and W [N][K] both K-contiguous (the layout F.linear feeds
// hipBLASLt), fp32 accumulation on v_mfma_f32_16x16x32_bf16, and three
// epilogues:
//
//   GM_EPI_STORE   C[M][N] = A·Wᵀ                         (bf16)
//   GM_EPI_SWIGLU  H[M][N/2] = silu(A·Wgᵀ) * (A·Wuᵀ)       (Llama gate/up)
//   GM_EPI_RESID   C[M][N] += A·Wᵀ   (bf16 C read + written; one rounding of
//                  the fp32 sum, as hipBLASLt's beta = 1: the o / down
//                  projections into the residual stream)
//
// The SwiGLU form removes the separate silu_mul pass and the HBM round trip
// of the [M][2F] gate/up product (profiles/r1_gemm_experiments.md): W rows are
// pre-permuted (`swiglu_permute` in ops/gemm.py) so that each wave's 64
// output columns are 32 gate features followed by the same 32 up features,
// i.e. every lane holds g and u of one (row, feature) in the same register
// slot of two accumulators -- the epilogue is pure register math.
//
// Structure (cdna_hip_programming.md §5, "the 256² 8-phase template"):
//   * 256x256 output tile, BK = 64, 512 threads = 8 waves as 2 (M) x 4 (N),
//     128x64 outputs per wave = 32 16x16 fp32 accumulators (128 AGPR/VGPR).
//   * LDS 128 KiB = 2 K-tile buffers x {A0, A1, B0, B1} half-tiles of 128
//     rows x 128 B.  A half h holds the rows of m-half h of BOTH wave rows,
//     B half h the columns of n-half h of all four wave columns, so each
//     half-tile is consumed in exactly one quadrant phase and can be
//     restaged as soon as that phase's reads retire.
//   * Staging by buffer_load_dwordx4 ... lds (16 B per lane, lane-linear LDS
//     image; fixed per-lane VGPR offset + scalar K offset, no VALU per load); the bank swizzle p = c ^ ((row >> 1) & 7) on the 16-B chunk is
//     applied to the per-lane SOURCE address and to the ds_read address
//     (rule 21), which makes the 16 x b128 fragment reads conflict-free
//     across the ds_read_b128 lane groups of the 128-B-row image.
//   * 8 phases per 2 K-tiles: each phase reads one operand half, issues one
//     half-tile prefetch (2 glds per lane), barrier, 16 MFMAs (one quadrant x
//     K = 64), barrier.  The prefetch runs 3 half-tiles ahead; a counted
//     `s_waitcnt vmcnt(6)` at phases 4 and 8 (never 0 in the steady state)
//     retires exactly the buffer the next phase reads, and raw s_barrier is
//     used throughout so no wait drains the DMA queue early.
//   * XCD-aware block order: blocks that the dispatcher puts on one XCD take
//     a contiguous run of tiles, grouped 8 M-tiles x N so concurrently
//     running tiles share A and W panels in that XCD's L2.
//   * M need not be a multiple of 256: A rows are clamped on load, rows >= M
//     are not stored.  K % 64 == 0 and N % 256 == 0 are checked by the host.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmq {

typedef __attribute__((ext_vector_type(8))) short gm_bf16x8;
typedef __attribute__((ext_vector_type(4))) float gm_f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int gm_u32x4;

constexpr int GM_BM = 256, GM_BN = 256, GM_BK = 64, GM_THREADS = 512;
constexpr int GM_HALF_BYTES = 128 * GM_BK * 2;     // 16 KiB
constexpr int GM_BUF_BYTES = 4 * GM_HALF_BYTES;    // A0 A1 B0 B1
constexpr int GM_LDS_BYTES = 2 * GM_BUF_BYTES;     // 128 KiB
constexpr int GM_GROUP_M = 8;                    // default M-tiles per block-order group

enum { GM_EPI_STORE = 0, GM_EPI_SWIGLU = 2, GM_EPI_ROPE = 3, GM_EPI_ARGMAX = 4, GM_EPI_RESID = 5,
       GM_EPI_RESID_LDS = 6, GM_EPI_RESID_PRE = 7, GM_EPI_RESID_RMS = 8 };
// GM_EPI_RESID_PRE: GM_EPI_RESID_LDS whose first quarter of the residual tile
// (rows 0-31 of every wave's 128 x 64 block) is fetched into the 32 KiB of
// LDS gfx950 has beyond the operand buffers at kernel start, so it is in LDS
// long before the epilogue; the launch asks for 160 KiB.
constexpr int GM_LDS_SPARE = 32768;
template <int EPI>
constexpr int gm_lds_bytes() { return EPI == GM_EPI_RESID_PRE ? GM_LDS_BYTES + GM_LDS_SPARE : GM_LDS_BYTES; }

// GM_EPI_ARGMAX: the LM head's greedy sampling as the epilogue -- no [M][N]
// logits tensor.  Each tile writes, per row, the max over its 256 columns and
// the (global) column of its first occurrence into pv / pi [M][N / 256];
// gemm_argmax_reduce_kernel picks the first maximum over the tiles (ties go
// to the lower column, as torch.argmax does).  Values are the fp32
// accumulators (not bf16-rounded logits).
// Epilogue side outputs.  GM_EPI_ARGMAX: per-(row, column tile) max value /
// index partials (pv, pi).  GM_EPI_RESID_RMS (GM_EPI_RESID_LDS plus): the
// RMSNorm row scale of the updated residual rows, fused into the epilogue --
// each block's per-row sums of squares of the bf16 values it stores (rpart
// [tiles_m][tiles_n][256], written through to memory), and the last of a
// row tile's tiles_n blocks (rticket[tiles_m], zero at launch, re-zeroed)
// adds them in column-tile order and writes 1 / sqrt(sum / N + reps) to
// rscale[tm * 256 + row]: what row_rms_kernel computes, in a fixed order,
// without the 33 MB re-read of the rows by a separate launch.
struct GmSide {
  float* pv;
  int32_t* pi;
  float* rpart;
  int* rticket;
  float* rscale;
  float reps;
};

// GM_EPI_ROPE: the fused qkv projection's epilogue = the rope_kv kernel
// (llama_kernels.h): RoPE (rotate-half) on q and k, q to ``q``, k / v into
// this layer's cache at (slot[row], pos[row]); W rows are the plain
// [q heads | k heads | v heads] order (N = (Hq + 2 Hkv) * 128).
struct GmRope {
  const int32_t* pos;
  const int32_t* slot;
  const float* cos_t;                              // [max_ctx][64]
  const float* sin_t;
  uint16_t* q;                                     // [M][Hq * 128]
  uint16_t* kc;                                    // [n_slots][Hkv][max_ctx][128]
  uint16_t* vc;
  int Hq, Hkv, max_ctx, n_slots;
};
enum { GM_A0 = 0, GM_A1 = 1, GM_B0 = 2, GM_B1 = 3 };

__device__ __forceinline__ uint16_t gm_f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);                 // round to nearest even (finite inputs)
  return (uint16_t)(u >> 16);
}

// Per-row scales of this lane's 32 accumulator rows (row0 + mh*64 + m*16 +
// fq*4 + j): eight 16-B loads issued together, one branch for the whole set
// (a per-element load under a runtime condition makes hipcc wait for each
// load in turn).  rs must hold ceil(M / 256) * 256 floats (ops/gemm.py pads).
__device__ __forceinline__ void gm_load_row_scales(const float* __restrict__ rs, int row0, int fq,
                                                   gm_f32x4 (&sc)[2][4]) {
  if (rs) {
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int m = 0; m < 4; ++m)
        sc[mh][m] = *reinterpret_cast<const gm_f32x4*>(rs + row0 + mh * 64 + m * 16 + fq * 4);
  } else {
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int m = 0; m < 4; ++m) sc[mh][m] = gm_f32x4{1.f, 1.f, 1.f, 1.f};
  }
}

// Split-K for the last partial wave of tiles (GM_EPI_ROPE): with 384 tiles on
// 256 CUs the second wave would run half empty.  Tiles [full, nwg) run as two
// blocks each over one half of K; the first to finish publishes its fp32
// accumulators (agent-scope release), the second adds them (acquire) and runs
// the epilogue -- cdna_hip_programming.md §5 "Projection GEMM" item 2.
#define GM_CPOL_SC1 16   // cache-policy bit: agent-scope coherent access
typedef unsigned int gm_u32x4 __attribute__((ext_vector_type(4)));

struct GmSplit {
  int full;       // tiles [0, full) run whole
  float* ws;      // [nwg - full][GM_THREADS * 128] fp32 accumulator slabs (nullptr: no split)
  int* cnt;       // [nwg - full][2]: ticket, ready -- zero at launch; the second half re-zeroes them
};

typedef __attribute__((address_space(3))) void* gm_lds_ptr;

// One half-tile (128 rows x 64 bf16) global -> LDS: 2 buffer_load ... lds per
// lane.  The per-lane row/chunk offset is a fixed VGPR, the K-tile offset a
// scalar (soffset), so the K-loop spends no VALU on staging addresses.
__device__ __forceinline__ void gm_stage(__amdgpu_buffer_rsrc_t rs, uint32_t v0, uint32_t v1, uint32_t soff,
                                         uint8_t* smem, uint32_t dst0, uint32_t dst1) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (gm_lds_ptr)(smem + dst0), 16, v0, soff, 0, 0);
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (gm_lds_ptr)(smem + dst1), 16, v1, soff, 0, 0);
}

#define GM_FENCE() __builtin_amdgcn_sched_barrier(0)
#define GM_BARRIER()                  \
  do {                                \
    GM_FENCE();                       \
    __builtin_amdgcn_s_barrier();     \
    GM_FENCE();                       \
  } while (0)

// One output tile (or one K-half of a split tile): block ``bid`` of the
// launch's block order.  gemm_bf16_kernel runs one per block, or -- PERSIST --
// a grid of at most one block per CU walks bid, bid + gridDim.x, ...
template <int EPI, bool STAGGER, int SCHED>
__device__ __forceinline__ void gemm_tile(
    uint8_t* __restrict__ smem, const uint16_t* __restrict__ A, const uint16_t* __restrict__ W,
    uint16_t* __restrict__ C, int M, int N, int K, int group_m, const float* __restrict__ rs, const GmRope& rp,
    const GmSplit& sp, const GmSide& am, const int bid) {
  static_assert(EPI != GM_EPI_RESID_PRE || SCHED >= 1, "the residual prefetch is issued by the SCHED >= 1 prologue");

  const int tiles_m = (M + GM_BM - 1) / GM_BM;
  const int tiles_n = N / GM_BN;
  const int nwg = tiles_m * tiles_n;
  const int full = sp.ws ? sp.full : nwg;
  // XCD-contiguous remap (bijective for any count) of the whole tiles, then
  // 8-M-tile grouping; split tiles take two consecutive blocks
  int pid, khalf = -1;
  if (bid < full) {
    const int xcd = bid & 7, loc = bid >> 3, q8 = full >> 3, r8 = full & 7;
    pid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
  } else {
    // split tiles: the same XCD-contiguous remap over the tail's blocks, so
    // an XCD runs both K-halves of a contiguous run of tiles (their A / B
    // panels share its L2) instead of one half of every 4th tile
    const int t = bid - full, nt2 = nwg - full;
    const int n2 = 2 * nt2;                        // blocks of the tail
    const int xcd = t & 7, loc = t >> 3, q8 = n2 >> 3, r8 = n2 & 7;
    const int j = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + loc;
    pid = full + (j >> 1);
    khalf = j & 1;
  }
  const int group = pid / (group_m * tiles_n);
  const int first_m = group * group_m;
  const int gsize = min(tiles_m - first_m, group_m);
  const int tm = first_m + (pid % (group_m * tiles_n)) % gsize;
  const int tn = (pid % (group_m * tiles_n)) / gsize;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // SCHED 8 / 9 (diagnostics): shader-clock and 100 MHz reference stamps at
  // entry and exit, written by thread 0 to am.pv as 4 x u64 per block --
  // the in-kernel clock = d(memtime) / d(memrealtime) x 100 MHz, unprofiled
  // (MI355X_MICROARCH.md 'DVFS give-back' item 6)
  uint64_t st_t0 = 0, st_r0 = 0;
  if constexpr (SCHED == 8 || SCHED == 9) {
    st_t0 = __builtin_amdgcn_s_memtime();
    st_r0 = __builtin_amdgcn_s_memrealtime();
  }
  const int wr = w >> 2, wc = w & 3;

  // ---- staging sources: half h, instruction i -> LDS local row lr = i*64 + w*8 + lane/8
  const int srow = w * 8 + (lane >> 3);            // 0..63
  const int schunk = (lane & 7) ^ ((srow >> 1) & 7);   // source chunk for LDS slot lane&7
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, M * K * 2, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsw = __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, N * K * 2, 0x00020000);
  uint32_t va[2][2], vb[2][2];                     // byte offsets (row, chunk) of K-tile 0
  // SCHED 10 (diagnostic, wrong numerics): every block stages the panels of
  // tile (0, 0), so nearly every staging read hits the XCD's L2
  const int ltm = SCHED == 10 ? 0 : tm, ltn = SCHED == 10 ? 0 : tn;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int row = ltm * GM_BM + i * 128 + h * 64 + srow;
      row = row < M ? row : M - 1;
      va[h][i] = (uint32_t)row * (uint32_t)K * 2u + (uint32_t)schunk * 16u;
      const int col = ltn * GM_BN + (2 * i + (w >> 2)) * 64 + h * 32 + (w & 3) * 8 + (lane >> 3);
      vb[h][i] = (uint32_t)col * (uint32_t)K * 2u + (uint32_t)schunk * 16u;
    }
  }
  // LDS destination (wave-uniform) of instruction i inside a half-tile
  const uint32_t dst_i0 = (uint32_t)(w * 8) * 128u;
  const uint32_t dst_i1 = (uint32_t)(64 + w * 8) * 128u;

  // ---- fragment read offsets (bytes inside a half-tile), per k-step kk
  const int fr = lane & 15, fq = lane >> 4;
  uint32_t aoff[2][2], boff[2][2];                 // [buffer][kk]; buffer 1 = +64 KiB (beyond ds offset:)
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) {
    const int c = fq + 4 * kk;
    aoff[0][kk] = (uint32_t)(wr * 64 + fr) * 128u + (uint32_t)((c ^ ((fr >> 1) & 7)) * 16);
    boff[0][kk] = (uint32_t)(wc * 32 + fr) * 128u + (uint32_t)((c ^ ((fr >> 1) & 7)) * 16) + 2 * GM_HALF_BYTES;
    aoff[1][kk] = aoff[0][kk] + GM_BUF_BYTES;
    boff[1][kk] = boff[0][kk] + GM_BUF_BYTES;
  }

  gm_f32x4 acc[2][4][2][2];                        // [mh][m][nh][n]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int d = 0; d < 2; ++d) acc[a][b][c][d] = gm_f32x4{0.f, 0.f, 0.f, 0.f};

  gm_bf16x8 af[4][2];                              // one m-half: [m][kk]
  gm_bf16x8 bfr[2][2][2];                          // both n-halves: [nh][n][kk]
  gm_bf16x8 b0y[2][2];                             // SCHED >= 1: buffer-1 B0 fragments

#define GM_STAGE(BUF, HALF, KT)                                                               \
  do {                                                                                        \
    const uint32_t _ko = (uint32_t)((KT) + kt0) * (GM_BK * 2);                                \
    const uint32_t _b = (uint32_t)(BUF) * GM_BUF_BYTES + (uint32_t)(HALF) * GM_HALF_BYTES;   \
    if constexpr ((HALF) < 2)                                                                 \
      gm_stage(rsa, va[(HALF)][0], va[(HALF)][1], _ko, smem, _b + dst_i0, _b + dst_i1);       \
    else                                                                                      \
      gm_stage(rsw, vb[(HALF)-2][0], vb[(HALF)-2][1], _ko, smem, _b + dst_i0, _b + dst_i1);   \
  } while (0)

#define GM_READ_A(BUF, MH)                                                                     \
  do {                                                                                         \
    _Pragma("unroll") for (int m = 0; m < 4; ++m)                                              \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        af[m][kk] = *reinterpret_cast<const gm_bf16x8*>(smem + aoff[BUF][kk] + (MH) * GM_HALF_BYTES + m * 2048); \
  } while (0)

#define GM_READ_B(BUF, NH)                                                                     \
  do {                                                                                         \
    _Pragma("unroll") for (int n = 0; n < 2; ++n)                                              \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        bfr[NH][n][kk] = *reinterpret_cast<const gm_bf16x8*>(smem + boff[BUF][kk] + (NH) * GM_HALF_BYTES + n * 2048); \
  } while (0)

#define GM_MFMA(MH, NH)                                                                        \
  do {                                                                                         \
    __builtin_amdgcn_s_setprio(1);                                                             \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                           \
      _Pragma("unroll") for (int m = 0; m < 4; ++m)                                            \
        _Pragma("unroll") for (int n = 0; n < 2; ++n)                                          \
          acc[MH][m][NH][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m][kk], bfr[NH][n][kk], \
                                                                      acc[MH][m][NH][n], 0, 0, 0); \
    __builtin_amdgcn_s_setprio(0);                                                             \
  } while (0)

// SCHED >= 1 helpers: B0 fragments into an explicit register set, MFMA with it
#define GM_READ_B0_INTO(BUF, DST)                                                              \
  do {                                                                                         \
    _Pragma("unroll") for (int n = 0; n < 2; ++n)                                              \
      _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                         \
        DST[n][kk] = *reinterpret_cast<const gm_bf16x8*>(smem + boff[BUF][kk] + n * 2048);     \
  } while (0)

#define GM_MFMA_WITH(MH, NH, BREG)                                                             \
  do {                                                                                         \
    if constexpr (SCHED == 1) __builtin_amdgcn_s_setprio(1);                                   \
    _Pragma("unroll") for (int kk = 0; kk < 2; ++kk)                                           \
      _Pragma("unroll") for (int m = 0; m < 4; ++m)                                            \
        _Pragma("unroll") for (int n = 0; n < 2; ++n)                                          \
          acc[MH][m][NH][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[m][kk], BREG[n][kk],  \
                                                                      acc[MH][m][NH][n], 0, 0, 0); \
    if constexpr (SCHED == 1) __builtin_amdgcn_s_setprio(0);                                   \
  } while (0)

#define GM_LGKM(N) asm volatile("s_waitcnt lgkmcnt(" #N ")" ::: "memory")
#define GM_VMCNT(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")

  // K-tiles of this block: all, or one half for a split tile (host: nt % 4 == 0)
  const int nt = khalf < 0 ? K / GM_BK : K / GM_BK / 2;
  const int kt0 = khalf > 0 ? nt : 0;

  if constexpr (SCHED >= 1) {
    // Wave priority.  SCHED 2 (default): one static s_setprio 1 for wave row
    // 1 (the later-dispatched half, cdna_hip_programming.md T5 static form),
    // no per-cluster flips -- 1.7 % faster than SCHED 1 (s_setprio 1 around
    // every MFMA cluster) at T = 4041 (profiles/r2_gemm_prio_ab.jsonl).
    // SCHED 3 / 4 (A/B only): the static priority on wave row 0 / none.
    if constexpr (SCHED == 2 || SCHED == 3 || SCHED >= 5) {
      if (wr == (SCHED == 3 ? 0 : 1)) __builtin_amdgcn_s_setprio(1);
    }
    // Balanced schedule: every phase retires the half-tile staged 3 phases
    // earlier (vmcnt(6) each phase), so the NEXT buffer's B0 fragments can be
    // read one phase early (phases 4 and 8, which otherwise read nothing):
    // 8/4/8/4 fragment reads per phase instead of 12/4/8/0.  Stage order per
    // buffer is B0, A0, B1, A1; every restage is >= 2 phases after the
    // half-tile's last read (safe with the wave-row stagger).
    if constexpr (EPI == GM_EPI_RESID_PRE) {
      // the residual rows 0-31 of this wave's output block -> spare LDS; the
      // prologue's counted vmcnt waits retire them with the first half-tiles
      const int col0p = tn * GM_BN + wc * 64, row0p = tm * GM_BM + wr * 128;
      const __amdgpu_buffer_rsrc_t rsp =
          __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, (uint32_t)M * (uint32_t)N * 2u, 0x00020000);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = i * 8 + (lane >> 3), c = lane & 7;
        const uint32_t vo = ((uint32_t)(row0p + r) * (uint32_t)N + (uint32_t)(col0p + c * 8)) * 2u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsp, (gm_lds_ptr)(smem + GM_LDS_BYTES + w * 4096 + i * 1024), 16,
                                                 vo, 0, 0, 0);
      }
    }
    GM_STAGE(0, GM_B0, 0);
    GM_STAGE(0, GM_A0, 0);
    GM_STAGE(0, GM_B1, 0);
    GM_STAGE(0, GM_A1, 0);
    GM_STAGE(1, GM_B0, 1);
    GM_STAGE(1, GM_A0, 1);
    GM_STAGE(1, GM_B1, 1);
    GM_VMCNT(6);
    GM_BARRIER();
    GM_READ_B0_INTO(0, bfr[0]);
    if constexpr (SCHED >= 5 && SCHED <= 7) {      // diagnostics: every fragment register defined
      GM_READ_A(0, 0);
      GM_READ_B(0, 1);
      GM_READ_B0_INTO(1, b0y);
    }
    if (STAGGER && wr == 1) GM_BARRIER();

#define GM_PHASE_END(MH, NH, BREG) \
  do {                             \
    GM_BARRIER();                  \
    GM_LGKM(0);                    \
    GM_MFMA_WITH(MH, NH, BREG);    \
    GM_BARRIER();                  \
  } while (0)

    int t = 0;
    // SCHED 5-7: power/energy DIAGNOSTICS only (bench/gemm_energy_diag.hip; wrong
    // numerics, never dispatched by the library): 5 skips the A fragment
    // reads of phases 3 / 7 (one third fewer LDS read bytes, what a 128x128
    // wave tile would read), 6 skips every fragment read of the loop, 7 skips
    // every staging DMA of the loop (no L2 / HBM traffic in steady state).
    // SCHED 8 / 9: production / no-DMA with in-kernel clock stamps (below).
    constexpr bool kRdA = SCHED != 6, kRdA2 = SCHED != 5 && SCHED != 6, kRdB = SCHED != 6;
    constexpr bool kDma = SCHED != 7 && SCHED != 9;
#define GM_D_READ_A(C, B, H) do { if constexpr (C) GM_READ_A(B, H); } while (0)
#define GM_D_READ_B(B, H) do { if constexpr (kRdB) GM_READ_B(B, H); } while (0)
#define GM_D_READ_B0(B, D) do { if constexpr (kRdB) GM_READ_B0_INTO(B, D); } while (0)
#define GM_D_STAGE(B, H, K) do { if constexpr (kDma) GM_STAGE(B, H, K); } while (0)
    for (; t < nt - 2; t += 2) {
      {
        GM_D_READ_A(kRdA, 0, 0); GM_D_STAGE(1, GM_A1, t + 1); GM_VMCNT(6); GM_PHASE_END(0, 0, bfr[0]);
        GM_D_READ_B(0, 1); GM_D_STAGE(0, GM_B0, t + 2); GM_VMCNT(6); GM_PHASE_END(0, 1, bfr[1]);
        GM_D_READ_A(kRdA2, 0, 1); GM_D_STAGE(0, GM_A0, t + 2); GM_VMCNT(6); GM_PHASE_END(1, 1, bfr[1]);
        GM_D_READ_B0(1, b0y); GM_D_STAGE(0, GM_B1, t + 2); GM_VMCNT(6); GM_PHASE_END(1, 0, bfr[0]);
        GM_D_READ_A(kRdA, 1, 0); GM_D_STAGE(0, GM_A1, t + 2); GM_VMCNT(6); GM_PHASE_END(0, 0, b0y);
        GM_D_READ_B(1, 1); GM_D_STAGE(1, GM_B0, t + 3); GM_VMCNT(6); GM_PHASE_END(0, 1, bfr[1]);
        GM_D_READ_A(kRdA2, 1, 1); GM_D_STAGE(1, GM_A0, t + 3); GM_VMCNT(6); GM_PHASE_END(1, 1, bfr[1]);
        GM_D_READ_B0(0, bfr[0]); GM_D_STAGE(1, GM_B1, t + 3); GM_VMCNT(6); GM_PHASE_END(1, 0, b0y);
      }
    }
#undef GM_D_READ_A
#undef GM_D_READ_B
#undef GM_D_READ_B0
#undef GM_D_STAGE
    {                                              // last two K-tiles: drain
        GM_READ_A(0, 0); GM_STAGE(1, GM_A1, t + 1); GM_VMCNT(6); GM_PHASE_END(0, 0, bfr[0]);
        GM_READ_B(0, 1); GM_VMCNT(4); GM_PHASE_END(0, 1, bfr[1]);
        GM_READ_A(0, 1); GM_VMCNT(2); GM_PHASE_END(1, 1, bfr[1]);
        GM_READ_B0_INTO(1, b0y); GM_VMCNT(0); GM_PHASE_END(1, 0, bfr[0]);
        GM_READ_A(1, 0); GM_PHASE_END(0, 0, b0y);
        GM_READ_B(1, 1); GM_PHASE_END(0, 1, bfr[1]);
        GM_READ_A(1, 1); GM_PHASE_END(1, 1, bfr[1]);
        GM_PHASE_END(1, 0, b0y);
    }
    if constexpr (SCHED == 2 || SCHED == 3 || SCHED >= 5) __builtin_amdgcn_s_setprio(0);
#undef GM_PHASE_END
  } else {
    // prologue: tile 0 -> buffer 0 (all halves), tile 1 -> buffer 1 (B0, A0, B1)
    GM_STAGE(0, GM_A0, 0);
    GM_STAGE(0, GM_A1, 0);
    GM_STAGE(0, GM_B0, 0);
    GM_STAGE(0, GM_B1, 0);
    GM_STAGE(1, GM_B0, 1);
    GM_STAGE(1, GM_A0, 1);
    GM_STAGE(1, GM_B1, 1);
    GM_VMCNT(6);
    GM_BARRIER();
    // wave-row 1 runs half a phase behind wave-row 0: on every SIMD (one wave
    // of each row) one wave's fragment reads + DMA issue overlap the other's
    // MFMA cluster.  One extra barrier here, balanced after the loop.
    if (STAGGER && wr == 1) GM_BARRIER();

    for (int t = 0; t < nt; t += 2) {
      const bool more = t + 2 < nt;                  // wave-uniform
      // ---- phase 1: buffer 0 quadrant (0,0); stage buffer 1 A1 (tile t+1)
      GM_READ_B(0, 0);
      GM_FENCE();
      GM_READ_A(0, 0);
      GM_STAGE(1, GM_A1, t + 1);
      GM_LGKM(8);
      GM_BARRIER();
      GM_LGKM(0);
      GM_MFMA(0, 0);
      GM_BARRIER();
      // ---- phase 2: quadrant (0,1); stage buffer 0 B0 (tile t+2)
      GM_READ_B(0, 1);
      if (more) GM_STAGE(0, GM_B0, t + 2);
      GM_BARRIER();
      GM_LGKM(0);
      GM_MFMA(0, 1);
      GM_BARRIER();
      // ---- phase 3: quadrant (1,1); stage buffer 0 A0
      GM_READ_A(0, 1);
      if (more) GM_STAGE(0, GM_A0, t + 2);
      GM_BARRIER();
      GM_LGKM(0);
      GM_MFMA(1, 1);
      GM_BARRIER();
      // ---- phase 4: quadrant (1,0); stage buffer 0 B1; retire buffer 1
      if (more) {
        GM_STAGE(0, GM_B1, t + 2);
        GM_VMCNT(6);
      } else {
        GM_VMCNT(0);
      }
      GM_BARRIER();
      GM_MFMA(1, 0);
      GM_BARRIER();
      // ---- phase 5: buffer 1 quadrant (0,0); stage buffer 0 A1
      GM_READ_B(1, 0);
      GM_FENCE();
      GM_READ_A(1, 0);
      if (more) GM_STAGE(0, GM_A1, t + 2);
      GM_LGKM(8);
      GM_BARRIER();
      GM_LGKM(0);
      GM_MFMA(0, 0);
      GM_BARRIER();
      // ---- phase 6: quadrant (0,1); stage buffer 1 B0 (tile t+3)
      GM_READ_B(1, 1);
      if (more) GM_STAGE(1, GM_B0, t + 3);
      GM_BARRIER();
      GM_LGKM(0);
      GM_MFMA(0, 1);
      GM_BARRIER();
      // ---- phase 7: quadrant (1,1); stage buffer 1 A0
      GM_READ_A(1, 1);
      if (more) GM_STAGE(1, GM_A0, t + 3);
      GM_BARRIER();
      GM_LGKM(0);
      GM_MFMA(1, 1);
      GM_BARRIER();
      // ---- phase 8: quadrant (1,0); stage buffer 1 B1; retire buffer 0
      if (more) {
        GM_STAGE(1, GM_B1, t + 3);
        GM_VMCNT(6);
      }
      GM_BARRIER();
      GM_MFMA(1, 0);
      GM_BARRIER();
    }
  }


  if (STAGGER && wr == 0) GM_BARRIER();

  // ---- split tile: the first K-half to finish hands its accumulators over
  if (khalf >= 0) {
    const int tix = pid - full;
    int* cnt = sp.cnt + 2 * tix;
    if (tid == 0) *reinterpret_cast<int*>(smem) =
        __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    const int ticket = *reinterpret_cast<volatile int*>(smem);
    __syncthreads();
    // The slab moves with agent-scope (sc1) stores / loads -- written through
    // and read past this XCD's L2 (the halves run on different XCDs) -- so
    // neither side needs the whole-L2 write-back / invalidate of an
    // agent-scope fence (measured: 156 vs 160 us at T=4041, fences cost L2
    // hits for every block on the XCD).  Order: all slab stores acknowledged
    // (vmcnt 0) -> barrier -> ready flag; the reader sees the flag before
    // its barrier and then loads.
    float* slab = sp.ws + (size_t)tix * GM_THREADS * 128;
    const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(slab, 0, GM_THREADS * 32 * 16, 0x00020000);
    if (ticket == 0) {                             // first: publish, then leave
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
#pragma unroll
          for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int d = 0; d < 2; ++d)
            {
              const int i = ((a * 4 + b) * 4 + c * 2 + d) * GM_THREADS + tid;
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(gm_u32x4, acc[a][b][c][d]), srs, i * 16,
                                                     0, GM_CPOL_SC1);
            }
      GM_VMCNT(0);
      __syncthreads();
      if (tid == 0) __hip_atomic_store(cnt + 1, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    if (tid == 0) {                                // second: wait for the slab (bounded)
      for (int spin = 0; spin < (1 << 24); ++spin) {
        if (__hip_atomic_load(cnt + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        __builtin_amdgcn_s_sleep(2);
      }
      GM_VMCNT(0);
      // both halves are done with the counters: leave them zeroed for the next launch
      __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(cnt + 1, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int d = 0; d < 2; ++d)
          {
            const int i = ((a * 4 + b) * 4 + c * 2 + d) * GM_THREADS + tid;
            acc[a][b][c][d] += __builtin_bit_cast(gm_f32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                   srs, i * 16, 0, GM_CPOL_SC1));
          }
  }

  // ---- epilogue through LDS (the staging buffers are free after the last barrier)
  const int row0 = tm * GM_BM + wr * 128;          // first output row of this wave
  if (EPI == GM_EPI_ARGMAX) {
    // per (row, wave): max over the wave's 64 columns -- 4 per lane, then the
    // 16 lanes of a row group (xor butterfly; ties keep the lower column)
    float* lv = reinterpret_cast<float*>(smem);                    // [256 rows][4 wave cols]
    int* lc = reinterpret_cast<int*>(smem + GM_BM * 4 * 4);
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          float v = acc[mh][m][0][0][j];
          int c = fr;
#pragma unroll
          for (int nh = 0; nh < 2; ++nh)
#pragma unroll
            for (int n = 0; n < 2; ++n) {
              const float x = acc[mh][m][nh][n][j];
              if (x > v) { v = x; c = nh * 32 + n * 16 + fr; }
            }
#pragma unroll
          for (int off = 1; off < 16; off <<= 1) {
            const float ov = __shfl_xor(v, off, 64);
            const int oc = __shfl_xor(c, off, 64);
            if (ov > v || (ov == v && oc < c)) { v = ov; c = oc; }
          }
          if (fr == 0) {
            const int r = wr * 128 + mh * 64 + m * 16 + fq * 4 + j;
            lv[r * 4 + wc] = v;
            lc[r * 4 + wc] = wc * 64 + c;
          }
        }
    __syncthreads();
    if (tid < GM_BM) {                             // one thread per tile row: the 4 wave columns
      const int grow = tm * GM_BM + tid;
      float v = lv[tid * 4];
      int c = lc[tid * 4];
#pragma unroll
      for (int k = 1; k < 4; ++k)
        if (lv[tid * 4 + k] > v) { v = lv[tid * 4 + k]; c = lc[tid * 4 + k]; }
      if (grow < M) {
        am.pv[(int64_t)grow * tiles_n + tn] = v;
        am.pi[(int64_t)grow * tiles_n + tn] = tn * GM_BN + c;
      }
    }
  } else if (EPI == GM_EPI_RESID) {
    // fp32 through LDS in four passes of 32 rows (8.5 KiB per wave, row
    // stride 68 floats: the four fq row groups of a write land on distinct
    // banks), then coalesced: 16 B of fp32 + 8 B of the bf16 residual per
    // lane, one rounding of the sum
    float* o = reinterpret_cast<float*>(smem + w * (32 * 68 * 4));
    const int col0 = tn * GM_BN + wc * 64;
    // every residual chunk of this lane loaded up front (64 VGPRs): after the
    // first store the compiler cannot move a load of C above a store to C, so
    // loads interleaved with the passes would wait out one round trip each
    uint2 cres[2][2][8];
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int mp = 0; mp < 2; ++mp)
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int qd = it * 64 + lane;
          const int grow = row0 + mh * 64 + mp * 32 + (qd >> 4);
          cres[mh][mp][it] = grow < M ? *reinterpret_cast<const uint2*>(C + (int64_t)grow * N + col0 + (qd & 15) * 4)
                                      : make_uint2(0u, 0u);
        }
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int mp = 0; mp < 2; ++mp) {
#pragma unroll
        for (int mm = 0; mm < 2; ++mm)
#pragma unroll
          for (int nh = 0; nh < 2; ++nh)
#pragma unroll
            for (int n = 0; n < 2; ++n)
#pragma unroll
              for (int j = 0; j < 4; ++j)
                o[(mm * 16 + fq * 4 + j) * 68 + nh * 32 + n * 16 + fr] = acc[mh][mp * 2 + mm][nh][n][j];
        GM_LGKM(0);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int it = 0; it < 8; ++it) {
          const int qd = it * 64 + lane;           // row qd/16, 4-float chunk qd%16
          const int r = qd >> 4, c4 = qd & 15;
          const int grow = row0 + mh * 64 + mp * 32 + r;
          const gm_f32x4 v = *reinterpret_cast<const gm_f32x4*>(o + r * 68 + c4 * 4);
          if (grow < M) {
            uint2* cp = reinterpret_cast<uint2*>(C + (int64_t)grow * N + col0 + c4 * 4);
            const uint2 cr = cres[mh][mp][it];
            const float r0 = __uint_as_float(cr.x << 16) + v[0], r1 = __uint_as_float(cr.x & 0xffff0000u) + v[1];
            const float r2 = __uint_as_float(cr.y << 16) + v[2], r3 = __uint_as_float(cr.y & 0xffff0000u) + v[3];
            *cp = make_uint2((uint32_t)gm_f2bf(r0) | ((uint32_t)gm_f2bf(r1) << 16),
                             (uint32_t)gm_f2bf(r2) | ((uint32_t)gm_f2bf(r3) << 16));
          }
        }
        GM_LGKM(0);
        __builtin_amdgcn_wave_barrier();
      }
  } else if (EPI == GM_EPI_RESID_LDS || EPI == GM_EPI_RESID_PRE || EPI == GM_EPI_RESID_RMS) {
    // The residual tile staged by DMA instead of through registers: the
    // wave's 128 x 64 bf16 block of C lands in its 16 KiB of LDS (16
    // buffer_load ... lds of 16 B per lane, row-major, the plain epilogue's
    // layout; rows >= M read 0 off the buffer descriptor), each lane adds its
    // fp32 accumulators in place (one rounding of the sum) and the block
    // leaves with the plain epilogue's 16-B coalesced stores.  Against the
    // four-pass fp32 staging (GM_EPI_RESID): half the global instructions
    // (16-B instead of 8-B loads and stores), no fp32 LDS round trip, one
    // wave barrier instead of eight.
    // (GM_EPI_RESID_PRE: rows 0-31 are already in the spare LDS, loaded at
    // kernel start; rows r < 32 are exactly mh = 0, m < 2 / it < 4 below)
    constexpr int kPre = EPI == GM_EPI_RESID_PRE ? 4 : 0;
    uint8_t* cw = smem + w * 16384;
    uint8_t* cpre = smem + GM_LDS_BYTES + w * 4096;
    auto rowp = [&](int r) -> uint8_t* { return (kPre && r < 32) ? cpre + r * 128 : cw + r * 128; };
    const int col0 = tn * GM_BN + wc * 64;
    const __amdgpu_buffer_rsrc_t rsc =
        __builtin_amdgcn_make_buffer_rsrc((void*)C, 0, (uint32_t)M * (uint32_t)N * 2u, 0x00020000);
#pragma unroll
    for (int i = kPre; i < 16; ++i) {              // LDS bytes [i KiB, i+1 KiB): rows 8i .. 8i+7
      const int r = i * 8 + (lane >> 3), c = lane & 7;
      const uint32_t vo = ((uint32_t)(row0 + r) * (uint32_t)N + (uint32_t)(col0 + c * 8)) * 2u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsc, (gm_lds_ptr)(cw + i * 1024), 16, vo, 0, 0, 0);
    }
    GM_VMCNT(0);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              const int r = mh * 64 + m * 16 + fq * 4 + j;
              uint16_t* e = reinterpret_cast<uint16_t*>(rowp(r) + (nh * 32 + n * 16 + fr) * 2);
              *e = gm_f2bf(__uint_as_float((uint32_t)*e << 16) + acc[mh][m][nh][n][j]);
            }
    GM_LGKM(0);
    __builtin_amdgcn_wave_barrier();
    constexpr bool rms = EPI == GM_EPI_RESID_RMS;   // + the RMSNorm row scales (GmSide.r*)
    float ssq[16];
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int qd = it * 64 + lane;               // row qd/8, chunk qd%8
      const int r = qd >> 3, cb = qd & 7;
      const int grow = row0 + r;
      const gm_u32x4 v = *reinterpret_cast<const gm_u32x4*>(rowp(r) + cb * 16);
      if (grow < M) *reinterpret_cast<gm_u32x4*>(C + (int64_t)grow * N + col0 + cb * 8) = v;
      if constexpr (rms) {                         // squares of the 8 stored bf16 values
        float q = 0.f;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float lo = __uint_as_float(v[e] << 16), hi = __uint_as_float(v[e] & 0xFFFF0000u);
          q += lo * lo + hi * hi;
        }
        ssq[it] = q;
      }
    }
    if constexpr (rms) {
      // row r = it * 8 + lane / 8 of this wave's 128: its 8 chunk lanes meet
      // by three xor-shuffles; the wave's 128 partials go to the start of its
      // own (now unused) 16 KiB of LDS, the block's 4 column waves of a row
      // half are added in wc order, written through to rpart, and the last
      // block of the row tile (ticket) finishes the scale
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        float q = ssq[it];
        q += __shfl_xor(q, 1, 64);
        q += __shfl_xor(q, 2, 64);
        q += __shfl_xor(q, 4, 64);
        ssq[it] = q;
      }
      GM_LGKM(0);
      __builtin_amdgcn_wave_barrier();
      float* wp = reinterpret_cast<float*>(cw);
      if ((lane & 7) == 0) {
#pragma unroll
        for (int it = 0; it < 16; ++it) wp[it * 8 + (lane >> 3)] = ssq[it];
      }
      __syncthreads();
      const int tiles_n_ = N / GM_BN;
      if (tid < 256) {                             // block row tid: wave row tid / 128, row tid % 128
        const int hw = tid >> 7, rr = tid & 127;
        float sum = 0.f;
#pragma unroll
        for (int c = 0; c < 4; ++c) sum += reinterpret_cast<const float*>(smem + (hw * 4 + c) * 16384)[rr];
        const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
            am.rpart + (size_t)(tm * tiles_n_ + tn) * 256, 0, 256 * 4, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(sum), prs, tid * 4, 0, GM_CPOL_SC1);
      }
      GM_VMCNT(0);
      __syncthreads();
      if (tid == 0)
        *reinterpret_cast<int*>(smem) = __hip_atomic_fetch_add(am.rticket + tm, 1, __ATOMIC_RELAXED,
                                                               __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      const int done = *reinterpret_cast<volatile int*>(smem);
      if (done == tiles_n_ - 1 && tid < 256) {     // the row tile's last block: finish its 256 scales
        float sum = 0.f;
        for (int t2 = 0; t2 < tiles_n_; ++t2) {
          const __amdgpu_buffer_rsrc_t prs = __builtin_amdgcn_make_buffer_rsrc(
              am.rpart + (size_t)(tm * tiles_n_ + t2) * 256, 0, 256 * 4, 0x00020000);
          sum += __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(prs, tid * 4, 0, GM_CPOL_SC1));
        }
        am.rscale[tm * 256 + tid] = rsqrtf(sum / (float)N + am.reps);
        if (tid == 0) __hip_atomic_store(am.rticket + tm, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  } else if (EPI == GM_EPI_SWIGLU) {
    // wave w: 128 rows x 32 features bf16 = 8 KiB at w * 8 KiB
    uint16_t* o = reinterpret_cast<uint16_t*>(smem + w * 8192);
    gm_f32x4 sc[2][4];
    gm_load_row_scales(rs, row0, fq, sc);
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int n = 0; n < 2; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const float g = acc[mh][m][0][n][j] * sc[mh][m][j];
            const float u = acc[mh][m][1][n][j] * sc[mh][m][j];
            const float s = g / (1.0f + __expf(-g));
            o[(mh * 64 + m * 16 + fq * 4 + j) * 32 + n * 16 + fr] = gm_f2bf(s * u);
          }
    GM_LGKM(0);
    __builtin_amdgcn_wave_barrier();
    const int F = N >> 1;
    const int col0 = tn * (GM_BN / 2) + wc * 32;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
      const int qd = it * 64 + lane;               // 16-B chunk: row qd/4, chunk qd%4
      const int r = qd >> 2, cb = qd & 3;
      const int grow = row0 + r;
      const gm_u32x4 v = *reinterpret_cast<const gm_u32x4*>(smem + w * 8192 + r * 64 + cb * 16);
      if (grow < M) *reinterpret_cast<gm_u32x4*>(C + (int64_t)grow * F + col0 + cb * 8) = v;
    }
  } else {
    // wave w: 128 rows x 64 columns bf16 = 16 KiB at w * 16 KiB
    uint16_t* o = reinterpret_cast<uint16_t*>(smem + w * 16384);
    gm_f32x4 sc[2][4];
    gm_load_row_scales(rs, row0, fq, sc);
#pragma unroll
    for (int mh = 0; mh < 2; ++mh)
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int nh = 0; nh < 2; ++nh)
#pragma unroll
          for (int n = 0; n < 2; ++n)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              o[(mh * 64 + m * 16 + fq * 4 + j) * 64 + nh * 32 + n * 16 + fr] =
                  gm_f2bf(acc[mh][m][nh][n][j] * sc[mh][m][j]);
    if (EPI == GM_EPI_STORE) {
      GM_LGKM(0);
      __builtin_amdgcn_wave_barrier();
      const int col0 = tn * GM_BN + wc * 64;
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int qd = it * 64 + lane;               // row qd/8, chunk qd%8
        const int r = qd >> 3, cb = qd & 7;
        const int grow = row0 + r;
        const gm_u32x4 v = *reinterpret_cast<const gm_u32x4*>(smem + w * 16384 + r * 128 + cb * 16);
        if (grow < M) *reinterpret_cast<gm_u32x4*>(C + (int64_t)grow * N + col0 + cb * 8) = v;
      }
    } else {                                       // GM_EPI_ROPE
      __syncthreads();                             // the rotary partner (d + 64) is another wave's column
      // (tile row r, tile column c) -> byte offset of the bf16 element in LDS
      auto at = [&](int r, int c) -> const uint8_t* {
        return smem + ((r >> 7) * 4 + (c >> 6)) * 16384 + (r & 127) * 128 + (c & 63) * 2;
      };
      const int nq = rp.Hq / 2, nk = rp.Hkv / 2;   // 256-column tiles of q / of k heads
      // Every thread keeps one (head, 8-dim chunk) and walks rows r0 + stride*k:
      // all row metadata and rotary factors are loaded up front (independent
      // loads in flight together, not one dependent round trip per row).
      if (tn < nq + nk) {
        const int hh = (tid >> 3) & 1, j = tid & 7, r0 = tid >> 4;   // rows r0 + 32k, k < 8
        int pk[8], sk[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int grow = min(tm * GM_BM + r0 + 32 * k, M - 1);
          pk[k] = rp.pos[grow];
          sk[k] = rp.slot[grow];
        }
        float4 c0[8], c1[8], s0[8], s1[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int64_t o = (int64_t)min(max(pk[k], 0), rp.max_ctx - 1) * 64 + 8 * j;
          c0[k] = *reinterpret_cast<const float4*>(rp.cos_t + o);
          c1[k] = *reinterpret_cast<const float4*>(rp.cos_t + o + 4);
          s0[k] = *reinterpret_cast<const float4*>(rp.sin_t + o);
          s1[k] = *reinterpret_cast<const float4*>(rp.sin_t + o + 4);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const int r = r0 + 32 * k;
          const int grow = tm * GM_BM + r;
          const int p = pk[k], sl = sk[k];
          if (grow >= M || (unsigned)sl >= (unsigned)rp.n_slots || (unsigned)p >= (unsigned)rp.max_ctx) continue;
          const gm_u32x4 lo = *reinterpret_cast<const gm_u32x4*>(at(r, hh * 128 + 8 * j));
          const gm_u32x4 hi = *reinterpret_cast<const gm_u32x4*>(at(r, hh * 128 + 64 + 8 * j));
          const float cc[8] = {c0[k].x, c0[k].y, c0[k].z, c0[k].w, c1[k].x, c1[k].y, c1[k].z, c1[k].w};
          const float ss[8] = {s0[k].x, s0[k].y, s0[k].z, s0[k].w, s1[k].x, s1[k].y, s1[k].z, s1[k].w};
          gm_u32x4 olo, ohi;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a0 = __uint_as_float(lo[e] << 16), a1 = __uint_as_float(lo[e] & 0xffff0000u);
            const float b0 = __uint_as_float(hi[e] << 16), b1 = __uint_as_float(hi[e] & 0xffff0000u);
            const float c_0 = cc[2 * e], c_1 = cc[2 * e + 1], s_0 = ss[2 * e], s_1 = ss[2 * e + 1];
            olo[e] = (uint32_t)gm_f2bf(a0 * c_0 - b0 * s_0) | ((uint32_t)gm_f2bf(a1 * c_1 - b1 * s_1) << 16);
            ohi[e] = (uint32_t)gm_f2bf(b0 * c_0 + a0 * s_0) | ((uint32_t)gm_f2bf(b1 * c_1 + a1 * s_1) << 16);
          }
          uint16_t* dst;
          if (tn < nq) {
            dst = rp.q + (int64_t)grow * rp.Hq * 128 + (2 * tn + hh) * 128;
          } else {
            const int kvh = 2 * (tn - nq) + hh;
            dst = rp.kc + (((int64_t)sl * rp.Hkv + kvh) * rp.max_ctx + p) * 128;
          }
          *reinterpret_cast<gm_u32x4*>(dst + 8 * j) = olo;
          *reinterpret_cast<gm_u32x4*>(dst + 64 + 8 * j) = ohi;
        }
      } else {
        const int hh = (tid >> 4) & 1, cb = tid & 15, r0 = tid >> 5;  // rows r0 + 16k, k < 16
        int pk[16], sk[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int grow = min(tm * GM_BM + r0 + 16 * k, M - 1);
          pk[k] = rp.pos[grow];
          sk[k] = rp.slot[grow];
        }
        const int kvh = 2 * (tn - nq - nk) + hh;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int r = r0 + 16 * k;
          const int grow = tm * GM_BM + r;
          const int p = pk[k], sl = sk[k];
          if (grow >= M || (unsigned)sl >= (unsigned)rp.n_slots || (unsigned)p >= (unsigned)rp.max_ctx) continue;
          uint16_t* dst = rp.vc + (((int64_t)sl * rp.Hkv + kvh) * rp.max_ctx + p) * 128;
          *reinterpret_cast<gm_u32x4*>(dst + 8 * cb) = *reinterpret_cast<const gm_u32x4*>(at(r, hh * 128 + 8 * cb));
        }
      }
    }
  }
  if constexpr (SCHED == 8 || SCHED == 9) {
    const uint64_t st_t1 = __builtin_amdgcn_s_memtime(), st_r1 = __builtin_amdgcn_s_memrealtime();
    if (tid == 0 && am.pv != nullptr) {
      uint64_t* dbg = reinterpret_cast<uint64_t*>(am.pv) + (size_t)bid * 4;
      dbg[0] = st_t0;
      dbg[1] = st_t1;
      dbg[2] = st_r0;
      dbg[3] = st_r1;
    }
  }
}

// PERSIST: the grid (host: at most one block per CU the stream can use, so
// every block is resident -- a split tile's second half may wait for its
// first) walks the block order with stride gridDim.x.  Block b keeps XCD
// b % 8 (gridDim.x % 8 == 0), so the XCD-contiguous tile runs are unchanged;
// what changes is that a tile's epilogue stores drain while the same block
// issues the next tile's prologue DMA, instead of the CU idling between a
// block's exit and the next block's first loads.
template <int EPI, bool STAGGER = true, int SCHED = 2, bool PERSIST = false>
__global__ __launch_bounds__(GM_THREADS) void gemm_bf16_kernel(
    const uint16_t* __restrict__ A, const uint16_t* __restrict__ W, uint16_t* __restrict__ C,
    int M, int N, int K, int group_m, const float* __restrict__ rs, const GmRope rp, const GmSplit sp,
    const GmSide am) {
  extern __shared__ __align__(16) uint8_t smem[];
  if constexpr (PERSIST) {
    const int tiles = ((M + GM_BM - 1) / GM_BM) * (N / GM_BN);
    const int nb = sp.ws ? sp.full + 2 * (tiles - sp.full) : tiles;
    for (int vb = blockIdx.x; vb < nb; vb += gridDim.x) {
      gemm_tile<EPI, STAGGER, SCHED>(smem, A, W, C, M, N, K, group_m, rs, rp, sp, am, vb);
      __syncthreads();                             // the tile's LDS reads retire before the next DMA
    }
  } else {
    gemm_tile<EPI, STAGGER, SCHED>(smem, A, W, C, M, N, K, group_m, rs, rp, sp, am, (int)blockIdx.x);
  }
}


// out[row] = column of the first maximum over the tiles' partials (one wave per row)
__global__ __launch_bounds__(256) void gemm_argmax_reduce_kernel(const float* __restrict__ pv,
                                                                 const int32_t* __restrict__ pi, int M, int tiles,
                                                                 int32_t* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= M) return;
  float v = -__builtin_inff();
  int c = 0x7fffffff;
  for (int t = lane; t < tiles; t += 64) {         // ascending tiles: a later equal value never wins
    const float x = pv[(int64_t)row * tiles + t];
    if (x > v) { v = x; c = pi[(int64_t)row * tiles + t]; }
  }
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const float ov = __shfl_xor(v, off, 64);
    const int oc = __shfl_xor(c, off, 64);
    if (ov > v || (ov == v && oc < c)) { v = ov; c = oc; }
  }
  if (lane == 0) out[row] = c == 0x7fffffff ? 0 : c;   // all-NaN row: token 0
}

#undef GM_STAGE
#undef GM_READ_A
#undef GM_READ_B
#undef GM_MFMA
#undef GM_READ_B0_INTO
#undef GM_MFMA_WITH
#undef GM_LGKM
#undef GM_VMCNT
#undef GM_BARRIER
#undef GM_FENCE

}  // namespace llmq
