// pybind11 bindings for every HIP kernel of llm_message_queue_amd (gfx950).
//
// Python passes raw device pointers (tensor.data_ptr()) plus the HIP stream
// handle (torch.cuda.current_stream().cuda_stream); shapes are re-validated
// here before every launch so a bad call raises instead of faulting the GPU.

#include <hip/hip_runtime.h>

#include <algorithm>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "classify_kernels.h"
#include "gemm_kernels.h"
#include "kv_migrate_kernels.h"
#include "llama_kernels.h"
#include "skinny_kernels.h"
#include "summarise_kernels.h"
#include "text_kernels.h"

namespace py = pybind11;
using namespace llmq;

#define HIP_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(_e));       \
  } while (0)

template <typename T>
static T* P(uintptr_t p) { return reinterpret_cast<T*>(p); }
static hipStream_t S(uintptr_t s) { return reinterpret_cast<hipStream_t>(s); }

static void check_launch() { HIP_CHECK(hipGetLastError()); }

static void require(bool cond, const char* what) {
  if (!cond) throw std::invalid_argument(what);
}

// ---------------------------------------------------------------------- text
static void text_analyze(uintptr_t bytes, uintptr_t offsets, int B, int L, py::bytes table,
                         uintptr_t stats, uintptr_t hashes, uintptr_t stream, uintptr_t zero_rows = 0,
                         int zero_len = 0) {
  require(zero_rows == 0 || (zero_len > 0 && zero_len % 4 == 0 && zero_rows % 16 == 0), "bad zero_rows");
  std::string t = table;
  require(t.size() == sizeof(PatternTable), "pattern table size mismatch");
  require(B >= 0 && L > 0, "bad B/L");
  PatternTable pt;
  std::memcpy(&pt, t.data(), sizeof(pt));
  require(pt.npat >= 0 && pt.npat <= TA_MAX_PAT, "npat out of range");
  for (int j = 0; j < pt.npat; ++j) {
    require(pt.len[j] >= 1 && pt.len[j] <= 16, "pattern length out of range");
    require(pt.slot[j] >= 0 && pt.slot[j] < TA_SLOTS, "pattern slot out of range");
  }
  if (B == 0) return;
  const int grid = (B + TA_WAVES - 1) / TA_WAVES;
  hipLaunchKernelGGL(text_analyze_kernel, dim3(grid), dim3(256), 0, S(stream), P<const uint8_t>(bytes),
                     P<const int64_t>(offsets), B, L, pt, P<int32_t>(stats), P<uint32_t>(hashes),
                     P<float>(zero_rows), zero_len);
  check_launch();
}

static void scan_rows(uintptr_t ntok, int stride, int B, uintptr_t row_off, uintptr_t stream) {
  require(B >= 0 && stride >= 1, "bad scan args");
  hipLaunchKernelGGL(scan_rows_kernel, dim3(1), dim3(1024), 0, S(stream), P<const int32_t>(ntok), stride,
                     B, P<int32_t>(row_off));
  check_launch();
}

static bool g_embed_attr = false;
static constexpr size_t EP_SMEM_BASE = EP_TM * EP_D * 2 + 3 * EP_TM * 4 + 16;
static constexpr size_t EP_SMEM_MAX = 160 * 1024 - 512;   // static __shared__ of the kernel (~280 B) counts too
// largest batch whose row offsets fit in LDS next to the tile (in-block scan)
static constexpr int EP_MAX_LDS_SCAN = (int)((EP_SMEM_MAX - EP_SMEM_BASE) / 4) - 1;
// every block reads all B token counts, so the redundant scan costs
// O(B x blocks) L2 traffic: above this batch size one scan_rows launch is cheaper
static constexpr int EP_IN_BLOCK_SCAN_MAX_B = 2048;

// ntok_src != 0: row_off is not read; every block scans the B token counts
// (ntok_src[i * ntok_stride]) into LDS itself (no scan_rows launch).
static void embed_pool(uintptr_t hashes, int L, uintptr_t row_off, int B, int rows_upper, uintptr_t E,
                       int V, uintptr_t W1t, uintptr_t b1, int H, uintptr_t pooled, uintptr_t stream,
                       uintptr_t ntok_src = 0, int ntok_stride = 0) {
  require(V > 0 && (V & (V - 1)) == 0, "vocab buckets must be a power of two");
  require(H % EP_NCHUNK == 0, "hidden dim must be a multiple of 256");
  require(B >= 0 && rows_upper >= 0, "bad sizes");
  require(ntok_src == 0 || (ntok_stride >= 1 && B <= EP_MAX_LDS_SCAN), "embed_pool: in-block scan bounds");
  require(ntok_src != 0 || row_off != 0, "embed_pool: row_off or ntok_src");
  if (B == 0 || rows_upper == 0) return;
  // + the in-block scan's B + 1 offsets, or the global path's 65-entry window
  const size_t smem = EP_SMEM_BASE + 4 * ((ntok_src ? (size_t)B : (size_t)EP_TM) + 1);
  if (!g_embed_attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)embed_pool_kernel,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)EP_SMEM_MAX));
    g_embed_attr = true;
  }
  const int grid = (rows_upper + EP_TM - 1) / EP_TM * (H / EP_NCHUNK);   // (tile, H chunk) blocks
  hipLaunchKernelGGL(embed_pool_kernel, dim3(grid), dim3(256), smem, S(stream), P<const uint32_t>(hashes),
                     L, P<const int32_t>(row_off), B, P<const uint16_t>(E), (uint32_t)(V - 1),
                     P<const uint16_t>(W1t), P<const float>(b1), H, P<float>(pooled),
                     P<const int32_t>(ntok_src), ntok_stride);
  check_launch();
}

static void classify_head(uintptr_t pooled, int B, int H, uintptr_t W2, uintptr_t b2, uintptr_t logits,
                          uintptr_t pred, uintptr_t stream, const ClassifyReadback& rb = ClassifyReadback{}) {
  require(H % (64 * CH_UNROLL) == 0, "classify_head: hidden dim must be a multiple of 256");
  if (B == 0) return;
  // large batches: 4 messages per wave share each W2 load (L2-bound 88 -> 47 us at 4096);
  // small ones: a message per wave (latency-bound; more waves, shorter chains)
  if (B > 1024)
    hipLaunchKernelGGL(classify_head_kernel<4>, dim3((B + 15) / 16), dim3(256), 0, S(stream), P<const float>(pooled),
                       B, H, P<const float>(W2), P<const float>(b2), P<float>(logits), P<int32_t>(pred), rb);
  else
    hipLaunchKernelGGL(classify_head_kernel<1>, dim3((B + 3) / 4), dim3(256), 0, S(stream), P<const float>(pooled),
                       B, H, P<const float>(W2), P<const float>(b2), P<float>(logits), P<int32_t>(pred), rb);
  check_launch();
}

static void copy_bytes(uintptr_t dst, uintptr_t src, int64_t n, uintptr_t stream);

// The whole GPU preprocess chain of one micro-batch in ONE host call (the
// serve loop's ingest path: one pybind crossing, no per-batch tensor
// allocations, four launches): copy from host-mapped staging, text_analyze
// (zeroing the pooled rows), embed_pool (row scan in LDS per block),
// classify_head with the readback into host-mapped memory riding along
// (without the classifier: one readback kernel).  The caller records the event.
static void text_batch(uintptr_t staging, uintptr_t dev_bytes, int64_t total, int64_t off_offsets, int B, int L,
                       py::bytes table, uintptr_t stats, uintptr_t hashes, bool classify, uintptr_t row_off,
                       int rows_upper, uintptr_t E, int V, uintptr_t W1t, uintptr_t b1, int H, uintptr_t pooled,
                       uintptr_t W2, uintptr_t b2, uintptr_t logits, uintptr_t pred, int cap, uintptr_t rb,
                       int64_t o_pred, int64_t o_ph, uintptr_t stream) {
  require(B > 0 && cap >= 0 && cap <= L, "text_batch: bad B / cap");
  require(off_offsets % 8 == 0 && off_offsets + 8 * (int64_t)(B + 1) <= total, "text_batch: offsets placement");
  require(o_pred >= (int64_t)B * TA_STAT_COLS && o_ph >= o_pred + (classify ? B : 0), "text_batch: readback layout");
  copy_bytes(dev_bytes, staging, total, stream);
  text_analyze(dev_bytes, dev_bytes + off_offsets, B, L, table, stats, hashes, stream, classify ? pooled : 0,
               classify ? H : 0);
  if (classify) {
    if (B <= EP_IN_BLOCK_SCAN_MAX_B && B <= EP_MAX_LDS_SCAN) {
      embed_pool(hashes, L, 0, B, rows_upper, E, V, W1t, b1, H, pooled, stream, stats + 4 * ST_NTOK,
                 TA_STAT_COLS);
    } else {
      scan_rows(stats + 4 * ST_NTOK, TA_STAT_COLS, B, row_off, stream);
      embed_pool(hashes, L, row_off, B, rows_upper, E, V, W1t, b1, H, pooled, stream);
    }
    const ClassifyReadback crb{P<int32_t>(rb), P<const int32_t>(stats), P<const uint32_t>(hashes), TA_STAT_COLS,
                               L, cap, o_pred, o_ph};
    classify_head(pooled, B, H, W2, b2, logits, pred, stream, crb);   // + the readback
    return;
  }
  const int64_t n = (int64_t)B * TA_STAT_COLS + (classify ? B : 0) + (int64_t)B * cap;
  const int blocks = (int)std::min<int64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(text_readback_kernel, dim3(blocks), dim3(256), 0, S(stream), P<const int32_t>(stats),
                     classify ? P<const int32_t>(pred) : nullptr, P<const uint32_t>(hashes), B, L, cap,
                     P<int32_t>(rb), o_pred, o_ph);
  check_launch();
}

// ---------------------------------------------------------------------- summarise
static void summarise_project(uintptr_t pooled, uintptr_t seg_off, int C, uintptr_t Pt, float alpha,
                              uintptr_t state, uintptr_t first_flag, int H, int DS, uintptr_t stream) {
  require(H == SM_H && DS == SM_DS, "summarise expects H=1024, DS=256");
  if (C == 0) return;
  // (16-conversation row block, 64-column block): 4 blocks per 16 conversations
  const dim3 grid((C + SM_ROWS - 1) / SM_ROWS, SM_DS / SM_NB);
  hipLaunchKernelGGL(summarise_project_kernel, grid, dim3(256), 0, S(stream), P<const float>(pooled),
                     P<const int32_t>(seg_off), C,
                     P<const uint16_t>(Pt), alpha, P<float>(state), P<int32_t>(first_flag));
  check_launch();
}

static void salient_topk(uintptr_t hashes, int L, uintptr_t ntok, int stride, uintptr_t seg_off, int C,
                         uintptr_t stop, int nstop, int K, uintptr_t out_hash, uintptr_t out_cnt,
                         uintptr_t out_overflow, uintptr_t stream) {
  require(K >= 0 && K <= 64, "K out of range");
  if (C == 0 || K == 0) return;
  hipLaunchKernelGGL(salient_topk_kernel, dim3(C), dim3(256), 0, S(stream), P<const uint32_t>(hashes), L,
                     P<const int32_t>(ntok), stride, P<const int32_t>(seg_off), P<const uint32_t>(stop),
                     nstop, K, P<uint32_t>(out_hash), P<int32_t>(out_cnt), P<int32_t>(out_overflow));
  check_launch();
}

// ---------------------------------------------------------------------- llama stub
static void rmsnorm(uintptr_t x, uintptr_t res, uintptr_t w, uintptr_t y, int T, int D, float eps,
                    uintptr_t stream) {
  require(D % 2048 == 0 && D >= 2048 && D <= 8192, "rmsnorm expects D in {2048, 4096, 6144, 8192}");
  if (T == 0) return;
  auto kern = D == 2048 ? rmsnorm_kernel<1> : D == 4096 ? rmsnorm_kernel<2> : D == 6144 ? rmsnorm_kernel<3>
                                                                            : rmsnorm_kernel<4>;
  hipLaunchKernelGGL(kern, dim3(T), dim3(256), 0, S(stream), P<const uint16_t>(x),
                     res ? P<uint16_t>(res) : nullptr, P<const uint16_t>(w), P<uint16_t>(y), D, eps);
  check_launch();
}

// C = A · Wᵀ (epi 0, C [M][N]) or H = silu(A·Wgᵀ) * (A·Wuᵀ) over a
// swiglu-permuted W (epi 2, C [M][N/2]); A [M][K], W [N][K], bf16.
// persist_cus > 0: the persistent form (gemm_bf16_kernel PERSIST) on a grid of
// min(blocks, persist_cus) -- persist_cus must not exceed the CUs the stream
// can run on (every block resident; a multiple of 8 keeps blocks on their XCD)
template <int EPI, bool STAGGER = true, int SCHED = 2>
static void launch_gemm(const uint16_t* a, const uint16_t* w, uint16_t* c, int M, int N, int K, hipStream_t st,
                        int group_m, const float* rs = nullptr, const GmRope& rp = GmRope{},
                        const GmSplit& sp = GmSplit{0, nullptr, nullptr},
                        const GmSide& am = GmSide{}, int persist_cus = 0) {
  static bool attr = false, attr_p = false;
  const int tiles = ((M + GM_BM - 1) / GM_BM) * (N / GM_BN);
  const int nb = sp.ws ? sp.full + 2 * (tiles - sp.full) : tiles;
  if (persist_cus > 0 && nb > persist_cus) {
    if (!attr_p) {
      HIP_CHECK(hipFuncSetAttribute((const void*)gemm_bf16_kernel<EPI, STAGGER, SCHED, true>,
                                    hipFuncAttributeMaxDynamicSharedMemorySize, gm_lds_bytes<EPI>()));
      attr_p = true;
    }
    hipLaunchKernelGGL((gemm_bf16_kernel<EPI, STAGGER, SCHED, true>), dim3(persist_cus), dim3(GM_THREADS),
                       gm_lds_bytes<EPI>(), st, a, w, c, M, N, K, group_m, rs, rp, sp, am);
    return;
  }
  if (!attr) {
    HIP_CHECK(hipFuncSetAttribute((const void*)gemm_bf16_kernel<EPI, STAGGER, SCHED>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, gm_lds_bytes<EPI>()));
    attr = true;
  }
  hipLaunchKernelGGL((gemm_bf16_kernel<EPI, STAGGER, SCHED>), dim3(nb), dim3(GM_THREADS), gm_lds_bytes<EPI>(), st,
                     a, w, c,
                     M, N, K, group_m, rs, rp, sp, am);
}

// C += A·Wᵀ (GM_EPI_RESID_RMS = the LDS epilogue) and the RMSNorm scale of the updated rows in
// the same launch: part [tiles_m * tiles_n * 256] fp32, ticket [tiles_m] int
// (zero; the kernel leaves it zero), scale [tiles_m * 256] fp32 (what
// row_rms_kernel writes, rows < M meaningful).
static void gemm_residual_rms(uintptr_t a, uintptr_t w, uintptr_t c, int M, int N, int K, uintptr_t stream,
                              int group_m, uintptr_t part, uintptr_t ticket, uintptr_t scale, float eps) {
  require(group_m >= 1 && group_m <= 64, "gemm: group_m out of range");
  require(M > 0 && N > 0 && K > 0, "gemm: empty operand");
  require(N % GM_BN == 0, "gemm: N must be a multiple of 256");
  require(K % (2 * GM_BK) == 0, "gemm: K must be a multiple of 128");
  require((int64_t)M * K < (int64_t)1 << 30 && (int64_t)N * K < (int64_t)1 << 30 && (int64_t)M * N < (int64_t)1 << 30,
          "gemm: operand too large (2 GiB buffer descriptors)");
  require(a % 16 == 0 && w % 16 == 0 && c % 16 == 0, "gemm: pointers must be 16-byte aligned");
  require(part != 0 && ticket != 0 && scale != 0, "gemm_residual_rms: null workspace");
  GmSide side{};
  side.rpart = P<float>(part);
  side.rticket = P<int>(ticket);
  side.rscale = P<float>(scale);
  side.reps = eps;
  launch_gemm<GM_EPI_RESID_RMS>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream),
                                group_m, nullptr, GmRope{}, GmSplit{0, nullptr, nullptr}, side);
  check_launch();
}

// epi: 0 / 2 / 5 = store / SwiGLU / residual add (C += A·Wᵀ); 16 / 32 = store with the round-1 phase
// schedule / without the wave-row stagger; 50 / 66 / 82 = SwiGLU with
// s_setprio around every MFMA cluster / the static priority on wave row 0 /
// no priority (A/B only; the default is a static priority on wave row 1).
// split_ws != 0: tiles [split_full, tiles) run split-K over two blocks each
// (GmSplit; epilogues store / SwiGLU / residual-LDS): a step too small to
// fill its CUs with whole tiles -- the realtime micro-forwards on their CU
// partition, where o / down are 16 tiles for 32 CUs.
static int device_cus() {
  static int cus[64] = {0};
  int dev = 0;
  HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) return 0;
  if (!cus[dev]) HIP_CHECK(hipDeviceGetAttribute(&cus[dev], hipDeviceAttributeMultiprocessorCount, dev));
  return cus[dev];
}

constexpr int GM_PERSIST_FLAG = 256;   // epi | flag: the persistent grid (one block per CU of the device)

static void gemm_bf16(uintptr_t a, uintptr_t w, uintptr_t c, int M, int N, int K, int epi, uintptr_t stream,
                      int group_m, uintptr_t rs, int split_full, uintptr_t split_ws, uintptr_t split_cnt) {
  const int pc = (epi & GM_PERSIST_FLAG) ? device_cus() & ~7 : 0;
  epi &= ~GM_PERSIST_FLAG;
  require(group_m >= 1 && group_m <= 64, "gemm: group_m out of range");
  require(M > 0 && N > 0 && K > 0, "gemm: empty operand");
  require(N % GM_BN == 0, "gemm: N must be a multiple of 256");
  require(K % (2 * GM_BK) == 0, "gemm: K must be a multiple of 128");
  require((int64_t)M * K < (int64_t)1 << 30 && (int64_t)N * K < (int64_t)1 << 30, "gemm: operand too large (2 GiB buffer descriptors)");
  require(a % 16 == 0 && w % 16 == 0 && c % 16 == 0, "gemm: pointers must be 16-byte aligned");
  const float* rsp = rs ? P<const float>(rs) : nullptr;
  GmSplit sp{0, nullptr, nullptr};
  if (split_ws) {
    const int tiles = ((M + GM_BM - 1) / GM_BM) * (N / GM_BN);
    require(split_full >= 0 && split_full < tiles, "gemm: bad split");
    require((K / GM_BK) % 4 == 0 && K / GM_BK >= 8, "gemm: split-K needs K % 256 == 0 and K >= 512");
    require(split_cnt != 0 && split_ws % 16 == 0, "gemm: split workspace");
    require(epi == GM_EPI_STORE || epi == GM_EPI_SWIGLU || epi == GM_EPI_RESID_LDS, "gemm: split-K epilogue");
    sp = GmSplit{split_full, P<float>(split_ws), P<int>(split_cnt)};
  }
  if (epi == GM_EPI_STORE)
    launch_gemm<GM_EPI_STORE>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream), group_m,
                              rsp, GmRope{}, sp, GmSide{}, pc);
  else if (epi == GM_EPI_SWIGLU)
    launch_gemm<GM_EPI_SWIGLU>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream), group_m,
                               rsp, GmRope{}, sp, GmSide{}, pc);
  else if (epi == GM_EPI_RESID)                    // C += A·Wᵀ in place (no row scales)
    launch_gemm<GM_EPI_RESID>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream), group_m);
  else if (epi == GM_EPI_RESID_LDS)                // the same, residual tile staged by DMA (A/B)
    launch_gemm<GM_EPI_RESID_LDS>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream),
                                  group_m, nullptr, GmRope{}, sp, GmSide{}, pc);
  else if (epi == GM_EPI_RESID_PRE)                // ... with its first quarter prefetched at start (A/B)
    launch_gemm<GM_EPI_RESID_PRE>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream),
                                  group_m);
  else if (epi == GM_EPI_STORE + 16)
    launch_gemm<GM_EPI_STORE, true, 0>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream), group_m);
  else if (epi == GM_EPI_STORE + 32)
    launch_gemm<GM_EPI_STORE, false, 2>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream), group_m);
  else if (epi == GM_EPI_SWIGLU + 48)
    launch_gemm<GM_EPI_SWIGLU, true, 1>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream),
                                        group_m, rsp);
  else if (epi == GM_EPI_SWIGLU + 64)
    launch_gemm<GM_EPI_SWIGLU, true, 3>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream),
                                        group_m, rsp);
  else if (epi == GM_EPI_SWIGLU + 80)
    launch_gemm<GM_EPI_SWIGLU, true, 4>(P<const uint16_t>(a), P<const uint16_t>(w), P<uint16_t>(c), M, N, K, S(stream),
                                        group_m, rsp);
  else
    throw std::invalid_argument("gemm: unknown epilogue");
  check_launch();
}

// q = RoPE(x · Wq^T); K/V cache rows (slot, pos) = (RoPE(x · Wk^T), x · Wv^T):
// the qkv projection with the rope_kv kernel as its epilogue (no [T][qkv]
// intermediate).  W [N][K] in the plain [q | k | v] head order.
static void gemm_qkv_rope(uintptr_t a, uintptr_t w, int M, int N, int K, uintptr_t pos, uintptr_t slot,
                          uintptr_t cos_t, uintptr_t sin_t, int Hq, int Hkv, int max_ctx, int n_slots,
                          uintptr_t q, uintptr_t kc, uintptr_t vc, uintptr_t stream, uintptr_t rs,
                          int split_full, uintptr_t split_ws, uintptr_t split_cnt, int group_m) {
  require(group_m >= 1 && group_m <= 64, "gemm_qkv_rope: group_m");
  require(M > 0 && K > 0, "gemm_qkv_rope: empty operand");
  require(Hq % 2 == 0 && Hkv % 2 == 0 && Hkv >= 2, "gemm_qkv_rope: head counts must be even");
  require(N == (Hq + 2 * Hkv) * 128, "gemm_qkv_rope: N must be (Hq + 2 Hkv) * 128");
  require(K % (2 * GM_BK) == 0, "gemm_qkv_rope: K must be a multiple of 128");
  require((int64_t)M * K < (int64_t)1 << 30 && (int64_t)N * K < (int64_t)1 << 30, "gemm_qkv_rope: operand too large");
  require(a % 16 == 0 && w % 16 == 0 && q % 16 == 0 && kc % 16 == 0 && vc % 16 == 0 && cos_t % 16 == 0 &&
              sin_t % 16 == 0, "gemm_qkv_rope: pointers must be 16-byte aligned");
  require(max_ctx > 0 && n_slots > 0, "gemm_qkv_rope: bad cache shape");
  GmRope rp{P<const int32_t>(pos), P<const int32_t>(slot), P<const float>(cos_t), P<const float>(sin_t),
            P<uint16_t>(q), P<uint16_t>(kc), P<uint16_t>(vc), Hq, Hkv, max_ctx, n_slots};
  GmSplit sp{0, nullptr, nullptr};
  if (split_ws) {
    const int tiles = ((M + GM_BM - 1) / GM_BM) * (N / GM_BN);
    require(split_full >= 0 && split_full < tiles, "gemm_qkv_rope: bad split");
    require((K / GM_BK) % 4 == 0 && K / GM_BK >= 8, "gemm_qkv_rope: split-K needs K % 256 == 0 and K >= 512");
    require(split_cnt != 0 && split_ws % 16 == 0, "gemm_qkv_rope: split workspace");
    sp = GmSplit{split_full, P<float>(split_ws), P<int>(split_cnt)};
  }
  launch_gemm<GM_EPI_ROPE>(P<const uint16_t>(a), P<const uint16_t>(w), nullptr, M, N, K, S(stream), group_m,
                           rs ? P<const float>(rs) : nullptr, rp, sp);
  check_launch();
}

// LM head + greedy sampling: out[m] = argmax_n (A[m] . W[n]) with the argmax
// in the GEMM epilogue (no [M][N] logits); pv / pi: [M][N / 256] scratch.
static void gemm_argmax(uintptr_t a, uintptr_t w, int M, int N, int K, uintptr_t pv, uintptr_t pi,
                        uintptr_t out, uintptr_t stream) {
  require(M > 0 && N % GM_BN == 0 && K % (2 * GM_BK) == 0, "gemm_argmax: M > 0, N % 256, K % 128");
  require((int64_t)M * K < (1LL << 30) && (int64_t)N * K < (1LL << 30), "gemm_argmax: operand > 2 GiB");
  require(a % 16 == 0 && w % 16 == 0 && pv % 4 == 0 && pi % 4 == 0 && out % 4 == 0, "gemm_argmax: alignment");
  launch_gemm<GM_EPI_ARGMAX>(P<const uint16_t>(a), P<const uint16_t>(w), nullptr, M, N, K, S(stream), GM_GROUP_M,
                             nullptr, GmRope{}, GmSplit{0, nullptr, nullptr}, GmSide{P<float>(pv), P<int32_t>(pi)});
  hipLaunchKernelGGL(gemm_argmax_reduce_kernel, dim3((M + 3) / 4), dim3(256), 0, S(stream), P<const float>(pv),
                     P<const int32_t>(pi), M, N / GM_BN, P<int32_t>(out));
  check_launch();
}

static void row_rms(uintptr_t x, uintptr_t r, int T, int D, float eps, uintptr_t stream) {
  require(T >= 0 && D > 0 && D % 512 == 0, "row_rms expects D % 512 == 0");
  require(x % 16 == 0 && r % 4 == 0, "row_rms: misaligned pointers");
  if (T == 0) return;
  hipLaunchKernelGGL(row_rms_kernel, dim3((T + 3) / 4), dim3(256), 0, S(stream), P<const uint16_t>(x), P<float>(r), T,
                     D, eps);
  check_launch();
}

static void silu_mul(uintptr_t gu, uintptr_t out, int T, int F, uintptr_t stream, bool perm) {
  require(F % 8 == 0, "F must be a multiple of 8");
  require(!perm || F % 128 == 0, "permuted silu_mul needs F % 128 == 0");
  const int64_t total = (int64_t)T * F / 8;
  if (total == 0) return;
  hipLaunchKernelGGL(silu_mul_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, S(stream),
                     P<const uint16_t>(gu), P<uint16_t>(out), T, F, perm ? 1 : 0);
  check_launch();
}

static void rope_kv(uintptr_t qkv, uintptr_t pos, uintptr_t slot, uintptr_t cos_t, uintptr_t sin_t, int T,
                    int Hq, int Hkv, int max_ctx, int n_slots, uintptr_t q_out, uintptr_t kc, uintptr_t vc,
                    uintptr_t stream) {
  require(Hq % 4 == 0 && Hkv >= 1, "bad head counts");
  if (T == 0) return;
  hipLaunchKernelGGL(rope_kv_kernel, dim3(T), dim3(256), 0, S(stream), P<const uint16_t>(qkv),
                     P<const int32_t>(pos), P<const int32_t>(slot), P<const float>(cos_t),
                     P<const float>(sin_t), Hq, Hkv, max_ctx, n_slots, P<uint16_t>(q_out), P<uint16_t>(kc),
                     P<uint16_t>(vc));
  check_launch();
}

static void attention(uintptr_t q, uintptr_t kc, uintptr_t vc, uintptr_t pos, uintptr_t slot, int T, int Hq,
                      int Hkv, int max_ctx, int n_slots, float scale, uintptr_t out, uintptr_t stream) {
  require(Hq % Hkv == 0 && Hq / Hkv <= 4, "attention expects a GQA group of <= 4 heads");
  if (T == 0) return;
  hipLaunchKernelGGL(attention_kernel, dim3(T * Hkv), dim3(256), 0, S(stream), P<const uint16_t>(q),
                     P<const uint16_t>(kc), P<const uint16_t>(vc), P<const int32_t>(pos),
                     P<const int32_t>(slot), Hq, Hkv, max_ctx, n_slots, scale, P<uint16_t>(out));
  check_launch();
}

// tiles: int32 [n_tiles][4] = {first token row, n (<= 16), slot, first position}.
// The first n_dec tiles are 1-token decode tiles (wave-per-item decode
// kernel); the rest go to the MFMA segment kernel.  Rows are disjoint.
static void attention_tiles(uintptr_t q, uintptr_t kc, uintptr_t vc, uintptr_t tiles, int n_tiles, int n_dec,
                            int Hq, int Hkv, int max_ctx, int n_slots, int T, float scale, uintptr_t out,
                            uintptr_t stream, int seg_keys, bool mixed) {
  require(seg_keys == 32 || seg_keys == 64, "seg_keys must be 32 or 64");
  require(Hq == 4 * Hkv, "attention_tiles expects a GQA group of exactly 4 heads");
  require(0 <= n_dec && n_dec <= n_tiles, "n_dec out of range");
  const float scale_log2 = scale * 1.4426950408889634f;
  if (mixed && n_dec > 0 && n_tiles > n_dec) {            // both kinds: one launch
    const int seg_blocks = (n_tiles - n_dec) * Hkv;
    const int dec_blocks = (n_dec * Hkv + 3) / 4;
    auto kern = seg_keys == 32 ? attention_mixed_kernel<32> : attention_mixed_kernel<64>;
    hipLaunchKernelGGL(kern, dim3(seg_blocks + dec_blocks), dim3(256), 0, S(stream), P<const uint16_t>(q),
                       P<const uint16_t>(kc), P<const uint16_t>(vc), P<const int32_t>(tiles), n_dec, seg_blocks,
                       Hq, Hkv, max_ctx, n_slots, T, scale_log2, P<uint16_t>(out));
    check_launch();
    return;
  }
  if (n_dec > 0) {
    const int items = n_dec * Hkv;
    hipLaunchKernelGGL(attention_dec_kernel, dim3((items + 3) / 4), dim3(256), 0, S(stream), P<const uint16_t>(q),
                       P<const uint16_t>(kc), P<const uint16_t>(vc), P<const int32_t>(tiles), items, Hq, Hkv,
                       max_ctx, n_slots, T, scale_log2, P<uint16_t>(out));
    check_launch();
  }
  if (n_tiles > n_dec) {
    auto kern = seg_keys == 32 ? attention_seg_kernel<32> : attention_seg_kernel<64>;
    hipLaunchKernelGGL(kern, dim3((n_tiles - n_dec) * Hkv), dim3(256), 0, S(stream),
                       P<const uint16_t>(q), P<const uint16_t>(kc), P<const uint16_t>(vc),
                       P<const int32_t>(tiles) + 4 * n_dec, Hq, Hkv, max_ctx, n_slots, T, scale_log2,
                       P<uint16_t>(out));
    check_launch();
  }
}

// ---------------------------------------------------------------------- N9 slot page
struct MappedPage {
  void* host = nullptr;
  void* dev = nullptr;
};

static py::tuple register_host_page(uintptr_t host_ptr, size_t bytes) {
  HIP_CHECK(hipHostRegister(reinterpret_cast<void*>(host_ptr), bytes, hipHostRegisterMapped));
  void* dev = nullptr;
  HIP_CHECK(hipHostGetDevicePointer(&dev, reinterpret_cast<void*>(host_ptr), 0));
  return py::make_tuple((uintptr_t)host_ptr, (uintptr_t)dev);
}

// device address of pinned host memory (torch pin_memory = hipHostMalloc)
static uintptr_t host_device_ptr(uintptr_t host_ptr) {
  void* dev = nullptr;
  HIP_CHECK(hipHostGetDevicePointer(&dev, reinterpret_cast<void*>(host_ptr), 0));
  return (uintptr_t)dev;
}

// dst/src: device or host-mapped device addresses; both 16-B aligned
static void copy_bytes(uintptr_t dst, uintptr_t src, int64_t n, uintptr_t stream) {
  if (n <= 0) return;
  require((dst % 16) == 0 && (src % 16) == 0, "copy_bytes needs 16-byte aligned pointers");
  const int64_t n16 = n / 16;
  const int blocks = (int)std::min<int64_t>(std::max<int64_t>((n16 + 255) / 256, 1), 1024);
  hipLaunchKernelGGL(copy_bytes_kernel, dim3(blocks), dim3(256), 0, S(stream), P<uint8_t>(dst),
                     P<const uint8_t>(src), n16, n);
  check_launch();
}

static void unregister_host_page(uintptr_t host_ptr) {
  HIP_CHECK(hipHostUnregister(reinterpret_cast<void*>(host_ptr)));
}

static void slot_census(uintptr_t slot_state, int S_, int tokens, uint32_t step, uintptr_t page_dev,
                        uintptr_t stream) {
  hipLaunchKernelGGL(slot_census_kernel, dim3(1), dim3(256), 0, S(stream), P<const int32_t>(slot_state), S_,
                     tokens, step, P<uint32_t>(page_dev));
  check_launch();
}

// ---------------------------------------------------------------------- KV migration
// pack=true: cache rows -> buf; false: buf -> cache rows (see kv_migrate_kernels.h)
static void kv_move(uintptr_t table, int layers, int slots, int slot, int n, int max_ctx, int hkv, int head_dim,
                    uintptr_t buf, bool pack, uintptr_t stream, int variant = KV_LOOP) {
  require(head_dim == 128, "kv_move: head_dim must be 128");
  require(layers > 0 && hkv > 0 && slots > 0, "kv_move: bad cache shape");
  require(slot >= 0 && slot < slots, "kv_move: slot out of range");
  require(n > 0 && n <= max_ctx, "kv_move: token count out of range");
  require(table != 0 && buf != 0 && buf % 16 == 0, "kv_move: null or misaligned buffer");
  require(variant >= KV_LOOP && variant <= KV_CHUNK_NT, "kv_move: unknown variant");
  const int runs = layers * 2 * hkv;
  const dim3 grid(runs, variant == KV_LOOP ? 1 : (n * 16 + KV_CHUNK_VECS - 1) / KV_CHUNK_VECS);
  auto k = pack ? (variant == KV_LOOP ? kv_move_kernel<true, KV_LOOP>
                   : variant == KV_CHUNK ? kv_move_kernel<true, KV_CHUNK> : kv_move_kernel<true, KV_CHUNK_NT>)
                : (variant == KV_LOOP ? kv_move_kernel<false, KV_LOOP>
                   : variant == KV_CHUNK ? kv_move_kernel<false, KV_CHUNK> : kv_move_kernel<false, KV_CHUNK_NT>);
  hipLaunchKernelGGL(k, grid, dim3(256), 0, S(stream), P<const uint64_t>(table), layers, slot, n, max_ctx, hkv,
                     P<uint4>(buf));
  check_launch();
}

// ---------------------------------------------------------------------- skinny GEMM (M <= SK_MAX_M)
// C (+)= A . W^T for the small steps (skinny_kernels.h): split-K partials into
// ws [S][M][N] fp32, then the finalize kernel (row scale, epilogue, bf16).
static void skinny_gemm(uintptr_t a, uintptr_t w, uintptr_t c, int M, int N, int K, int epi, uintptr_t rs,
                        uintptr_t ws, int nsplit, uintptr_t stream) {
  require(M >= 1 && M <= SK_MAX_M, "skinny_gemm: M must be in [1, SK_MAX_M]");
  require(N % SK_NB == 0, "skinny_gemm: N must be a multiple of 128");
  require(nsplit >= 1 && K % (SK_KS * nsplit) == 0, "skinny_gemm: K must be a multiple of 128 * S");
  require(epi == SK_EPI_STORE || epi == SK_EPI_RESID || epi == SK_EPI_SWIGLU, "skinny_gemm: unknown epilogue");
  require(epi != SK_EPI_SWIGLU || N % 256 == 0, "skinny_gemm: SwiGLU needs N % 256 == 0");
  require(a % 16 == 0 && w % 16 == 0 && c % 16 == 0 && ws % 16 == 0 && ws != 0, "skinny_gemm: alignment");
  require((int64_t)N * K < (int64_t)1 << 31, "skinny_gemm: weight too large");
  const int nm = (M + 127) / 128;                   // 128-row chunks of A (M > 128)
  const int mt = nm > 1 ? 8 : (M + 15) / 16;
  const dim3 grid(N / SK_NB * nm, nsplit);
  const int kc = K / nsplit;
  auto* A_ = P<const uint16_t>(a);
  auto* W_ = P<const uint16_t>(w);
  auto* ws_ = P<float>(ws);
#define SK_LAUNCH(T) hipLaunchKernelGGL(skinny_partial_kernel<T>, grid, dim3(256), 0, S(stream), A_, W_, ws_, M, N, K, kc, nm)
  switch (mt) {
    case 1: SK_LAUNCH(1); break;
    case 2: SK_LAUNCH(2); break;
    case 3: SK_LAUNCH(3); break;
    case 4: SK_LAUNCH(4); break;
    case 5: SK_LAUNCH(5); break;
    case 6: SK_LAUNCH(6); break;
    case 7: SK_LAUNCH(7); break;
    default: SK_LAUNCH(8); break;
  }
#undef SK_LAUNCH
  check_launch();
  const int nout = epi == SK_EPI_SWIGLU ? N / 2 : N;
  const int threads = M * (nout / 4);
  const dim3 fgrid((threads + 255) / 256);
  const float* rs_ = rs ? P<const float>(rs) : nullptr;
  auto* C_ = P<uint16_t>(c);
  if (epi == SK_EPI_STORE)
    hipLaunchKernelGGL(skinny_finalize_kernel<SK_EPI_STORE>, fgrid, dim3(256), 0, S(stream), ws_, nsplit, M, N, rs_, C_);
  else if (epi == SK_EPI_RESID)
    hipLaunchKernelGGL(skinny_finalize_kernel<SK_EPI_RESID>, fgrid, dim3(256), 0, S(stream), ws_, nsplit, M, N, rs_, C_);
  else
    hipLaunchKernelGGL(skinny_finalize_kernel<SK_EPI_SWIGLU>, fgrid, dim3(256), 0, S(stream), ws_, nsplit, M, N, rs_, C_);
  check_launch();
}

// ---------------------------------------------------------------------- CU partitions
// Which hardware unit a workgroup ran on: HW_ID (cu / sh / se ids, gfx9
// layout) and XCC_ID, read from the wave's hardware registers by lane 0.
// The spin keeps each workgroup resident for a while so a launch of many
// workgroups spreads over every CU the stream may use.
__global__ void hw_probe_kernel(uint32_t* out, int spin) {
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((4) | (31 << 11));      // HW_REG_HW_ID
    out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((20) | (31 << 11));  // HW_REG_XCC_ID
  }
  float x = (float)threadIdx.x;
  for (int i = 0; i < spin; ++i) x = x * 1.0000001f + 1e-7f;
  if (x == -1.0f) out[0] = 0;                      // (keeps the loop)
}

static std::vector<uint32_t> hw_probe(int blocks, int spin, uintptr_t stream) {
  require(blocks > 0 && blocks <= (1 << 20), "hw_probe: bad block count");
  uint32_t* d = nullptr;
  HIP_CHECK(hipMalloc(&d, sizeof(uint32_t) * 2 * blocks));
  hipLaunchKernelGGL(hw_probe_kernel, dim3(blocks), dim3(64), 0, S(stream), d, spin);
  check_launch();
  HIP_CHECK(hipStreamSynchronize(S(stream)));
  std::vector<uint32_t> h(2 * (size_t)blocks);
  HIP_CHECK(hipMemcpy(h.data(), d, sizeof(uint32_t) * 2 * blocks, hipMemcpyDeviceToHost));
  HIP_CHECK(hipFree(d));
  return h;
}

// A stream whose kernels may only use the CUs set in ``mask`` (32 CUs a
// word, the runtime's CU numbering): the serving steps and the realtime
// micro-forwards each get a partition of the chip.
static uintptr_t stream_with_cu_mask(std::vector<uint32_t> mask) {
  require(!mask.empty(), "stream_with_cu_mask: empty mask");
  hipStream_t s = nullptr;
  HIP_CHECK(hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data()));
  return (uintptr_t)s;
}

static void stream_destroy(uintptr_t s) { HIP_CHECK(hipStreamDestroy(S(s))); }

static py::dict device_info(int dev) {
  hipDeviceProp_t p;
  HIP_CHECK(hipGetDeviceProperties(&p, dev));
  py::dict d;
  d["name"] = std::string(p.name);
  d["gcn_arch"] = std::string(p.gcnArchName);
  d["cus"] = p.multiProcessorCount;
  d["lds_per_cu"] = (int64_t)p.maxSharedMemoryPerMultiProcessor;
  d["lds_per_block"] = (int64_t)p.sharedMemPerBlock;
  d["hbm_bytes"] = (int64_t)p.totalGlobalMem;
  d["clock_khz"] = p.clockRate;
  d["warp_size"] = p.warpSize;
  return d;
}

PYBIND11_MODULE(_hipops, m) {
  m.doc() = "llm_message_queue_amd HIP kernels (gfx950)";
  m.attr("PATTERN_TABLE_BYTES") = (int)sizeof(PatternTable);
  m.attr("MAX_PATTERNS") = TA_MAX_PAT;
  m.attr("STAT_COLS") = TA_STAT_COLS;
  m.attr("SLOTS") = TA_SLOTS;
  m.attr("MAX_TOKEN_BYTES") = TA_MAX_TOKEN_BYTES;
  m.def("text_analyze", &text_analyze, py::arg("bytes"), py::arg("offsets"), py::arg("B"), py::arg("L"),
        py::arg("table"), py::arg("stats"), py::arg("hashes"), py::arg("stream"), py::arg("zero_rows") = 0,
        py::arg("zero_len") = 0);
  m.def("text_batch", &text_batch);
  m.def("scan_rows", &scan_rows);
  m.def("embed_pool", [](uintptr_t hashes, int L, uintptr_t row_off, int B, int rows_upper, uintptr_t E, int V,
                         uintptr_t W1t, uintptr_t b1, int H, uintptr_t pooled, uintptr_t stream, uintptr_t ntok_src,
                         int ntok_stride) {
          embed_pool(hashes, L, row_off, B, rows_upper, E, V, W1t, b1, H, pooled, stream, ntok_src, ntok_stride);
        }, py::arg("hashes"), py::arg("L"), py::arg("row_off"), py::arg("B"), py::arg("rows_upper"), py::arg("E"),
        py::arg("V"), py::arg("W1t"), py::arg("b1"), py::arg("H"), py::arg("pooled"), py::arg("stream"),
        py::arg("ntok_src") = 0, py::arg("ntok_stride") = 0);
  m.def("classify_head", [](uintptr_t pooled, int B, int H, uintptr_t W2, uintptr_t b2, uintptr_t logits,
                            uintptr_t pred, uintptr_t stream) {
    classify_head(pooled, B, H, W2, b2, logits, pred, stream);
  });
  m.attr("EMBED_POOL_MAX_LDS_SCAN") = EP_MAX_LDS_SCAN;
  m.def("summarise_project", &summarise_project);
  m.def("salient_topk", &salient_topk);
  m.def("rmsnorm", &rmsnorm);
  m.def("silu_mul", &silu_mul, py::arg("gu"), py::arg("out"), py::arg("T"), py::arg("F"), py::arg("stream"),
        py::arg("perm") = false);
  m.def("gemm_residual_rms", &gemm_residual_rms, py::arg("a"), py::arg("w"), py::arg("c"), py::arg("M"),
        py::arg("N"), py::arg("K"), py::arg("stream"), py::arg("group_m"), py::arg("part"), py::arg("ticket"),
        py::arg("scale"), py::arg("eps"));
  m.def("gemm_bf16", &gemm_bf16, py::arg("a"), py::arg("w"), py::arg("c"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("epi"), py::arg("stream"), py::arg("group_m") = (int)GM_GROUP_M, py::arg("rs") = 0,
        py::arg("split_full") = 0, py::arg("split_ws") = 0, py::arg("split_cnt") = 0);
  m.def("gemm_qkv_rope", &gemm_qkv_rope, py::arg("a"), py::arg("w"), py::arg("M"), py::arg("N"), py::arg("K"),
        py::arg("pos"), py::arg("slot"), py::arg("cos_t"), py::arg("sin_t"), py::arg("Hq"), py::arg("Hkv"),
        py::arg("max_ctx"), py::arg("n_slots"), py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("stream"),
        py::arg("rs") = 0, py::arg("split_full") = 0, py::arg("split_ws") = 0, py::arg("split_cnt") = 0,
        py::arg("group_m") = GM_GROUP_M);
  m.def("gemm_argmax", &gemm_argmax);
  m.def("row_rms", &row_rms);
  m.attr("GEMM_EPI_STORE") = (int)GM_EPI_STORE;
  m.attr("GEMM_EPI_SWIGLU") = (int)GM_EPI_SWIGLU;
  m.def("rope_kv", &rope_kv);
  m.def("attention", &attention);
  m.def("attention_tiles", &attention_tiles, py::arg("q"), py::arg("kc"), py::arg("vc"), py::arg("tiles"),
        py::arg("n_tiles"), py::arg("n_dec"), py::arg("Hq"), py::arg("Hkv"), py::arg("max_ctx"), py::arg("n_slots"),
        py::arg("T"), py::arg("scale"), py::arg("out"), py::arg("stream"), py::arg("seg_keys"),
        py::arg("mixed") = true);
  m.def("register_host_page", &register_host_page);
  m.def("host_device_ptr", &host_device_ptr);
  m.def("copy_bytes", &copy_bytes);
  m.def("unregister_host_page", &unregister_host_page);
  m.def("slot_census", &slot_census);
  m.def("device_info", &device_info);
  m.def("hw_probe", &hw_probe, py::arg("blocks"), py::arg("spin"), py::arg("stream"));
  m.def("skinny_gemm", &skinny_gemm, py::arg("a"), py::arg("w"), py::arg("c"), py::arg("M"), py::arg("N"),
        py::arg("K"), py::arg("epi"), py::arg("rs"), py::arg("ws"), py::arg("S"), py::arg("stream"));
  m.def("stream_with_cu_mask", &stream_with_cu_mask);
  m.def("stream_destroy", &stream_destroy);
  m.def("kv_move", &kv_move, py::arg("table"), py::arg("layers"), py::arg("slots"), py::arg("slot"), py::arg("n"),
        py::arg("max_ctx"), py::arg("hkv"), py::arg("head_dim"), py::arg("buf"), py::arg("pack"), py::arg("stream"),
        py::arg("variant") = (int)KV_LOOP);
}
