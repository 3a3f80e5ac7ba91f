// Where does the gate/up GEMM's time go on a power-bound MI355X?  A/B of the
// production 8-wave kernel (SCHED 2) against diagnostic builds of the same
// template that drop one kind of work from the steady-state K loop while
// keeping every MFMA (numerics are WRONG for 5-7; timing only):
//
//   2  production
//   5  A fragment reads of phases 3 / 7 skipped: one third fewer LDS read
//      bytes -- what a 128 x 128 wave tile (4 waves) would read per MFMA
//   6  no fragment reads in the loop (MFMA + staging DMA only)
//   7  no staging DMA in the loop (MFMA + LDS fragment reads only)
//   8 / 9  2 / 7 with entry and exit clock stamps: the in-kernel shader
//      clock, unprofiled
//   10 every block stages tile (0, 0)'s panels: staging served from L2
//      (what better L2 reuse could be worth at most)
//
// If 5 or 6 run much faster, LDS read traffic (its issue time or its energy
// under the power cap) limits the kernel and a bigger wave tile pays; if only
// 7 does, it is the L2 / HBM side.  Interleaved rounds in one process,
// random operands (cdna_hip_programming.md §5.4 rules 24 / 25).
//
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -I csrc bench/gemm_energy_diag.hip -o /tmp/gemm_energy_diag
//   /tmp/gemm_energy_diag [M N K rounds warm_ms]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "kernels/gemm_kernels.h"

using namespace llmq;

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

// approximately N(0, scale^2) bf16 from a counter hash (sum of 4 uniforms)
__global__ void fill_bf16(uint16_t* p, size_t n, uint32_t seed, float scale) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    uint32_t h = (uint32_t)i * 2654435761u ^ seed;
    float s = 0.f;
    for (int k = 0; k < 4; ++k) {
      h ^= h >> 16; h *= 0x7feb352du; h ^= h >> 15; h *= 0x846ca68bu; h ^= h >> 16;
      s += (float)(h >> 8) * (1.0f / 16777216.0f);
    }
    const float v = (s - 2.0f) * 1.7320508f * scale;  // var of the sum of 4 U(0,1) = 1/3
    uint32_t u = __float_as_uint(v);
    p[i] = (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
  }
}

template <int SCHED>
static void launch(const uint16_t* a, const uint16_t* w, uint16_t* c, int M, int N, int K,
                   uint64_t* dbg = nullptr) {
  static bool attr = false;
  if (!attr) {
    CK(hipFuncSetAttribute((const void*)gemm_bf16_kernel<GM_EPI_SWIGLU, true, SCHED>,
                           hipFuncAttributeMaxDynamicSharedMemorySize, GM_LDS_BYTES));
    attr = true;
  }
  const int tiles = ((M + GM_BM - 1) / GM_BM) * (N / GM_BN);
  hipLaunchKernelGGL((gemm_bf16_kernel<GM_EPI_SWIGLU, true, SCHED>), dim3(tiles), dim3(GM_THREADS), GM_LDS_BYTES, 0,
                     a, w, c, M, N, K, GM_GROUP_M, nullptr, GmRope{}, GmSplit{0, nullptr, nullptr},
                     GmSide{reinterpret_cast<float*>(dbg), nullptr});
}

int main(int argc, char** argv) {
  const int M = argc > 1 ? atoi(argv[1]) : 4096;
  const int N = argc > 2 ? atoi(argv[2]) : 28672;
  const int K = argc > 3 ? atoi(argv[3]) : 4096;
  const int rounds = argc > 4 ? atoi(argv[4]) : 9;
  const float warm_ms = argc > 5 ? (float)atof(argv[5]) : 2500.f;   // 0 under a PMC pass
  const int iters = 10;
  if (N % GM_BN || K % (2 * GM_BK) || M <= 0) {
    fprintf(stderr, "shape: N %% 256, K %% 128\n");
    return 2;
  }
  uint16_t *a, *w, *c;
  CK(hipMalloc(&a, (size_t)M * K * 2));
  CK(hipMalloc(&w, (size_t)N * K * 2));
  CK(hipMalloc(&c, (size_t)M * (N / 2) * 2));
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, a, (size_t)M * K, 1u, 1.0f);
  hipLaunchKernelGGL(fill_bf16, dim3(4096), dim3(256), 0, 0, w, (size_t)N * K, 2u, 0.02f);
  CK(hipDeviceSynchronize());

  const int NV = 5;
  const int scheds[NV] = {2, 5, 6, 7, 10};
  auto run = [&](int s) {
    switch (s) {
      case 2: launch<2>(a, w, c, M, N, K); break;
      case 5: launch<5>(a, w, c, M, N, K); break;
      case 6: launch<6>(a, w, c, M, N, K); break;
      case 7: launch<7>(a, w, c, M, N, K); break;
      default: launch<10>(a, w, c, M, N, K); break;
    }
  };
  // ~2 s of back-to-back launches first so the clock has settled (DVFS give-back)
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int i = 0; warm_ms > 0.f && i < 3000; ++i) {
    run(2);
    if (i % 100 == 99) {
      CK(hipDeviceSynchronize());
      float ms = 0;
      CK(hipEventRecord(e0));
      run(2);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms * (i + 1) > warm_ms) break;
    }
  }
  CK(hipDeviceSynchronize());
  std::vector<std::vector<float>> t(NV);
  for (int r = 0; r < rounds; ++r)
    for (int v = 0; v < NV; ++v) {
      run(scheds[v]);
      CK(hipEventRecord(e0));
      for (int i = 0; i < iters; ++i) run(scheds[v]);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[v].push_back(ms / iters);
    }
  const double flop = 2.0 * M * (double)N * K;
  for (int v = 0; v < NV; ++v) {
    std::sort(t[v].begin(), t[v].end());
    const float med = t[v][t[v].size() / 2];
    printf("{\"sched\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"ms_median\": %.4f, \"ms_min\": %.4f, \"tflops\": %.1f}\n",
           scheds[v], M, N, K, med, t[v][0], flop / med / 1e9);
  }
  // In-kernel clock, unprofiled: the production schedule (8) and the
  // no-DMA build (9) with entry / exit stamps, each after 1 s of its own
  // back-to-back launches; median over the last launch's blocks.
  const int tiles = ((M + GM_BM - 1) / GM_BM) * (N / GM_BN);
  uint64_t* dbg;
  CK(hipMalloc(&dbg, (size_t)tiles * 4 * sizeof(uint64_t)));
  for (int sv : {8, 9}) {
    auto go = [&]() { if (sv == 8) launch<8>(a, w, c, M, N, K, dbg); else launch<9>(a, w, c, M, N, K, dbg); };
    CK(hipEventRecord(e0));
    int n = 0;
    for (;; ++n) {
      go();
      if (n % 50 == 49) {
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms > 1000.f) break;
      }
    }
    CK(hipMemset(dbg, 0, (size_t)tiles * 4 * sizeof(uint64_t)));
    go();
    CK(hipDeviceSynchronize());
    std::vector<uint64_t> h((size_t)tiles * 4);
    CK(hipMemcpy(h.data(), dbg, h.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    for (int b = 0; b < tiles; ++b) {
      const double dt = (double)(h[b * 4 + 1] - h[b * 4 + 0]), dr = (double)(h[b * 4 + 3] - h[b * 4 + 2]);
      if (dr > 0) ghz.push_back(dt / dr * 0.1);             // memrealtime ticks at 100 MHz
    }
    std::sort(ghz.begin(), ghz.end());
    if (!ghz.empty())
      printf("{\"sched\": %d, \"M\": %d, \"N\": %d, \"K\": %d, \"clock_ghz_median\": %.3f, \"clock_ghz_p10\": %.3f, "
             "\"clock_ghz_p90\": %.3f, \"blocks\": %zu, \"warm_launches\": %d}\n",
             sv, M, N, K, ghz[ghz.size() / 2], ghz[ghz.size() / 10], ghz[ghz.size() * 9 / 10], ghz.size(), n + 1);
  }
  return 0;
}
