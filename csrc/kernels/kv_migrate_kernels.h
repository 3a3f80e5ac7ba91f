// Conversation KV migration (N11): gather / scatter one conversation's K/V
// rows of EVERY layer between the slot KV cache and one contiguous buffer, in
// a single launch each (the round-2 path issued 2 x 32 copy launches per
// conversation on the compute stream).
//
// Cache layout per layer (llama_kernels.h): [slot][kv_head][max_ctx][128] bf16,
// so the first n positions of one (slot, kv head) are ONE contiguous run of
// n x 256 bytes.  Buffer layout: [layer][k|v][kv_head][n][128] -- the wire
// format RCCL sends between GPUs (llm_message_queue_amd/parallel/migration.py).
//
// Grid: (layer, k|v, kv head) run x 32 KiB chunks of the run: each 256-thread
// workgroup moves KV_UNROLL x 16 B per thread with all KV_UNROLL loads in
// flight before the first store, non-temporal both ways (touched once).  The
// round-4 form (one workgroup per run, a load -> store chain of one 16-byte
// vector per thread per iteration: ~2 MiB in flight chip-wide) moved 4.37
// TB/s beyond the 256 MiB Infinity Cache against a plain copy's 5.04 TB/s
// (profiles/r5_preprocess_kernels_pmc.md); at 512 tokens this grid is 2048
// workgroups with 32 MiB in flight.
// The per-layer base pointers come from a device table [2 L] (k0..kL-1,
// v0..vL-1) built once by the migrator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmq {

constexpr int KV_UNROLL = 8;
constexpr int KV_CHUNK = 256 * KV_UNROLL;   // 16-byte vectors per workgroup
typedef unsigned int kv_u32x4 __attribute__((ext_vector_type(4)));

template <bool PACK>
__global__ __launch_bounds__(256) void kv_move_kernel(const uint64_t* __restrict__ table, int layers, int slot,
                                                      int n, int max_ctx, int hkv, uint4* __restrict__ buf) {
  const int seg = blockIdx.x;                // ((layer * 2 + kv) * hkv + h)
  const int h = seg % hkv;
  const int lk = seg / hkv;
  const int layer = lk >> 1, kv = lk & 1;
  uint4* cache = reinterpret_cast<uint4*>(table[kv * layers + layer]);
  // 128 bf16 per position = 256 B = 16 vectors
  kv_u32x4* c = reinterpret_cast<kv_u32x4*>(cache + ((size_t)slot * hkv + h) * (size_t)max_ctx * 16);
  kv_u32x4* b = reinterpret_cast<kv_u32x4*>(buf + (size_t)seg * (size_t)n * 16);
  const kv_u32x4* src = PACK ? c : b;
  kv_u32x4* dst = PACK ? b : c;
  const int nv = n * 16;
  const int i0 = blockIdx.y * KV_CHUNK + threadIdx.x;
  kv_u32x4 v[KV_UNROLL];
#pragma unroll
  for (int u = 0; u < KV_UNROLL; ++u) {
    const int i = i0 + u * 256;
    if (i < nv) v[u] = __builtin_nontemporal_load(src + i);
  }
#pragma unroll
  for (int u = 0; u < KV_UNROLL; ++u) {
    const int i = i0 + u * 256;
    if (i < nv) __builtin_nontemporal_store(v[u], dst + i);
  }
}

}  // namespace llmq
