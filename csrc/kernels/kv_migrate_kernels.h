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
// Grid, KV_CHUNK_NT (the migrator's default, round 5): the (layer, k|v, kv
// head) run split into 32 KiB chunks, one per 256-thread workgroup, all 8
// loads of a thread in flight before its first store, non-temporal both ways
// (the bytes are touched once): 5.50 TB/s beyond the 256 MiB Infinity Cache,
// 1.09x a torch copy of the same bytes.  KV_LOOP (round 4): one workgroup per
// run looping over it -- 4.47 TB/s there, though 6.5 TB/s on cache-resident
// buffers.  KV_CHUNK: the chunked form with plain loads / stores.
// Measured in profiles/r5_preprocess_kernels_pmc.md ("kv_move" section).
// The per-layer base pointers come from a device table [2 L] (k0..kL-1,
// v0..vL-1) built once by the migrator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmq {

constexpr int KV_UNROLL = 8;
constexpr int KV_CHUNK_VECS = 256 * KV_UNROLL;   // 16-byte vectors per chunk workgroup
enum { KV_LOOP = 0, KV_CHUNK = 1, KV_CHUNK_NT = 2 };
typedef unsigned int kv_u32x4 __attribute__((ext_vector_type(4)));

template <bool PACK, int MODE>
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
  if (MODE == KV_LOOP) {
    for (int i = threadIdx.x; i < nv; i += 256) dst[i] = src[i];
    return;
  }
  const int i0 = blockIdx.y * KV_CHUNK_VECS + threadIdx.x;
  // loads unconditional (clamped into the run), stores predicated: a
  // predicated load form compiled to a load -> vmcnt(0) chain
  kv_u32x4 v[KV_UNROLL];
#pragma unroll
  for (int u = 0; u < KV_UNROLL; ++u) {
    const int i = min(i0 + u * 256, nv - 1);
    v[u] = MODE == KV_CHUNK_NT ? __builtin_nontemporal_load(src + i) : src[i];
  }
#pragma unroll
  for (int u = 0; u < KV_UNROLL; ++u) {
    const int i = i0 + u * 256;
    if (i < nv) {
      if (MODE == KV_CHUNK_NT) __builtin_nontemporal_store(v[u], dst + i);
      else dst[i] = v[u];
    }
  }
}

}  // namespace llmq
