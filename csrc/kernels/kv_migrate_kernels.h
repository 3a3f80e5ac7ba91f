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
// Grid: one 256-thread workgroup per (layer, k|v, kv head) run: 32 x 2 x 8 =
// 512 workgroups for Llama-3-8B (two per CU on 256 CUs), 16-byte vector
// loads/stores, a pure HBM stream (n = 512 tokens: 64 MiB moved per launch).
// The per-layer base pointers come from a device table [2 L] (k0..kL-1,
// v0..vL-1) built once by the migrator.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace llmq {

template <bool PACK>
__global__ __launch_bounds__(256) void kv_move_kernel(const uint64_t* __restrict__ table, int layers, int slot,
                                                      int n, int max_ctx, int hkv, uint4* __restrict__ buf) {
  const int seg = blockIdx.x;                // ((layer * 2 + kv) * hkv + h)
  const int h = seg % hkv;
  const int lk = seg / hkv;
  const int layer = lk >> 1, kv = lk & 1;
  uint4* cache = reinterpret_cast<uint4*>(table[kv * layers + layer]);
  // 128 bf16 per position = 256 B = 16 uint4
  uint4* c = cache + ((size_t)slot * hkv + h) * (size_t)max_ctx * 16;
  uint4* b = buf + (size_t)seg * (size_t)n * 16;
  const int nv = n * 16;
  for (int i = threadIdx.x; i < nv; i += 256) {
    if (PACK)
      b[i] = c[i];
    else
      c[i] = b[i];
  }
}

}  // namespace llmq
