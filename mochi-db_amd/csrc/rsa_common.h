// rsa_common.h — helpers shared by the two RSA kernels (rsa_pow.hip, rsa_final.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mochi_hip.h"
#include "kernels.h"
#include "mont.h"

namespace mochi {

// Wave setup for the signer-bucketed grid.  Buckets are 64-aligned and padded
// only at their tail, so lane 0 of every non-empty wave is active and all
// active lanes share lane 0's signer (k_bucket_scatter guarantees it).
struct WaveSlot {
  uint32_t slot, g;   // bucket slot / grant index (g valid only when active)
  bool active;
  uint32_t s;         // wave-uniform signer (SGPR)
};

__device__ __forceinline__ bool wave_setup(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                           const uint16_t* __restrict__ signer, WaveSlot& ws) {
  ws.slot = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t g = ws.slot < n_slots ? perm[ws.slot] : 0xFFFFFFFFu;
  ws.active = g != 0xFFFFFFFFu;
  const uint64_t amask = __ballot(ws.active);
  if (amask == 0) return false;
  const int lead = __builtin_ctzll(amask);
  const uint32_t g_lead = __builtin_amdgcn_readlane(g, lead);
  ws.g = ws.active ? g : g_lead;  // inactive lanes shadow the lead grant (never stored)
  ws.s = __builtin_amdgcn_readfirstlane((uint32_t)signer[g_lead]);
  return true;
}

__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// 256 big-endian signature bytes -> 64 little-endian words.
__device__ __forceinline__ void load_sig_words(const uint8_t* __restrict__ sig, uint32_t g, uint32_t (&w)[64]) {
  const uint4* s128 = (const uint4*)(sig + (size_t)g * MOCHI_RSA_BYTES);
#pragma unroll
  for (int q = 0; q < 16; q++) {
    const uint4 v = s128[q];  // big-endian bytes [16q, 16q+16)
    w[63 - 4 * q] = bswap32(v.x);
    w[62 - 4 * q] = bswap32(v.y);
    w[61 - 4 * q] = bswap32(v.z);
    w[60 - 4 * q] = bswap32(v.w);
  }
}

}  // namespace mochi
