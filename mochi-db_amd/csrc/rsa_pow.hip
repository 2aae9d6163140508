// rsa_pow.hip — k_rsa_pow: the RSA-2048 squaring chain, one signature per lane.
//
//   z = s^(2^16) * R^-(2^16 - 1) mod n   (16 Montgomery squarings of s itself)
//
// The to-Montgomery multiply is folded into k_rsa_final's constant
// K = R^65537 mod n, so this kernel contains only the squaring body
// (8,251 v_mad_u64_u32 per squaring, mont.h) and runs at 3 waves/SIMD.
#include "rsa_common.h"

namespace mochi {

__global__ __launch_bounds__(256, 3) void k_rsa_pow(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                                    const uint8_t* __restrict__ sig,
                                                    const uint16_t* __restrict__ signer,
                                                    const KeyEntry* __restrict__ keys, uint32_t* __restrict__ zout) {
  WaveSlot ws;
  if (!wave_setup(perm, n_slots, signer, ws)) return;
  const KeyEntry* key = keys + ws.s;
  const cptr n = as_const(key->n);
  const uint32_t n0inv = *as_const(&key->n0inv);
  uint32_t x[kL];
  {
    uint32_t w[64];
    load_sig_words(sig, ws.g, w);
    words_to_limbs(w, x);
  }
#pragma unroll 1
  for (int it = 0; it < 16; it++) mont_sqr(x, n, n0inv);
  if (ws.active) {
#pragma unroll
    for (int j = 0; j < kL; j++) zout[(size_t)j * n_slots + ws.slot] = x[j];
  }
}

void launch_rsa_pow(const LaunchArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_rsa_pow, dim3((a.n_slots + 255) / 256), dim3(256), 0, st, a.perm, a.n_slots, a.sig, a.signer,
                     a.keys, a.xbuf);
}

}  // namespace mochi
