// rsa_raw.hip — k_rsa_raw: the raw RSA-2048 public operation s^65537 mod n,
// written out per grant.  Serves only mochi_rsa_public_op (the tests pin the
// bignum arithmetic with it); the verify path uses k_rsa_final (rsa_final.hip),
// which never materialises s^65537 mod n.
//
//   w = MontMul(z, K)  = s^(2^16) * R        (z = s^(2^16) from k_rsa_pow, K = R^2 mod n)
//   y = MontMul(w, s)  = s^65537 mod n       (< 2n, reduced once below)
//   valid = s < n  &&  y == 00 01 FF..FF 00 || DigestInfo(SHA-256) || H
//
// s < n mirrors OpenSSL's RSA_R_DATA_TOO_LARGE_FOR_MODULUS reject.
#include "rsa_common.h"

namespace mochi {

// EM as 64 little-endian words: 00 01 FF*202 00 || 30 31 30 0d 06 09 60 86 48
// 01 65 03 04 02 01 05 00 04 20 || H.
__device__ __forceinline__ uint32_t em_word(int i, const uint32_t (&h)[8]) {
  if (i < 8) return h[7 - i];
  switch (i) {
    case 8: return 0x05000420u;   // bytes 220..223
    case 9: return 0x03040201u;   // bytes 216..219
    case 10: return 0x86480165u;  // bytes 212..215
    case 11: return 0x0d060960u;  // bytes 208..211
    case 12: return 0x00303130u;  // bytes 204..207
    case 63: return 0x0001FFFFu;  // bytes 0..3
    default: return 0xFFFFFFFFu;  // PS
  }
}

__global__ __launch_bounds__(256, 2) void k_rsa_raw(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                                      const uint8_t* __restrict__ sig,
                                                      const uint16_t* __restrict__ signer,
                                                      const KeyEntry* __restrict__ keys,
                                                      const uint32_t* __restrict__ zin,
                                                      const uint32_t* __restrict__ digest, uint32_t n_grants,
                                                      uint8_t* __restrict__ flags, uint32_t* __restrict__ dbg_y) {
  WaveSlot ws;
  if (!wave_setup(perm, n_slots, signer, ws)) return;
  const KeyEntry* key = keys + ws.s;
  const cptr n = as_const(key->n);
  const cptr n32 = as_const(key->n32);
  const uint32_t n0inv = *as_const(&key->n0inv);
  uint32_t w[64], sv[kL], x[kL];
  load_sig_words(sig, ws.g, w);
  // s < n (32-bit words, borrow chain)
  uint32_t borrow = 0;
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const uint64_t d = (uint64_t)w[i] - n32[i] - borrow;
    borrow = (uint32_t)(d >> 63);
  }
  const bool s_lt_n = borrow != 0;
  words_to_limbs(w, sv);
#pragma unroll
  for (int j = 0; j < kL; j++) x[j] = zin[(size_t)j * n_slots + ws.slot];
  uint32_t unused[kL];
  mont_mul<true>(x, x, as_const(key->kfix), unused, n, n0inv);
  mont_mul<false>(x, x, nullptr, sv, n, n0inv);
  // reduce [0, 2n) -> [0, n)
  uint32_t t[kL];
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < kL; j++) {
    const int32_t d = (int32_t)x[j] - (int32_t)n[j] - br;
    br = d < 0 ? 1 : 0;
    t[j] = (uint32_t)d & kLimbMask;
  }
  const bool ge = br == 0;
#pragma unroll
  for (int j = 0; j < kL; j++) x[j] = ge ? t[j] : x[j];
  limbs_to_words(x, w);
  uint32_t h[8];
#pragma unroll
  for (int q = 0; q < 8; q++) h[q] = digest[(size_t)q * n_grants + ws.g];
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 64; i++) diff |= w[i] ^ em_word(i, h);
  if (ws.active && dbg_y) {
#pragma unroll
    for (int i = 0; i < 64; i++) dbg_y[(size_t)ws.g * 64 + i] = w[i];
  }
  if (ws.active) {
    const bool ok = s_lt_n && diff == 0;
    flags[ws.g] = flags[ws.g] | (ok ? MOCHI_GRANT_SIG_OK : 0);
  }
}

void launch_rsa_raw(const LaunchArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(k_rsa_raw, dim3((a.n_slots + 255) / 256), dim3(256), 0, st, a.perm, a.n_slots, a.sig,
                     a.signer, a.keys, a.xbuf, a.digest, a.n_grants, a.flags, a.dbg_y);
}

}  // namespace mochi
