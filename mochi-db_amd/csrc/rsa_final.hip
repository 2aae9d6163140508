// rsa_final.hip — k_rsa_final: finish the RSA-2048 verify and the
// EMSA-PKCS1-v1_5 check (RFC 8017 §8.2.2 / §9.2, "SHA256withRSA") with ONE
// general Montgomery multiply per grant.
//
// k_rsa_pow leaves z = s^(2^16) (mod n), z < 2^2064 = R / 2^8.  Then
//   u = MontMul(z, s) = s^65537 * Q (mod n),   Q = R^-1 mod n,
// u = (z s + m n) / R < (2^-8 + 1) n < 2n.
// The grant is valid iff s < n and s^65537 mod n == EM.  Both sides lie in
// [0, n) (EM < 2^2041 < n), so equality <=> u == EM * Q (mod n).  With
// EM = Cpad + H (Cpad: the fixed padding + DigestInfo, H: the 256-bit digest)
// and the per-key constant A2 = (Cpad * Q mod n) + 2n this is
//   D = A2 + H * Q - u == 0 (mod n),          0 < D < (2^256 + 3) n.
// One short Montgomery reduction by 2^280 (10 limbs) gives
//   D' = (D + m * n) / 2^280,   D' == D * 2^-280 (mod n),   0 < D' < 2n,
// so valid <=> D' == n exactly.  Cost: 10,952 (u) + 740 (H*Q) + 740 (m*n)
// multiply-accumulates instead of two general Montgomery multiplies
// (21,904) plus the final subtraction, and s^65537 mod n is never formed
// (k_rsa_raw in rsa_raw.hip still forms it for mochi_rsa_public_op).
//
// s < n mirrors OpenSSL's RSA_R_DATA_TOO_LARGE_FOR_MODULUS reject.
#include "rsa_common.h"

namespace mochi {

constexpr int kHL = 10;  // digest limbs: 256 bits in radix 2^28

__global__ __launch_bounds__(256, 2) void k_rsa_final(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                                      const uint8_t* __restrict__ sig,
                                                      const uint16_t* __restrict__ signer,
                                                      const KeyEntry* __restrict__ keys,
                                                      const uint32_t* __restrict__ zin,
                                                      const uint32_t* __restrict__ digest, uint32_t n_grants,
                                                      uint8_t* __restrict__ flags) {
  WaveSlot ws;
  if (!wave_setup(perm, n_slots, signer, ws)) return;
  const KeyEntry* key = keys + ws.s;
  const cptr n = as_const(key->n);
  const cptr q = as_const(key->q);
  const cptr a2 = as_const(key->a2);
  const uint32_t n0inv = *as_const(&key->n0inv);
  uint32_t sv[kL], x[kL];
  {
    uint32_t w[64];
    load_sig_words(sig, ws.g, w);
    words_to_limbs(w, sv);
  }
  // s < n on the normalised limbs (borrow chain)
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < kL; j++) br = ((int32_t)sv[j] - (int32_t)n[j] - br) < 0 ? 1 : 0;
  const bool s_lt_n = br != 0;
#pragma unroll
  for (int j = 0; j < kL; j++) x[j] = zin[(size_t)j * n_slots + ws.slot];
  mont_mul<false>(x, x, nullptr, sv, n, n0inv);  // x = u
  // keep the scalar loads of q / a2 below this point: hoisted above the
  // multiply they would sit in SGPRs beside n's 74 limbs and spill
  __asm__ volatile("" ::: "memory");

  // digest H as 10 limbs (digest word 0 = most significant 4 bytes of H)
  uint32_t hl[kHL];
  {
    uint32_t hw[8];
#pragma unroll
    for (int i = 0; i < 8; i++) hw[i] = digest[(size_t)(7 - i) * n_grants + ws.g];
#pragma unroll
    for (int j = 0; j < kHL; j++) {
      const int bit = j * kLimbBits, wi = bit >> 5, sh = bit & 31;
      const uint64_t v = ((uint64_t)(wi + 1 < 8 ? hw[wi + 1] : 0u) << 32) | hw[wi];
      hl[j] = (uint32_t)(v >> sh) & kLimbMask;
    }
  }

  // D' = (A2 + H*Q - u + m*n) / 2^280, product scanning with a signed 64-bit
  // column accumulator (|column| < 2^62), compared with n limb by limb.
  uint32_t m[kHL];
  int64_t carry = 0;
  uint32_t diff = 0;
  static_for<0, kL + kHL - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - (kL - 1) > 0 ? k - (kL - 1) : 0;
    constexpr int hhi = k < kHL - 1 ? k : kHL - 1;
    constexpr int mhi = k < kHL ? k - 1 : kHL - 1;
    uint64_t acc0 = (uint64_t)carry, acc1 = 0;
    if constexpr (k < kL) acc1 = (uint64_t)((int64_t)a2[k] - (int64_t)x[k]);
    static_for<lo, hhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i & 1) acc1 = mad64(hl[i], q[k - i], acc1);
      else acc0 = mad64(hl[i], q[k - i], acc0);
    });
    static_for<lo, mhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i & 1) acc0 = mad64(m[i], n[k - i], acc0);
      else acc1 = mad64(m[i], n[k - i], acc1);
    });
    uint64_t acc = acc0 + acc1;
    if constexpr (k < kHL) {
      const uint32_t mk = ((uint32_t)acc * n0inv) & kLimbMask;
      m[k] = mk;
      acc = mad64(mk, n[0], acc);
    } else {
      diff |= ((uint32_t)acc & kLimbMask) ^ n[k - kHL];
    }
    carry = (int64_t)acc >> kLimbBits;
  });
  diff |= carry != (int64_t)n[kL - 1] ? 1u : 0u;
  if (ws.active) {
    const bool ok = s_lt_n && diff == 0;
    flags[ws.g] = flags[ws.g] | (ok ? MOCHI_GRANT_SIG_OK : 0);
  }
}

void launch_rsa_final(const LaunchArgs& a, hipStream_t st) {
  if (a.dbg_y) {  // mochi_rsa_public_op: materialise s^65537 mod n
    launch_rsa_raw(a, st);
    return;
  }
  hipLaunchKernelGGL(k_rsa_final, dim3((a.n_slots + 255) / 256), dim3(256), 0, st, a.perm, a.n_slots, a.sig,
                     a.signer, a.keys, a.xbuf, a.digest, a.n_grants, a.flags);
}

}  // namespace mochi
