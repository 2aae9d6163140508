// kara_dev.h — one level of Karatsuba for the 74-limb products of k_rsa_pow
// (x^2, 16 per grant) and k_rsa_final (z * s), one operand pair per lane.
//
// With x = a + 2^(28*37) b (two 37-limb halves, radix 2^28):
//   t = L + 2^(28*37) (M - L - H) + 2^(28*74) H,
//   L = a a', H = b b', M = (a + b)(a' + b')       (a', b' the other operand)
// i.e. three 37 x 37 products (3 x 703 = 2,109 mads for a square instead of
// 2,775; 3 x 1,369 = 4,107 for a product instead of 5,476).  Each product is
// product-scanned with its 64-bit carry chain into normalised 28-bit limbs
// (a + b has 29-bit limbs: a column is < 37 * 2^58 < 2^64), M straight into
// t[37..111], then L and H are subtracted / added in place as they come out
// of their chains -- no limb of L or H is stored, and the combination is left
// unnormalised: t[37..111] are int32 in (-2^29, 2^29) (tests/fold_model.py
// kara_terms asserts the range and the identity).  The fold (fold_dev.h) takes
// such limbs directly: bytes 0..2 biased, byte 3 a signed digit, the low limbs
// 37..72 added into its 64-bit carry chain; FoldKey.cadd carries the matching
// bias and a multiple of n that keeps the result positive (fold.h).
#pragma once
#include "fold.h"
#include "mont.h"

#ifndef MOCHI_KARA_FUSE
#define MOCHI_KARA_FUSE 1
#endif

namespace mochi {

constexpr int kKH = kL / 2;  // 37: the Karatsuba split
static_assert(2 * kKH == kL, "even limb count");
constexpr int kSignedLo = kKH;          // first t limb that may be negative
constexpr int kSignedHi = 3 * kKH + 1;  // one past the last (t[111] = M_74 + H_37 >= 0, but unnormalised)

// Normalised limbs 0..74 of a 37 x 37 product: emit(k, limb) in order.  SQR:
// b is a (cross products once, column doubled).  AO / BO: the halves' offsets.
template <bool SQR, int AO, int BO, int NA, int NB, typename EMIT>
__device__ __forceinline__ void half_product(const uint32_t (&a)[NA], const uint32_t (&b)[NB], EMIT&& emit) {
  uint64_t carry = 0;
  static_for<0, 2 * kKH - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - kKH + 1 > 0 ? k - kKH + 1 : 0;
    uint64_t acc;
    if constexpr (SQR) {
      constexpr int xhi = k > 0 ? (k - 1) / 2 : -1;
      uint64_t xs = 0;
      static_for<lo, xhi + 1>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        xs = mad64(a[AO + i], a[AO + k - i], xs);
      });
      asm("" : "+v"(xs));  // double the column sum once (else hipcc doubles every a_i)
      acc = carry + (xs << 1);  // one v_lshl_add_u64
      if constexpr ((k & 1) == 0) {
#if MOCHI_KARA_FUSE
        asm("" : "+v"(acc));  // keep it fused (else hipcc shifts, mads the square, then adds: one op more)
#endif
        acc = mad64(a[AO + (k >> 1)], a[AO + (k >> 1)], acc);
      }
    } else {
      constexpr int hi = k < kKH - 1 ? k : kKH - 1;
      acc = carry;
      static_for<lo, hi + 1>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        acc = mad64(a[AO + i], b[BO + k - i], acc);
      });
    }
    emit(std::integral_constant<int, k>{}, (uint32_t)acc & kLimbMask);
    carry = acc >> kLimbBits;
    // column by column: left alone the scheduler hoists later columns' mads
    // and keeps dozens of 64-bit column sums live
    __builtin_amdgcn_sched_barrier(0);
  });
  emit(std::integral_constant<int, 2 * kKH - 1>{}, (uint32_t)carry & kLimbMask);
  emit(std::integral_constant<int, 2 * kKH>{}, (uint32_t)(carry >> kLimbBits));
}

// t = x * y (SQR: x * x) as 148 limbs: t[0..36] and t[112..147] normalised,
// t[37..111] signed / unnormalised; t_hi (t[73..147]) leaves with its bytes 0..2
// XOR kFoldBias (the fold's signed B operand), fused where a limb is final.
template <bool SQR>
__device__ __forceinline__ void kara_product(const uint32_t (&x)[kL], const uint32_t (&y)[kL], uint32_t (&t)[2 * kL]) {
  // M = (x_lo + x_hi)(y_lo + y_hi) -> t[37 + k]
  {
    uint32_t sx[kKH];
#pragma unroll
    for (int i = 0; i < kKH; i++) sx[i] = x[i] + x[kKH + i];
    if constexpr (SQR) {
      half_product<true, 0, 0>(sx, sx, [&](auto kc, uint32_t v) { t[kKH + decltype(kc)::value] = v; });
    } else {
      uint32_t sy[kKH];
#pragma unroll
      for (int i = 0; i < kKH; i++) sy[i] = y[i] + y[kKH + i];
      half_product<false, 0, 0>(sx, sy, [&](auto kc, uint32_t v) { t[kKH + decltype(kc)::value] = v; });
    }
  }
  // L = x_lo y_lo: t[k] (+)= L_k, t[37 + k] -= L_k
  half_product<SQR, 0, 0>(x, y, [&](auto kc, uint32_t v) {
    constexpr int k = decltype(kc)::value;
    if constexpr (k < kL) {  // L_74 == 0
      if constexpr (k < kKH) t[k] = v;
      else t[k] += v;
      t[kKH + k] -= v;
    }
  });
  // H = x_hi y_hi: t[37 + m] -= H_m, t[74 + m] (+)= H_m; a t_hi limb is biased
  // once it is final
  half_product<SQR, kKH, kKH>(x, y, [&](auto mc, uint32_t v) {
    constexpr int m = decltype(mc)::value;
    if constexpr (m < kL) {  // H_74 == 0
      t[kKH + m] -= v;
      if constexpr (kKH + m >= kFoldF) t[kKH + m] ^= kFoldBias;  // its last update
      if constexpr (m <= kKH) {
        t[2 * kKH + m] += v;
        if constexpr (m == kKH) t[2 * kKH + m] ^= kFoldBias;  // t[111]: final
      } else {
        t[2 * kKH + m] = v ^ kFoldBias;
      }
    }
  });
}

}  // namespace mochi
