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

namespace mochi {

constexpr int kKH = kL / 2;  // 37: the Karatsuba split
static_assert(2 * kKH == kL, "even limb count");
constexpr int kSignedLo = kKH;          // first t limb that may be negative
constexpr int kSignedHi = 3 * kKH + 1;  // one past the last (t[111] = M_74 + H_37 >= 0, but unnormalised)

// Normalised limbs 0..74 of a 37 x 37 product a * b: emit(k, limb) in order.
// AO / BO: the halves' offsets.
template <int AO, int BO, int NA, int NB, typename EMIT>
__device__ __forceinline__ void half_product(const uint32_t (&a)[NA], const uint32_t (&b)[NB], EMIT&& emit) {
  uint64_t carry = 0;
  static_for<0, 2 * kKH - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - kKH + 1 > 0 ? k - kKH + 1 : 0;
    constexpr int hi = k < kKH - 1 ? k : kKH - 1;
    uint64_t acc = carry;
    static_for<lo, hi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      acc = mad64(a[AO + i], b[BO + k - i], acc);
      asm volatile("" ::"v"(acc));  // one chain from the carry (see half_square)
    });
    emit(std::integral_constant<int, k>{}, (uint32_t)acc & kLimbMask);
    carry = acc >> kLimbBits;
    // column by column: left alone the scheduler hoists later columns' mads
    // and keeps dozens of 64-bit column sums live
    __builtin_amdgcn_sched_barrier(0);
  });
  emit(std::integral_constant<int, 2 * kKH - 1>{}, (uint32_t)carry & kLimbMask);
  emit(std::integral_constant<int, 2 * kKH>{}, (uint32_t)(carry >> kLimbBits));
}

// A 37-limb square, product-scanned with the doubling folded into the
// operands: column k = carry + sum_{i < k-i} (2 a_i) a_{k-i} + a_{k/2}^2, one
// chain of v_mad_u64_u32 with the square term in it (the schoolbook form sums
// the cross products, doubles the sum with a v_lshl_add_u64 and needs an asm
// barrier to keep hipcc from doubling every a_i, whose hazard pads cost ~250
// s_nop per squaring).  a_m is needed undoubled only up to column 2m (as the
// higher index of a cross product, or squared) and doubled only after it (as
// the lower index), so it is doubled IN PLACE right after column 2m: no extra
// registers, 36 v_lshlrev per square; `a` is clobbered.  Bound: limbs of a
// are < 2^29 (M's a_lo + a_hi), so 2a_i < 2^30, a product < 2^59, and a column
// < 18 * 2^59 + 2^58 + carry (< 2^36) < 2^64 (tests/fold_model.py asserts every
// column).
template <int AO, int NA, typename EMIT>
__device__ __forceinline__ void half_square(uint32_t (&a)[NA], EMIT&& emit) {
  uint64_t carry = 0;
  static_for<0, 2 * kKH - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - kKH + 1 > 0 ? k - kKH + 1 : 0;
    constexpr int xhi = k > 0 ? (k - 1) / 2 : -1;
    uint64_t acc = carry;
    static_for<lo, xhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      acc = mad64(a[AO + i], a[AO + k - i], acc);  // a[AO + i] is already 2 a_i
      // every partial sum is an operand of an (empty, input-only) asm: with a
      // second use it cannot be re-associated, so the column stays one chain
      // from the carry -- no v_lshl_add_u64 to add the carry afterwards, and no
      // hazard s_nop (that pad follows asm that DEFINES a register)
      asm volatile("" ::"v"(acc));
    });
    if constexpr ((k & 1) == 0) {
      acc = mad64(a[AO + (k >> 1)], a[AO + (k >> 1)], acc);
      if constexpr ((k >> 1) < kKH - 1) a[AO + (k >> 1)] += a[AO + (k >> 1)];
    }
    emit(std::integral_constant<int, k>{}, (uint32_t)acc & kLimbMask);
    carry = acc >> kLimbBits;
    __builtin_amdgcn_sched_barrier(0);  // column by column (see half_product)
  });
  emit(std::integral_constant<int, 2 * kKH - 1>{}, (uint32_t)carry & kLimbMask);
  emit(std::integral_constant<int, 2 * kKH>{}, (uint32_t)(carry >> kLimbBits));
}

// The combination t = L + 2^(28*37) (M - L - H) + 2^(28*74) H once M is in
// t[37..111]: L's limbs (run by `low`) and H's (run by `high`) are folded in as
// their chains emit them -- no limb of L or H is stored.  t_hi (t[73..147])
// leaves with its bytes 0..2 XOR kFoldBias (the fold's signed B operand),
// applied where a limb is final.
template <typename LOW, typename HIGH>
__device__ __forceinline__ void kara_combine(uint32_t (&t)[2 * kL], LOW&& low, HIGH&& high) {
  low([&](auto kc, uint32_t v) {  // t[k] (+)= L_k, t[37 + k] -= L_k
    constexpr int k = decltype(kc)::value;
    if constexpr (k < kL) {  // L_74 == 0
      if constexpr (k < kKH) t[k] = v;
      else t[k] += v;
      t[kKH + k] -= v;
    }
  });
  high([&](auto mc, uint32_t v) {  // t[37 + m] -= H_m, t[74 + m] (+)= H_m
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

// t = x^2 as 148 limbs (k_rsa_pow): t[0..36] and t[112..147] normalised,
// t[37..111] signed / unnormalised, t_hi biased.  x is clobbered (the fold
// overwrites it next).
__device__ __forceinline__ void kara_square(uint32_t (&x)[kL], uint32_t (&t)[2 * kL]) {
  {  // M = (x_lo + x_hi)^2 -> t[37 + k]
    uint32_t sx[kKH];
#pragma unroll
    for (int i = 0; i < kKH; i++) sx[i] = x[i] + x[kKH + i];
    half_square<0>(sx, [&](auto kc, uint32_t v) { t[kKH + decltype(kc)::value] = v; });
  }
  kara_combine(t, [&](auto&& emit) { half_square<0>(x, emit); }, [&](auto&& emit) { half_square<kKH>(x, emit); });
}

// t = x * y as 148 limbs (k_rsa_final), the same layout as kara_square.
__device__ __forceinline__ void kara_product(const uint32_t (&x)[kL], const uint32_t (&y)[kL], uint32_t (&t)[2 * kL]) {
  {  // M = (x_lo + x_hi)(y_lo + y_hi) -> t[37 + k]
    uint32_t sx[kKH], sy[kKH];
#pragma unroll
    for (int i = 0; i < kKH; i++) {
      sx[i] = x[i] + x[kKH + i];
      sy[i] = y[i] + y[kKH + i];
    }
    half_product<0, 0>(sx, sy, [&](auto kc, uint32_t v) { t[kKH + decltype(kc)::value] = v; });
  }
  kara_combine(t, [&](auto&& emit) { half_product<0, 0>(x, y, emit); },
               [&](auto&& emit) { half_product<kKH, kKH>(x, y, emit); });
}

}  // namespace mochi
