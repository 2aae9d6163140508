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

// Column K (0..74) of a 37 x 37 product a * b, normalised; `carry` runs from
// column to column (columns 73 and 74 are the last carry's two limbs).  AO / BO:
// the halves' offsets.
template <int AO, int BO, int K, int NA, int NB>
__device__ __forceinline__ uint32_t product_col(const uint32_t (&a)[NA], const uint32_t (&b)[NB], uint64_t& carry) {
  if constexpr (K == 2 * kKH - 1) {
    return (uint32_t)carry & kLimbMask;
  } else if constexpr (K == 2 * kKH) {
    return (uint32_t)(carry >> kLimbBits);
  } else {
    constexpr int lo = K - kKH + 1 > 0 ? K - kKH + 1 : 0;
    constexpr int hi = K < kKH - 1 ? K : kKH - 1;
    uint64_t acc = carry;
    static_for<lo, hi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      acc = mad64(a[AO + i], b[BO + K - i], acc);
      asm volatile("" ::"v"(acc));  // one chain from the carry (see square_col)
    });
    carry = acc >> kLimbBits;
    return (uint32_t)acc & kLimbMask;
  }
}

// Column K of a 37-limb square, product-scanned with the doubling folded into
// the operands: column k = carry + sum_{i < k-i} (2 a_i) a_{k-i} + a_{k/2}^2,
// one chain of v_mad_u64_u32 with the square term in it (the schoolbook form
// sums the cross products, doubles the sum with a v_lshl_add_u64 and needs an
// asm barrier to keep hipcc from doubling every a_i, whose hazard pads cost
// ~250 s_nop per squaring).  a_m is needed undoubled only up to column 2m (as
// the higher index of a cross product, or squared) and doubled only after it
// (as the lower index), so it is doubled IN PLACE right after column 2m: no
// extra registers, 36 v_lshlrev per square; `a` is clobbered.  Bound: limbs of
// a are < 2^29 (M's a_lo + a_hi), so 2a_i < 2^30, a product < 2^59, and a
// column < 18 * 2^59 + 2^58 + carry (< 2^36) < 2^64 (tests/fold_model.py
// asserts every column).
template <int AO, int K, int NA>
__device__ __forceinline__ uint32_t square_col(uint32_t (&a)[NA], uint64_t& carry) {
  if constexpr (K == 2 * kKH - 1) {
    return (uint32_t)carry & kLimbMask;
  } else if constexpr (K == 2 * kKH) {
    return (uint32_t)(carry >> kLimbBits);
  } else {
    constexpr int lo = K - kKH + 1 > 0 ? K - kKH + 1 : 0;
    constexpr int xhi = K > 0 ? (K - 1) / 2 : -1;
    uint64_t acc = carry;
    static_for<lo, xhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      acc = mad64(a[AO + i], a[AO + K - i], acc);  // a[AO + i] is already 2 a_i
      // every partial sum is an operand of an (empty, input-only) asm: with a
      // second use it cannot be re-associated, so the column stays one chain
      // from the carry -- no v_lshl_add_u64 to add the carry afterwards, and no
      // hazard s_nop (that pad follows asm that DEFINES a register)
      asm volatile("" ::"v"(acc));
    });
    if constexpr ((K & 1) == 0) {
      acc = mad64(a[AO + (K >> 1)], a[AO + (K >> 1)], acc);
      if constexpr ((K >> 1) < kKH - 1) a[AO + (K >> 1)] += a[AO + (K >> 1)];
    }
    carry = acc >> kLimbBits;
    return (uint32_t)acc & kLimbMask;
  }
}

// M = (a_lo + a_hi)(b_lo + b_hi) (`col` gives its columns) straight into
// t[37..111], column by column: left alone the scheduler hoists later columns'
// mads and keeps dozens of 64-bit column sums live.
template <typename COL>
__device__ __forceinline__ void kara_middle(uint32_t (&t)[2 * kL], COL&& col) {
  uint64_t carry = 0;
  static_for<0, 2 * kKH + 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    t[kKH + k] = col(kc, carry);
    __builtin_amdgcn_sched_barrier(0);
  });
}

// The combination t = L + 2^(28*37) (M - L - H) + 2^(28*74) H once M is in
// t[37..111], written with Q = L - 2^(28*37) H as
//     t_k = Q_k + M_(k-37) - Q_(k-37)
// so each Q_k = L_k - H_(k-37) (k = 37..73) is formed once and used twice
// (186 adds instead of 223).  The L chain (`low`) and the H chain (`high`) run
// in lockstep, column c of L beside column c-37 of H -- two independent mad
// chains per step for the scheduler to interleave -- and no limb of either is
// stored.  t_hi (t[73..147]) leaves with its bytes 0..2 XOR kFoldBias (the
// fold's signed B operand), applied where a limb is final.
template <typename LOW, typename HIGH>
__device__ __forceinline__ void kara_combine(uint32_t (&t)[2 * kL], LOW&& low, HIGH&& high) {
  uint64_t cl = 0, ch = 0;
  static_for<0, 3 * kKH>([&](auto cc) {
    constexpr int c = decltype(cc)::value;
    if constexpr (c < kKH) {  // Q_c = L_c
      const uint32_t l = low(cc, cl);
      t[c] = l;
      t[kKH + c] -= l;  // M_c - Q_c
    } else if constexpr (c < kL) {  // Q_c = L_c - H_(c-37)
      const uint32_t l = low(cc, cl);
      const uint32_t h = high(std::integral_constant<int, c - kKH>{}, ch);
      const uint32_t q = l - h;
      t[c] += q;  // final: M_(c-37) - Q_(c-37) + Q_c
      if constexpr (c >= kFoldF) t[c] ^= kFoldBias;
      t[kKH + c] -= q;  // M_c - Q_c
    } else {  // Q_c = -H_(c-37), and t_(c+37) = -Q_c = H_(c-37)
      constexpr int m = c - kKH;
      const uint32_t h = high(std::integral_constant<int, m>{}, ch);
      t[c] -= h;  // final
      t[c] ^= kFoldBias;
      if constexpr (m == kKH) {
        t[kKH + c] += h;  // t[111] = M_74 + H_37: final
        t[kKH + c] ^= kFoldBias;
      } else {
        t[kKH + c] = h ^ kFoldBias;
      }
    }
    __builtin_amdgcn_sched_barrier(0);
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
    kara_middle(t, [&](auto kc, uint64_t& carry) { return square_col<0, decltype(kc)::value>(sx, carry); });
  }
  kara_combine(
      t, [&](auto kc, uint64_t& carry) { return square_col<0, decltype(kc)::value>(x, carry); },
      [&](auto kc, uint64_t& carry) { return square_col<kKH, decltype(kc)::value>(x, carry); });
}

#ifndef MOCHI_KARA2
#define MOCHI_KARA2 0  // A/B (round 6): a second Karatsuba level on x^2's L and H squares
#endif

// Column K of the square of the N limbs a[AO..AO+N) (28- or 29-bit), product-
// scanned exactly like square_col (operands doubled in place after their
// column): K < 2N-1 a column sum, K = 2N-1 and 2N the last carry's two limbs.
template <int AO, int K, int N, int NA>
__device__ __forceinline__ uint32_t square_col_n(uint32_t (&a)[NA], uint64_t& carry) {
  if constexpr (K == 2 * N - 1) {
    return (uint32_t)carry & kLimbMask;
  } else if constexpr (K == 2 * N) {
    return (uint32_t)(carry >> kLimbBits);
  } else {
    constexpr int lo = K - N + 1 > 0 ? K - N + 1 : 0;
    constexpr int xhi = K > 0 ? (K - 1) / 2 : -1;
    uint64_t acc = carry;
    static_for<lo, xhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      acc = mad64(a[AO + i], a[AO + K - i], acc);
      asm volatile("" ::"v"(acc));
    });
    if constexpr ((K & 1) == 0) {
      acc = mad64(a[AO + (K >> 1)], a[AO + (K >> 1)], acc);
      if constexpr ((K >> 1) < N - 1) a[AO + (K >> 1)] += a[AO + (K >> 1)];
    }
    carry = acc >> kLimbBits;
    return (uint32_t)acc & kLimbMask;
  }
}

// The square of the 37 limbs a[AO..AO+37) (28-bit), one more Karatsuba level,
// streamed column by column in order (col<c>() for c = 0..73, normalised):
// A = A0 + B' A1 (A0 19 limbs, A1 18, B' = 2^(28*19)), P0 = A0^2, P1 = A1^2,
// P2 = (A0 + A1)^2 (19 limbs of 29 bits: 190 + 171 + 190 = 551 mads instead of
// 703), and with R = P0 - B' P1,  A^2_c = R_c + P2_(c-19) - R_(c-19): R is kept
// for 19 columns, the three chains advance in step, and a running carry
// normalises the (signed) combination.  `a` is clobbered (doubled in place).
template <int AO, int NA>
struct Square2 {
  static constexpr int N0 = 19, N1 = kKH - N0;  // 19 + 18
  uint32_t (&a)[NA];
  uint32_t s[N0];
  int32_t r[N0];
  uint64_t c0 = 0, c1 = 0, c2 = 0;
  int32_t cn = 0;
  __device__ __forceinline__ explicit Square2(uint32_t (&x)[NA]) : a(x) {
#pragma unroll
    for (int i = 0; i < N0; i++) s[i] = a[AO + i] + (i < N1 ? a[AO + N0 + i] : 0u);
  }
  template <int C>
  __device__ __forceinline__ uint32_t col() {
    int32_t p0 = 0, p1 = 0, p2 = 0;
    if constexpr (C <= 2 * N0) p0 = (int32_t)square_col_n<AO, C, N0>(a, c0);
    if constexpr (C - N0 >= 0 && C - N0 <= 2 * N1) p1 = (int32_t)square_col_n<AO + N0, C - N0, N1>(a, c1);
    if constexpr (C - N0 >= 0 && C - N0 <= 2 * N0) p2 = (int32_t)square_col_n<0, C - N0, N0>(s, c2);
    const int32_t rc = p0 - p1;
    int32_t v = rc + p2 + cn;
    if constexpr (C >= N0) v -= r[C % N0];
    r[C % N0] = rc;
    cn = v >> kLimbBits;  // arithmetic: the combination is signed
    return (uint32_t)v & kLimbMask;
  }
};

// MOCHI_KARA2 == 4: kara_square's lockstep Q-form with L by Square2.
__device__ __forceinline__ void kara_square2_lockstep(uint32_t (&x)[kL], uint32_t (&t)[2 * kL]) {
  {  // M = (x_lo + x_hi)^2 -> t[37 + k]
    uint32_t sx[kKH];
#pragma unroll
    for (int i = 0; i < kKH; i++) sx[i] = x[i] + x[kKH + i];
    kara_middle(t, [&](auto kc, uint64_t& carry) { return square_col<0, decltype(kc)::value>(sx, carry); });
  }
  Square2<0, kL> lo(x);
#if MOCHI_KARA2 == 5  // both L and H by Square2
  Square2<kKH, kL> hi(x);
  kara_combine(
      t, [&](auto kc, uint64_t&) { return lo.template col<decltype(kc)::value>(); },
      [&](auto kc, uint64_t&) { return hi.template col<decltype(kc)::value>(); });
#else
  kara_combine(
      t, [&](auto kc, uint64_t&) { return lo.template col<decltype(kc)::value>(); },
      [&](auto kc, uint64_t& carry) { return square_col<kKH, decltype(kc)::value>(x, carry); });
#endif
}

// kara_square with L and H by Square2, combined directly (t[c] += L_c,
// t[37+c] -= L_c; then t[37+m] -= H_m, t[74+m] += H_m): the same t as
// kara_square's lockstep Q-form, with one inner square's state live at a time.
__device__ __forceinline__ void kara_square2(uint32_t (&x)[kL], uint32_t (&t)[2 * kL]) {
  {  // M = (x_lo + x_hi)^2 -> t[37 + k]
    uint32_t sx[kKH];
#pragma unroll
    for (int i = 0; i < kKH; i++) sx[i] = x[i] + x[kKH + i];
    kara_middle(t, [&](auto kc, uint64_t& carry) { return square_col<0, decltype(kc)::value>(sx, carry); });
  }
  {
#if MOCHI_KARA2 == 3  // (diagnostic) the direct combination with one level for both
    uint64_t cl = 0;
#else
    Square2<0, kL> lo(x);
#endif
    static_for<0, kL>([&](auto cc) {
      constexpr int c = decltype(cc)::value;
#if MOCHI_KARA2 == 3
      const uint32_t l = square_col<0, c>(x, cl);
#else
      const uint32_t l = lo.template col<c>();
#endif
      if constexpr (c < kKH) t[c] = l;
      else t[c] += l;
      t[kKH + c] -= l;
      __builtin_amdgcn_sched_barrier(0);
    });
  }
  {
#if MOCHI_KARA2 >= 2  // the second level for L only (H one level, square_col)
    uint64_t ch = 0;
#else
    Square2<kKH, kL> hi(x);
#endif
    static_for<0, kL>([&](auto mc) {
      constexpr int m = decltype(mc)::value;
#if MOCHI_KARA2 >= 2
      const uint32_t h = square_col<kKH, m>(x, ch);
#else
      const uint32_t h = hi.template col<m>();
#endif
      t[kKH + m] -= h;
      if constexpr (m <= kKH) t[kL + m] += h;
      else t[kL + m] = h;
      __builtin_amdgcn_sched_barrier(0);
    });
  }
#pragma unroll
  for (int k = kFoldF; k < 2 * kL; k++) t[k] ^= kFoldBias;
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
    kara_middle(t, [&](auto kc, uint64_t& carry) { return product_col<0, 0, decltype(kc)::value>(sx, sy, carry); });
  }
  kara_combine(
      t, [&](auto kc, uint64_t& carry) { return product_col<0, 0, decltype(kc)::value>(x, y, carry); },
      [&](auto kc, uint64_t& carry) { return product_col<kKH, kKH, decltype(kc)::value>(x, y, carry); });
}

}  // namespace mochi
