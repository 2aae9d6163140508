// mont.h — RSA-2048 Montgomery arithmetic for gfx950, one signature per lane.
//
// Representation: radix 2^28, L = 74 limbs (2072 bits), R = 2^2072 > 4n, so
// every Montgomery product of inputs < 2n is < 2n and no conditional
// subtraction is needed inside the exponentiation chain (final reduction
// once, in the compare).  Each 28x28 product is < 2^56, so a whole product-
// scanning column (<= 2L-1 = 147 products + the incoming carry) fits a
// 64-bit accumulator with no per-MAC carry handling: every MAC is exactly one
// v_mad_u64_u32 (measured peak ~3.5e13/s on MI355X, microbench/int_peak.hip),
// versus mad + v_addc for 32-bit limbs.
//
// Algorithm: FIPS (Koc et al. "product scanning" Montgomery), columns
// interleave a*b and m*n; the modulus n and R^2 mod n are wave-uniform (the
// verify grid is bucketed by signer) and come from SGPRs via scalar loads.
// Squaring computes each cross product once and doubles the column sum.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace mochi {

constexpr int kLimbBits = 28;
constexpr uint32_t kLimbMask = (1u << kLimbBits) - 1;
constexpr int kL = 74;  // 74 * 28 = 2072 bits

// Per-key device table entry (uploaded once per context).
struct KeyEntry {
  uint32_t n[kL];     // modulus, 28-bit limbs, little-endian limb order
  uint32_t kfix[kL];  // R^2 mod n (R = 2^2072): MontMul(z, kfix) = s^(2^16) R, Montgomery form (k_rsa_raw)
  uint32_t q[kL];     // Q = R^-1 mod n: MontMul(z, s) = s^65537 Q, the verify target is EM * Q (k_rsa_final)
  uint32_t a2[kL];    // (Cpad * Q mod n) + 2n, Cpad = EM with a zero digest (k_rsa_final)
  uint32_t n0inv;     // -n^{-1} mod 2^28
  uint32_t n32[64];   // modulus as 32-bit words, little-endian word order
  uint32_t pad[7];    // 4*74+1+64+7 = 368 words = 1472 bytes
};
static_assert(sizeof(KeyEntry) == 1472, "KeyEntry layout");

// Wave-uniform table reads go through the constant address space so the
// compiler emits scalar loads (SGPR operands for v_mad_u64_u32).
typedef const __attribute__((address_space(4))) uint32_t* cptr;
__device__ __forceinline__ cptr as_const(const uint32_t* p) { return (cptr)(p); }

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
  return (uint64_t)a * b + c;  // v_mad_u64_u32
}

// Compile-time loop: the product-scanning columns must be fully unrolled so
// every limb index is a constant (register-resident arrays, no scratch).
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// r = a * b * R^{-1} mod n  (r < 2n for a, b < 2n).  r may alias a.
// B_UNIFORM: b is a wave-uniform pointer (scalar loads) instead of registers.
template <bool B_UNIFORM>
__device__ __forceinline__ void mont_mul(uint32_t (&r)[kL], const uint32_t (&a)[kL], cptr bu,
                                         const uint32_t (&bv)[kL], cptr n, uint32_t n0inv) {
  uint32_t m[kL];
  uint64_t carry = 0;
  static_for<0, 2 * kL - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - kL + 1 > 0 ? k - kL + 1 : 0;
    constexpr int hi = k < kL - 1 ? k : kL - 1;
    constexpr int mhi = k < kL ? k - 1 : kL - 1;
    uint64_t acc0 = carry, acc1 = 0;
    static_for<lo, hi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      const uint32_t bj = B_UNIFORM ? bu[k - i] : bv[k - i];
      if constexpr (i & 1) acc1 = mad64(a[i], bj, acc1);
      else acc0 = mad64(a[i], bj, acc0);
    });
    static_for<lo, mhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i & 1) acc0 = mad64(m[i], n[k - i], acc0);
      else acc1 = mad64(m[i], n[k - i], acc1);
    });
    uint64_t acc = acc0 + acc1;
    if constexpr (k < kL) {
      const uint32_t mk = ((uint32_t)acc * n0inv) & kLimbMask;
      m[k] = mk;
      acc = mad64(mk, n[0], acc);
      carry = acc >> kLimbBits;
    } else {
      r[k - kL] = (uint32_t)acc & kLimbMask;
      carry = acc >> kLimbBits;
    }
  });
  r[kL - 1] = (uint32_t)carry;
}

// a = a^2 * R^{-1} mod n  (a < 2n).
__device__ __forceinline__ void mont_sqr(uint32_t (&a)[kL], cptr n, uint32_t n0inv) {
  uint32_t m[kL];
  uint64_t carry = 0;
  static_for<0, 2 * kL - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - kL + 1 > 0 ? k - kL + 1 : 0;
    constexpr int mhi = k < kL ? k - 1 : kL - 1;
    constexpr int xhi = k > 0 ? (k - 1) / 2 : -1;  // last i with 2i < k (C++ division truncates: k = 0 has none)
    // cross products a_i * a_{k-i}, i < k - i, counted once then doubled
    uint64_t x0 = 0, x1 = 0;
    static_for<lo, xhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i & 1) x1 = mad64(a[i], a[k - i], x1);
      else x0 = mad64(a[i], a[k - i], x0);
    });
    uint64_t acc0 = carry + ((x0 + x1) << 1), acc1 = 0;
    if constexpr ((k & 1) == 0) acc1 = mad64(a[k >> 1], a[k >> 1], acc1);
    static_for<lo, mhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i & 1) acc0 = mad64(m[i], n[k - i], acc0);
      else acc1 = mad64(m[i], n[k - i], acc1);
    });
    uint64_t acc = acc0 + acc1;
    if constexpr (k < kL) {
      const uint32_t mk = ((uint32_t)acc * n0inv) & kLimbMask;
      m[k] = mk;
      acc = mad64(mk, n[0], acc);
      carry = acc >> kLimbBits;
    } else {
      a[k - kL] = (uint32_t)acc & kLimbMask;
      carry = acc >> kLimbBits;
    }
  });
  a[kL - 1] = (uint32_t)carry;
}

// 64 little-endian 32-bit words -> 74 28-bit limbs.
__device__ __forceinline__ void words_to_limbs(const uint32_t (&w)[64], uint32_t (&x)[kL]) {
#pragma unroll
  for (int j = 0; j < kL; j++) {
    const int bit = j * kLimbBits;
    const int wi = bit >> 5, sh = bit & 31;
    uint32_t lo = wi < 64 ? w[wi] : 0u;
    uint32_t hi = wi + 1 < 64 ? w[wi + 1] : 0u;
    uint64_t v = ((uint64_t)hi << 32) | lo;
    x[j] = (uint32_t)(v >> sh) & kLimbMask;
  }
}

// 74 28-bit limbs (value < 2^2048) -> 64 little-endian 32-bit words.
__device__ __forceinline__ void limbs_to_words(const uint32_t (&x)[kL], uint32_t (&w)[64]) {
#pragma unroll
  for (int i = 0; i < 64; i++) {
    const int bit = i * 32;
    const int j = bit / kLimbBits, sh = bit % kLimbBits;
    // word i = bits [32i, 32i+32) = limbs j, j+1, (j+2)
    uint64_t v = (uint64_t)x[j] >> sh;
    if (j + 1 < kL) v |= (uint64_t)x[j + 1] << (kLimbBits - sh);
    if (j + 2 < kL) v |= (uint64_t)x[j + 2] << (2 * kLimbBits - sh);
    w[i] = (uint32_t)v;
  }
}

}  // namespace mochi
