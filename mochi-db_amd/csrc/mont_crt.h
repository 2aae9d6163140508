// mont_crt.h — Montgomery arithmetic on L-limb (radix 2^28) operands for the
// RSA-CRT signer (rsa_sign.hip): the same product-scanning scheme as mont.h
// (one v_mad_u64_u32 per multiply-accumulate, 64-bit column accumulators, no
// conditional subtraction inside a chain because R = 2^(28L) > 4p), written
// for a generic limb count (L = 37 for the 1024-bit CRT primes).
#pragma once
#include "mont.h"

namespace mochi {

// r = a * b * R^-1 mod p  (r < 2p for a, b < 2p).  r may alias a.
// B_UNIFORM: b is a wave-uniform pointer (scalar loads) instead of registers.
template <int L, bool B_UNIFORM>
__device__ __forceinline__ void mont_mul_n(uint32_t (&r)[L], const uint32_t (&a)[L], cptr bu, const uint32_t (&bv)[L],
                                           cptr n, uint32_t n0inv) {
  uint32_t m[L];
  uint64_t carry = 0;
  static_for<0, 2 * L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - L + 1 > 0 ? k - L + 1 : 0;
    constexpr int hi = k < L - 1 ? k : L - 1;
    constexpr int mhi = k < L ? k - 1 : L - 1;
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
    if constexpr (k < L) {
      const uint32_t mk = ((uint32_t)acc * n0inv) & kLimbMask;
      m[k] = mk;
      acc = mad64(mk, n[0], acc);
      carry = acc >> kLimbBits;
    } else {
      r[k - L] = (uint32_t)acc & kLimbMask;
      carry = acc >> kLimbBits;
    }
  });
  r[L - 1] = (uint32_t)carry;
}

// a = a^2 * R^-1 mod p  (a < 2p).
template <int L>
__device__ __forceinline__ void mont_sqr_n(uint32_t (&a)[L], cptr n, uint32_t n0inv) {
  uint32_t m[L];
  uint64_t carry = 0;
  static_for<0, 2 * L - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - L + 1 > 0 ? k - L + 1 : 0;
    constexpr int mhi = k < L ? k - 1 : L - 1;
    constexpr int xhi = k > 0 ? (k - 1) / 2 : -1;
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
    if constexpr (k < L) {
      const uint32_t mk = ((uint32_t)acc * n0inv) & kLimbMask;
      m[k] = mk;
      acc = mad64(mk, n[0], acc);
      carry = acc >> kLimbBits;
    } else {
      a[k - L] = (uint32_t)acc & kLimbMask;
      carry = acc >> kLimbBits;
    }
  });
  a[L - 1] = (uint32_t)carry;
}

// r = T * R^-1 mod p for a 2L-limb T < R*p given limb by limb by t(k)
// (Montgomery REDC; r < 2p).
template <int L, typename TL>
__device__ __forceinline__ void redc_wide(uint32_t (&r)[L], TL&& t, cptr n, uint32_t n0inv) {
  uint32_t m[L];
  uint64_t carry = 0;
  static_for<0, 2 * L>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - L + 1 > 0 ? k - L + 1 : 0;
    constexpr int mhi = k < L ? k - 1 : L - 1;
    uint64_t acc0 = carry + t(std::integral_constant<int, k>{}), acc1 = 0;
    static_for<lo, mhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i & 1) acc0 = mad64(m[i], n[k - i], acc0);
      else acc1 = mad64(m[i], n[k - i], acc1);
    });
    uint64_t acc = acc0 + acc1;
    if constexpr (k < L) {
      const uint32_t mk = ((uint32_t)acc * n0inv) & kLimbMask;
      m[k] = mk;
      acc = mad64(mk, n[0], acc);
      carry = acc >> kLimbBits;
    } else {
      r[k - L] = (uint32_t)acc & kLimbMask;
      carry = acc >> kLimbBits;
    }
  });
  // T < R*p  =>  result < 2p < 2^(28L): the final carry is zero
}

// [0, 2p) -> [0, p)
template <int L>
__device__ __forceinline__ void reduce_once(uint32_t (&x)[L], cptr n) {
  uint32_t t[L];
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < L; j++) {
    const int32_t d = (int32_t)x[j] - (int32_t)n[j] - br;
    br = d < 0 ? 1 : 0;
    t[j] = (uint32_t)d & kLimbMask;
  }
  const bool ge = br == 0;
#pragma unroll
  for (int j = 0; j < L; j++) x[j] = ge ? t[j] : x[j];
}

}  // namespace mochi
