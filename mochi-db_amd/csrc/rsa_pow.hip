// rsa_pow.hip — k_rsa_pow: the RSA-2048 squaring chain z = s^(2^16) mod n
// (z < 2^2064, not fully reduced), one signature per lane, with the modular
// reduction on the matrix cores (fold.h):
//
//   per squaring   t = x^2          VALU product scanning, 2,775 v_mad_u64_u32
//                  x = t_lo + W t_hi  v_mfma_i32_32x32x32_i8, 10 M-tiles x 10 K-steps
//                                   x 2 N-tiles (the wave's 64 signatures)
//
// versus 8,251 v_mad_u64_u32 per squaring for a Montgomery squaring on the
// VALU alone (mont.h): the m*n half of Montgomery's work, a product with the
// fixed modulus, becomes a product with a fixed matrix — shared by every
// signature of the signer, so it is GEMM-shaped.
//
// Lanes and MFMA fragments: lane l owns signature l of the wave.  An N-tile is
// 32 signatures, and a 32x32x32 B fragment gives lane l (half h = l >> 5) the
// K slots 16h..16h+15 of column l & 31, so one v_permlane32_swap per operand
// register pair turns "own t_hi limbs 8s+0..3 | 8s+4..7" into the two N-tiles'
// operands; one swap per accumulator pair turns the D fragments (half h = rows
// 4h + 8u + 0..3 = limb 2u + h of the M-tile) back into "own even | own odd".
//
// Group = 512 slots of ONE signer (buckets are 512-aligned), block = 8 waves
// = one group at a time; the signer's 100 KB image is staged in LDS; 2 waves
// per SIMD; persistent blocks, one per CU.
#include "fold_dev.h"
#include "rsa_common.h"

namespace mochi {
namespace {

#ifndef MOCHI_SQR
#define MOCHI_SQR 1
#endif

// column k of x^2: cross products x_i x_{k-i}, i in [sq_lo(k), sq_hi(k)]
constexpr int sq_lo(int k) { return k - kL + 1 > 0 ? k - kL + 1 : 0; }
constexpr int sq_hi(int k) { return k > 0 ? (k - 1) / 2 : -1; }
constexpr int sq_len(int k) { return sq_hi(k) - sq_lo(k) + 1 > 0 ? sq_hi(k) - sq_lo(k) + 1 : 0; }

__device__ __forceinline__ void fold_sqr(uint32_t (&x)[kL], const v4i* __restrict__ wl, cptr cadd) {
  // ---- t = x^2: product scanning, cross products once, column sum doubled ----
  uint32_t t[2 * kL];
#if MOCHI_SQR == 4
  // four columns at a time (four independent accumulation chains)
  {
    uint64_t carry = 0;
    static_for<0, kL / 2 + 1>([&](auto pc) {
      constexpr int kb = 4 * decltype(pc)::value;
      constexpr int nq0 = kb < 2 * kL ? sq_len(kb) : 0, nq1 = kb + 1 < 2 * kL ? sq_len(kb + 1) : 0;
      constexpr int nq2 = kb + 2 < 2 * kL ? sq_len(kb + 2) : 0, nq3 = kb + 3 < 2 * kL ? sq_len(kb + 3) : 0;
      constexpr int nmax = nq0 > nq1 ? (nq0 > nq2 ? (nq0 > nq3 ? nq0 : nq3) : (nq2 > nq3 ? nq2 : nq3))
                                     : (nq1 > nq2 ? (nq1 > nq3 ? nq1 : nq3) : (nq2 > nq3 ? nq2 : nq3));
      uint64_t c[4] = {0, 0, 0, 0};
      static_for<0, nmax>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        static_for<0, 4>([&](auto jc) {
          constexpr int j = decltype(jc)::value, k = kb + j;
          constexpr int n = j == 0 ? nq0 : j == 1 ? nq1 : j == 2 ? nq2 : nq3;
          if constexpr (i < n) c[j] = mad64(x[sq_lo(k) + i], x[k - sq_lo(k) - i], c[j]);
        });
      });
      static_for<0, 4>([&](auto jc) {
        constexpr int j = decltype(jc)::value, k = kb + j;
        if constexpr (k < 2 * kL - 1) {
          asm("" : "+v"(c[j]));
          uint64_t acc = carry + (c[j] << 1);
          if constexpr ((k & 1) == 0) acc = mad64(x[k >> 1], x[k >> 1], acc);
          t[k] = k < kFoldF ? (uint32_t)acc & kLimbMask : ((uint32_t)acc & kLimbMask) ^ 0x80808080u;
          asm volatile("" : "+v"(t[k]));
          carry = acc >> kLimbBits;
        } else if constexpr (k == 2 * kL - 1) {
          t[k] = (uint32_t)carry ^ 0x80808080u;
        }
      });
      __builtin_amdgcn_sched_barrier(0);
    });
  }
#elif MOCHI_SQR == 1
  // two columns at a time: their cross-product chains are independent, so the
  // mads interleave (one accumulation chain per column would issue each mad
  // behind its predecessor's result, and the 64-bit chain result is read by
  // the carry step one wait state later)
  {
    uint64_t carry = 0;
    static_for<0, kL>([&](auto pc) {
      constexpr int k0 = 2 * decltype(pc)::value, k1 = k0 + 1;
      constexpr int n0 = sq_len(k0), n1 = sq_len(k1), nmax = n0 > n1 ? n0 : n1;
      uint64_t c0 = 0, c1 = 0;
      static_for<0, nmax>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i < n0) c0 = mad64(x[sq_lo(k0) + i], x[k0 - sq_lo(k0) - i], c0);
        if constexpr (i < n1) c1 = mad64(x[sq_lo(k1) + i], x[k1 - sq_lo(k1) - i], c1);
      });
      asm("" : "+v"(c0));  // double each column sum once
      asm("" : "+v"(c1));
      uint64_t acc = mad64(x[k0 >> 1], x[k0 >> 1], carry + (c0 << 1));
      t[k0] = k0 < kFoldF ? (uint32_t)acc & kLimbMask : ((uint32_t)acc & kLimbMask) ^ 0x80808080u;
      asm volatile("" : "+v"(t[k0]));
      carry = acc >> kLimbBits;
      if constexpr (k1 < 2 * kL - 1) {
        acc = carry + (c1 << 1);
        t[k1] = k1 < kFoldF ? (uint32_t)acc & kLimbMask : ((uint32_t)acc & kLimbMask) ^ 0x80808080u;
        asm volatile("" : "+v"(t[k1]));
        carry = acc >> kLimbBits;
      } else {
        t[k1] = (uint32_t)carry ^ 0x80808080u;
      }
      __builtin_amdgcn_sched_barrier(0);
    });
  }
#else
  {
    uint64_t carry = 0;
    static_for<0, 2 * kL - 1>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int lo = k - kL + 1 > 0 ? k - kL + 1 : 0;
      constexpr int xhi = k > 0 ? (k - 1) / 2 : -1;
      uint64_t x0 = 0, x1 = 0;
      static_for<lo, xhi + 1>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i & 1) x1 = mad64(x[i], x[k - i], x1);
        else x0 = mad64(x[i], x[k - i], x0);
      });
      uint64_t xs = x0 + x1;
      asm("" : "+v"(xs));  // double the column sum once (else hipcc doubles every x_i: extra mads and registers)
      uint64_t acc = carry + (xs << 1);
      if constexpr ((k & 1) == 0) acc = mad64(x[k >> 1], x[k >> 1], acc);
      // t_hi limbs leave here already biased for the fold's signed B operand
      t[k] = k < kFoldF ? (uint32_t)acc & kLimbMask : ((uint32_t)acc & kLimbMask) ^ 0x80808080u;
      asm volatile("" : "+v"(t[k]));  // materialise the 28-bit limb (else the 64-bit column stays live)
      carry = acc >> kLimbBits;
      // column by column: left alone the scheduler hoists later columns' mads
      // and keeps ~40 64-bit column sums live
      __builtin_amdgcn_sched_barrier(0);
    });
    t[2 * kL - 1] = (uint32_t)carry ^ 0x80808080u;
  }
#endif
  fold_reduce<false, true>(t, x, wl, cadd, nullptr);
}

// Persistent: one block per CU walks a contiguous range of 512-slot groups, so
// the CU never idles between blocks (a block's 8 waves would otherwise all wait
// for its slowest before the next block could take the LDS) and the signer's
// image is staged only when the key changes along the range (block-uniform).
__global__ __launch_bounds__(512, 1) void k_rsa_pow(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                                    const uint8_t* __restrict__ sig,
                                                    const uint16_t* __restrict__ signer,
                                                    const FoldKey* __restrict__ fold, uint32_t* __restrict__ zout) {
  __shared__ v4i w[kFoldImgBytes / 16];
  for_groups(perm, n_slots, signer, fold, w, [&](uint32_t base, uint32_t key, uint32_t g_lead) {
    const uint32_t slot = base + threadIdx.x;
    const uint32_t g = slot < n_slots ? perm[slot] : 0xFFFFFFFFu;
    const bool active = g != 0xFFFFFFFFu;
    if (__ballot(active) == 0) return;  // this wave's quarter of the group is padding
    uint32_t x[kL];
    {
      uint32_t wd[64];
      load_sig_words(sig, active ? g : g_lead, wd);  // inactive lanes shadow the lead grant (never stored)
      words_to_limbs(wd, x);
    }
    const cptr c = as_const(fold[key].cadd);
#pragma unroll 1
    for (int it = 0; it < 16; it++) {
      cptr ci = c;
      asm volatile("" : "+s"(ci));  // keep the 74 cadd loads inside the loop (SGPR pressure if hoisted)
      fold_sqr(x, w + (threadIdx.x & 63), ci);
    }
    if (active) {
#pragma unroll
      for (int j = 0; j < kL; j++) zout[(size_t)j * n_slots + slot] = x[j];
    }
  });
}

}  // namespace

void launch_rsa_pow(const LaunchArgs& a, hipStream_t st) {
  const uint32_t blocks = fold_grid(a.n_slots);
  if (blocks)
    hipLaunchKernelGGL(k_rsa_pow, dim3(blocks), dim3(kBucketAlign), 0, st, a.perm, a.n_slots, a.sig, a.signer, a.fold,
                       a.xbuf);
}

}  // namespace mochi
