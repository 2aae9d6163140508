// rsa_pow.hip — k_rsa_pow: the RSA-2048 squaring chain z = s^(2^16) mod n
// (z < 2^2064, not fully reduced), one signature per lane, with the modular
// reduction on the matrix cores (fold.h):
//
//   per squaring   t = x^2          VALU, one level of Karatsuba over three
//                                   37-limb squares: 2,109 v_mad_u64_u32 (kara_dev.h)
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

// MOCHI_POW_STAMPS (measurement builds only, `make ab`): per wave, s_memtime
// cycles spent in x^2, in the fold, and in the whole kernel, read back with
// mochi_debug_pow_stamps() (scripts/pow_stamps.py)
#ifndef MOCHI_POW_STAMPS
#define MOCHI_POW_STAMPS 0
#endif

namespace mochi {
#if MOCHI_POW_STAMPS
__device__ unsigned long long g_pow_stamps[4096][5];
#endif
namespace {

struct Stamps {
  uint64_t x2 = 0, fold = 0, n = 0, mid = 0;
};

__device__ __forceinline__ uint64_t stamp() {
#if MOCHI_POW_STAMPS
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
#else
  return 0;
#endif
}

__device__ __forceinline__ void fold_sqr(uint32_t (&x)[kL], const v4i* __restrict__ wl, cptr cadd, Stamps& st) {
  uint32_t t[2 * kL];
  const uint64_t t0 = stamp();
#if MOCHI_POW_STAMPS
  {  // kara_square with a stamp after the middle product (M's one chain vs L and H in lockstep)
    uint32_t sx[kKH];
#pragma unroll
    for (int i = 0; i < kKH; i++) sx[i] = x[i] + x[kKH + i];
    kara_middle(t, [&](auto kc, uint64_t& carry) { return square_col<0, decltype(kc)::value>(sx, carry); });
  }
  st.mid += stamp() - t0;
  kara_combine(
      t, [&](auto kc, uint64_t& carry) { return square_col<0, decltype(kc)::value>(x, carry); },
      [&](auto kc, uint64_t& carry) { return square_col<kKH, decltype(kc)::value>(x, carry); });
#else
  kara_square(x, t);  // t = x^2, Karatsuba, t_hi biased (kara_dev.h)
#endif
  const uint64_t t1 = stamp();
  fold_reduce<false, true>(t, x, wl, cadd, nullptr);
  const uint64_t t2 = stamp();
  st.x2 += t1 - t0;
  st.fold += t2 - t1;
  st.n++;
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
  Stamps st;
  const uint64_t t_begin = stamp();
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
      fold_sqr(x, w + (threadIdx.x & 63), ci, st);
    }
    if (active) {
#pragma unroll
      for (int j = 0; j < kL; j++) zout[(size_t)j * n_slots + slot] = x[j];
    }
  });
#if MOCHI_POW_STAMPS
  const uint64_t t_end = stamp();
  const uint32_t wv = blockIdx.x * 8 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && wv < 4096) {
    g_pow_stamps[wv][0] = st.x2;
    g_pow_stamps[wv][1] = st.fold;
    g_pow_stamps[wv][2] = t_end - t_begin;
    g_pow_stamps[wv][3] = st.n;
    g_pow_stamps[wv][4] = st.mid;
  }
#else
  (void)t_begin;
#endif
}

}  // namespace

#if MOCHI_POW_STAMPS
extern "C" int mochi_debug_pow_stamps(unsigned long long* out, unsigned n_waves) {
  if (n_waves > 4096) n_waves = 4096;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pow_stamps), 40 * (size_t)n_waves, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

void launch_rsa_pow(const LaunchArgs& a, hipStream_t st) {
  const uint32_t blocks = fold_grid(a.n_slots);
  if (blocks)
    hipLaunchKernelGGL(k_rsa_pow, dim3(blocks), dim3(kBucketAlign), 0, st, a.perm, a.n_slots, a.sig, a.signer, a.fold,
                       a.xbuf);
}

}  // namespace mochi
