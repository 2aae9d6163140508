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
//
// SIMD partners in opposite phases.  Waves w and w + 4 share a SIMD.  A
// squaring is two phases of very different shape -- x^2 is VALU issue (2,109
// 64-bit mads + glue), the fold is the matrix pipe (200 MFMAs x 32 cycles) plus
// a short assembly -- and left free-running the partners' phases fall where
// they may: both in x^2 (VALU saturated, matrix pipe idle) or both in the fold
// (the reverse) much of the time.  So waves 4-7 run one phase behind waves 0-3
// and a block barrier ends every phase: one wave's x^2 always runs beside its
// partner's fold, whose MFMAs (at s_setprio 1, so they issue the moment they
// are ready) co-execute with the x^2's VALU.  33 phases per group (one
// half-empty at each end).  Grant prep is its own kernel (kernels.hip): parse
// and SHA-256 are latency-bound, and in the half-empty phases or the fold's
// VALU gaps here they ran at one wave per SIMD-half, 2-3x slower than the
// k_grant_prep launch they replaced.
#include "fold_dev.h"
#include "rsa_common.h"

#include <cstdlib>

// MOCHI_POW_STAMPS (measurement builds only, `make ab`): per wave, s_memtime
// cycles spent in x^2, in the fold, and in the whole kernel, read back with
// mochi_debug_pow_stamps() (scripts/pow_stamps.py)
#ifndef MOCHI_POW_STAMPS
#define MOCHI_POW_STAMPS 0
#endif
// MOCHI_POW_DYN (default): blocks take 512-slot groups from a device counter
// instead of fixed contiguous ranges, so a CU that starts late or clocks lower
// does fewer groups: k_rsa_pow -1.5 %, C4 +1.4 % (round 5, alternated A/B,
// DESIGN.md section 9); -DMOCHI_POW_DYN=0 builds the static ranges
#ifndef MOCHI_POW_DYN
#define MOCHI_POW_DYN 1
#endif
#ifndef MOCHI_LAT_RAW
#define MOCHI_LAT_RAW 0
#endif
#ifndef MOCHI_LAT_ONE_TILE
#define MOCHI_LAT_ONE_TILE 1  // A/B (0): k_rsa_pow_lat always folds both N-tiles
#endif
#ifndef MOCHI_POW_NEXT_AHEAD
#define MOCHI_POW_NEXT_AHEAD 1  // the next group's index fetched one group ahead (below)
#endif
// MOCHI_LAT_STAMPS (measurement builds only): k_rsa_pow_lat's phases per wave,
// s_memtime cycles summed over the 16 squarings -- squares, barrier 1, combine
// (wave 0) + barrier 2, fold (+ barrier 3), barrier 4, carry chain, barrier 5,
// whole loop -- read back with mochi_debug_lat_stamps() (scripts/lat_stamps.py)
#ifndef MOCHI_LAT_STAMPS
#define MOCHI_LAT_STAMPS 0
#endif
namespace mochi {
#if MOCHI_POW_STAMPS
__device__ unsigned long long g_pow_stamps[4096][5];
#endif
#if MOCHI_LAT_STAMPS
__device__ unsigned long long g_lat_stamps[256][4][8];  // [block][wave][phase]
#endif
namespace {

struct Stamps {
  uint64_t x2 = 0, fold = 0, n = 0;
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

__device__ __forceinline__ uint64_t lstamp() {
#if MOCHI_LAT_STAMPS
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
#else
  return 0;
#endif
}

__device__ __forceinline__ void phase_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
}

struct PowArgs {
  const uint32_t* perm;
  uint32_t n_slots;
  const uint8_t* sig;
  const uint16_t* signer;
  const FoldKey* fold;
  uint32_t* zout;
  uint32_t* ctr;  // MOCHI_POW_DYN group counter
};

// Persistent: one block per CU takes 512-slot groups in order from a device
// counter (or walks a contiguous range), so the CU never idles between blocks
// and the signer's image is staged only when the key changes (block-uniform;
// groups come in bucket order, so that is about once per bucket boundary).
__global__ __launch_bounds__(512, 1) void k_rsa_pow(const PowArgs a) {
  __shared__ v4i w[kFoldImgBytes / 16];
  Stamps st;
  const uint64_t t_begin = stamp();

  // waves 4-7 run one phase behind.  Read through readfirstlane so the compiler
  // KNOWS it is wave-uniform: the barriers below sit under `if (lag)`, and a
  // barrier under a branch it takes for divergent is exec-masked code, into
  // whose join it once hoisted a VALU constant that the masked-off waves never
  // wrote (half the signatures wrong)
  const bool lag = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) >= 4;
  const uint32_t n_groups = (a.n_slots + kBucketAlign - 1) / kBucketAlign;
  uint32_t cur_key = 0xFFFFFFFFu;
#if MOCHI_POW_DYN
  // groups from a device counter (zeroed by k_bucket_scan), double-buffered
  // in LDS.  The next group's index is fetched at the start of this one and
  // published at its end, so the atomic's round trip runs under this group's
  // signature loads instead of stalling every wave at the group boundary.
  __shared__ uint32_t s_grp[2];
  // no more groups than blocks: one each, by index -- with the counter a block
  // that started first could take two groups while another had not started yet
  // (a 2-message batch's pow took 161 or 338 us depending on the dispatch order)
  const bool one_each = n_groups <= gridDim.x;
  if (threadIdx.x == 0) s_grp[0] = one_each ? blockIdx.x : atomicAdd(a.ctr, 1u);
  __syncthreads();
  for (uint32_t it_g = 0;; it_g ^= 1) {
    const uint32_t grp = __builtin_amdgcn_readfirstlane(s_grp[it_g]);
    if (grp >= n_groups) break;
    uint32_t nxt = 0;
    if (threadIdx.x == 0) nxt = one_each ? n_groups : atomicAdd(a.ctr, 1u);
#if !MOCHI_POW_NEXT_AHEAD  // A/B: wait for the fetch here, as every wave did before
    if (threadIdx.x == 0) s_grp[it_g ^ 1] = nxt;
    __syncthreads();
#endif
    // publishes the next index: every path through the group body ends here
    auto publish = [&]() {
      if (MOCHI_POW_NEXT_AHEAD && threadIdx.x == 0) s_grp[it_g ^ 1] = nxt;
      __syncthreads();
    };
#else
  const uint32_t g_begin = (uint32_t)((uint64_t)blockIdx.x * n_groups / gridDim.x);
  const uint32_t g_end = (uint32_t)((uint64_t)(blockIdx.x + 1) * n_groups / gridDim.x);
  for (uint32_t grp = g_begin; grp < g_end; grp++) {
#endif
    const uint32_t base = grp * kBucketAlign;
    // buckets are 512-aligned and padded only at their tail: a group whose
    // first slot is empty is all padding (every thread reads the same slot)
    const uint32_t g_lead = __builtin_amdgcn_readfirstlane(a.perm[base]);
    if (g_lead == 0xFFFFFFFFu) {
#if MOCHI_POW_DYN
      publish();
#endif
      continue;
    }
    const uint32_t key = __builtin_amdgcn_readfirstlane((uint32_t)a.signer[g_lead]);
    if (key != cur_key) {
      __syncthreads();  // the old image is no longer read
      const v4i* src = (const v4i*)a.fold[key].img;
      for (uint32_t i = threadIdx.x; i < kFoldImgBytes / 16; i += blockDim.x) w[i] = src[i];
      __syncthreads();
      cur_key = key;
    }
    const uint32_t slot = base + threadIdx.x;
    const uint32_t g = slot < a.n_slots ? a.perm[slot] : 0xFFFFFFFFu;
    const bool active = g != 0xFFFFFFFFu;
    if (__ballot(active) == 0) {  // this wave's quarter of the group is padding: keep the barrier count
#pragma unroll 1
      for (int i = 0; i < 33; i++) phase_barrier();
#if MOCHI_POW_DYN
      publish();
#endif
      continue;
    }
    if (lag) phase_barrier();  // phase 0: the partner squares, this wave waits its turn
    uint32_t x[kL];
    {
      uint32_t wd[64];
      load_sig_words(a.sig, active ? g : g_lead, wd);  // inactive lanes shadow the lead grant (never stored)
      words_to_limbs(wd, x);
    }
    const cptr c = as_const(a.fold[key].cadd);
#pragma unroll 1
    for (int it = 0; it < 16; it++) {
      cptr ci = c;
      asm volatile("" : "+s"(ci));  // keep the 74 cadd loads inside the loop (SGPR pressure if hoisted)
      uint32_t t[2 * kL];
      const uint64_t t0 = stamp();
#if MOCHI_KARA2 >= 4
      kara_square2_lockstep(x, t);  // A/B: the second level for L in the lockstep form
#elif MOCHI_KARA2
      kara_square2(x, t);  // A/B: two Karatsuba levels for L and H (kara_dev.h)
#else
      kara_square(x, t);  // t = x^2, Karatsuba, t_hi biased (kara_dev.h)
#endif
      const uint64_t t1 = stamp();
      phase_barrier();
      __builtin_amdgcn_s_setprio(1);
      const uint64_t t2 = stamp();
      fold_reduce<false, true>(t, x, w + (threadIdx.x & 63), ci, nullptr);
      const uint64_t t3 = stamp();
      __builtin_amdgcn_s_setprio(0);
      phase_barrier();
      st.x2 += t1 - t0;
      st.fold += t3 - t2;
      st.n++;
    }
    if (active) {
#pragma unroll
      for (int q = 0; q < kL; q++) a.zout[(size_t)q * a.n_slots + slot] = x[q];
    }
    if (!lag) phase_barrier();  // phase 32: the partner folds its last squaring
#if MOCHI_POW_DYN
    publish();
#endif
  }
#if MOCHI_POW_STAMPS
  const uint64_t t_end = stamp();
  const uint32_t wv = blockIdx.x * 8 + (threadIdx.x >> 6);
  if ((threadIdx.x & 63) == 0 && wv < 4096) {
    g_pow_stamps[wv][0] = st.x2;
    g_pow_stamps[wv][1] = st.fold;
    g_pow_stamps[wv][2] = t_end - t_begin;
    g_pow_stamps[wv][3] = st.n;
    g_pow_stamps[wv][4] = 0;
  }
#else
  (void)t_begin;
#endif
}

// ---------------------------------------------------------------------------
// k_rsa_pow_lat — the same 16 squarings for a SMALL batch (a batcher flush of a
// few messages), where the chain's latency is the cost: in k_rsa_pow one
// signature's chain runs on one wave, and alone on its SIMD that wave spends
// most of each squaring in the fold's dependent MFMA chains (10 M-tiles x 10
// K-steps, ~20k cycles per squaring with x^2).  Here a block of 4 waves owns
// one 64-slot chunk (the same 64 signatures on every wave) and spreads each
// squaring over the CU's four SIMDs:
//   x^2:  wave 0 L = x_lo^2 (registers), wave 1 H = x_hi^2, wave 2 M = (x_lo +
//         x_hi)^2 (both to LDS); wave 0 combines them into t (kara_combine) and
//         writes t to LDS;
//   fold: wave w computes M-tiles w, w+4, w+8 (their 32-row weight slices of
//         the key's image, every wave building the B operands from t_hi), and
//         writes each of its output limbs' two int32 halves (fold_dev.h: p =
//         c0 + 2^8 c1 + t_lo + cadd, h = c2 + 2^8 c3) to LDS;
//   then every wave runs the 74-limb carry chain itself (x' = h 2^16 + p +
//         carry), so x' needs no broadcast.
// The limb arithmetic is fold_reduce's, split by tile -- bit-exact with
// k_rsa_pow by construction, and every small batch of the parity tests runs
// through it.  Five block barriers per squaring; one block per CU (the image +
// 38 KB of exchange), one wave per SIMD.
// ---------------------------------------------------------------------------
// A 37-limb square's columns as independent 64-bit sums (no carry between
// them, so the scheduler interleaves the chains -- a wave alone on its SIMD
// would wait out each mad's latency along one chain), then one carry pass into
// normalised limbs: out[0..2N].  a: 28- or 29-bit limbs (a column of the
// 29-bit M sum stays < 19 * 2^59 < 2^64).
template <int AO, int NOUT, int NA>
__device__ __forceinline__ void lat_square(const uint32_t (&a)[NA], uint32_t (&out)[NOUT]) {
  uint32_t d[kKH];
#pragma unroll
  for (int i = 0; i < kKH; i++) d[i] = a[AO + i] << 1;
  uint64_t col[2 * kKH - 1];
  static_for<0, 2 * kKH - 1>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - kKH + 1 > 0 ? k - kKH + 1 : 0;
    constexpr int xhi = k > 0 ? (k - 1) / 2 : -1;
    uint64_t acc = 0;
    if constexpr ((k & 1) == 0) acc = (uint64_t)a[AO + (k >> 1)] * a[AO + (k >> 1)];
    static_for<lo, xhi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      acc = mad64(d[i], a[AO + k - i], acc);
    });
    col[k] = acc;
  });
  uint64_t carry = 0;
  static_for<0, NOUT>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    if constexpr (k < 2 * kKH - 1) {
      const uint64_t v = col[k] + carry;
      out[k] = (uint32_t)v & kLimbMask;
      carry = v >> kLimbBits;
    } else if constexpr (k == 2 * kKH - 1) {
      out[k] = (uint32_t)carry & kLimbMask;
    } else {
      out[k] = (uint32_t)(carry >> kLimbBits);
    }
  });
}

__global__ __launch_bounds__(256, 1) void k_rsa_pow_lat(const PowArgs a) {
  __shared__ v4i w[kFoldImgBytes / 16];
  __shared__ uint32_t xr[kLatRows][kLatChunk];  // the exchange rows (lane-major: conflict-free)
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * kLatChunk;
  if (base >= a.n_slots) return;
  // buckets are filled from their start: a chunk whose first slot is empty is all padding
  const uint32_t g_lead = __builtin_amdgcn_readfirstlane(a.perm[base]);
  if (g_lead == 0xFFFFFFFFu) return;
  const uint32_t key = __builtin_amdgcn_readfirstlane((uint32_t)a.signer[g_lead]);
  // a signature among slots 32-63 (else the fold's second N-tile is skipped)
  const bool two = MOCHI_LAT_ONE_TILE == 0 ||
                   __builtin_amdgcn_readfirstlane(base + 32 < a.n_slots && a.perm[base + 32] != 0xFFFFFFFFu);
  {
    const v4i* src = (const v4i*)a.fold[key].img;
    for (uint32_t i = threadIdx.x; i < kFoldImgBytes / 16; i += blockDim.x) w[i] = src[i];
  }
  const uint32_t slot = base + lane;
  const uint32_t g = slot < a.n_slots ? a.perm[slot] : 0xFFFFFFFFu;
  const bool active = g != 0xFFFFFFFFu;
  uint32_t x[kL];
  {
    uint32_t wd[64];
    load_sig_words(a.sig, active ? g : g_lead, wd);  // inactive lanes shadow the lead grant (never stored)
    words_to_limbs(wd, x);
  }
  __syncthreads();
  const cptr c = as_const(a.fold[key].cadd);
  const v4i* wl = w + lane;
  const uint32_t kNoH[kHL] = {};  // nothing subtracted (k_rsa_final_lat subtracts the digest)
  uint64_t ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  const uint64_t t_loop = lstamp();
#pragma unroll 1
  for (int it = 0; it < 16; it++) {
    uint32_t lv[kL];
    uint64_t t0 = lstamp();
#if MOCHI_LAT_RAW  // A/B: columns as independent sums + one carry pass (measured slower: 148 vs 138 us)
    if (wv == 0) {  // L = x_lo^2, normalised, into registers
      lat_square<0>(x, lv);
    } else if (wv == 1) {  // H = x_hi^2 -> rows 0..73
      uint32_t hv[kL];
      lat_square<kKH>(x, hv);
#pragma unroll
      for (int k = 0; k < kL; k++) xr[k][lane] = hv[k];
    } else if (wv == 2) {  // M = (x_lo + x_hi)^2 -> rows 74..148
      uint32_t sx[kKH], mv[kL + 1];
#pragma unroll
      for (int i = 0; i < kKH; i++) sx[i] = x[i] + x[kKH + i];
      lat_square<0>(sx, mv);
#pragma unroll
      for (int k = 0; k <= kL; k++) xr[kL + k][lane] = mv[k];
    }
#else
    if (wv == 0) {  // L = x_lo^2, normalised, into registers
      uint64_t carry = 0;
      static_for<0, kL>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        lv[k] = square_col<0, k>(x, carry);
      });
    } else if (wv == 1) {  // H = x_hi^2 -> rows 0..73
      // (the limbs kept in registers and stored after the chain: stored per
      // column, this wave's squares took 5.7k cycles against wave 0's 4.4k)
      uint32_t hv[kL];
      uint64_t carry = 0;
      static_for<0, kL>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        hv[k] = square_col<kKH, k>(x, carry);
      });
#pragma unroll
      for (int k = 0; k < kL; k++) xr[k][lane] = hv[k];
    } else if (wv == 2) {  // M = (x_lo + x_hi)^2 -> rows 74..148
      uint32_t sx[kKH], mv[kL + 1];
#pragma unroll
      for (int i = 0; i < kKH; i++) sx[i] = x[i] + x[kKH + i];
      uint64_t carry = 0;
      static_for<0, kL + 1>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        mv[k] = square_col<0, k>(sx, carry);
      });
#pragma unroll
      for (int k = 0; k <= kL; k++) xr[kL + k][lane] = mv[k];
    }
#endif
    uint64_t t1 = lstamp();
    ph[0] += t1 - t0;
    __syncthreads();  // barrier 1: H and M written
    t0 = lstamp();
    ph[1] += t0 - t1;
    if (wv == 0) {  // t = L + 2^(28*37) (M - L - H) + 2^(28*74) H (t_hi biased) -> rows 0..147
      // M and H read from LDS up front, all loads in flight together (read inside
      // kara_combine's per-column scheduling fences, each waited for alone: 6.7k of
      // a squaring's 19k cycles, MOCHI_LAT_STAMPS)
      uint32_t t[2 * kL], hv[kL];
#pragma unroll
      for (int k = 0; k <= kL; k++) t[kKH + k] = xr[kL + k][lane];
#pragma unroll
      for (int k = 0; k < kL; k++) hv[k] = xr[k][lane];
      kara_combine(
          t, [&](auto kc, uint64_t&) { return lv[decltype(kc)::value]; },
          [&](auto kc, uint64_t&) { return hv[decltype(kc)::value]; });
#pragma unroll
      for (int k = 0; k < 2 * kL; k++) xr[k][lane] = t[k];
    }
    __syncthreads();  // barrier 2: t written
    t1 = lstamp();
    ph[2] += t1 - t0;
    cptr ci = c;
    asm volatile("" : "+s"(ci));
    if (two) {  // each contains barrier 3
      if (wv == 0) lat_fold<0, true>(wl, ci, xr, lane, kNoH);
      else if (wv == 1) lat_fold<1, true>(wl, ci, xr, lane, kNoH);
      else if (wv == 2) lat_fold<2, true>(wl, ci, xr, lane, kNoH);
      else lat_fold<3, true>(wl, ci, xr, lane, kNoH);
    } else {
      if (wv == 0) lat_fold<0, false>(wl, ci, xr, lane, kNoH);
      else if (wv == 1) lat_fold<1, false>(wl, ci, xr, lane, kNoH);
      else if (wv == 2) lat_fold<2, false>(wl, ci, xr, lane, kNoH);
      else lat_fold<3, false>(wl, ci, xr, lane, kNoH);
    }
    t0 = lstamp();
    ph[3] += t0 - t1;
    __syncthreads();  // barrier 4: every (p, h) pair written
    t1 = lstamp();
    ph[4] += t1 - t0;
    if (wv < 3) {  // x' = sum_q (h_q 2^16 + p_q) 2^(28 q), normalised (fold_reduce's carry chain)
      int pq[2 * kL];  // every pair read first: the loads in flight together, then the chain
#pragma unroll
      for (int i = 0; i < 2 * kL; i++) pq[i] = (int)xr[i][lane];
      int64_t carry = 0;
#pragma unroll
      for (int q = 0; q < kL; q++) {
        const int64_t v = mad_i64(pq[2 * q + 1], 65536, mad_i64(pq[2 * q], 1, carry));
        x[q] = (uint32_t)v & kLimbMask;
        carry = v >> kLimbBits;
      }
    }
    t0 = lstamp();
    ph[5] += t0 - t1;
    __syncthreads();  // barrier 5: the pairs are read before the next H / M overwrite them
    ph[6] += lstamp() - t0;
  }
#if MOCHI_LAT_STAMPS
  ph[7] = lstamp() - t_loop;
  if (lane == 0 && blockIdx.x < 256) {
#pragma unroll
    for (int i = 0; i < 8; i++) g_lat_stamps[blockIdx.x][wv][i] = ph[i];
  }
#else
  (void)ph, (void)t_loop;
#endif
  if (wv == 0 && active) {
#pragma unroll
    for (int q = 0; q < kL; q++) a.zout[(size_t)q * a.n_slots + slot] = x[q];
  }
}

}  // namespace

#if MOCHI_POW_STAMPS
extern "C" int mochi_debug_pow_stamps(unsigned long long* out, unsigned n_waves) {
  if (n_waves > 4096) n_waves = 4096;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_pow_stamps), 40 * (size_t)n_waves, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif

#if MOCHI_LAT_STAMPS
extern "C" int mochi_debug_lat_stamps(unsigned long long* out, unsigned n_blocks) {
  if (n_blocks > 256) n_blocks = 256;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mochi::g_lat_stamps), 256 * (size_t)n_blocks, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif

// MOCHI_NO_LAT=1 (A/B): small batches take k_rsa_pow as well
static bool lat_off() {
  static const bool off = [] {
    const char* e = getenv("MOCHI_NO_LAT");
    return e && e[0] == '1';
  }();
  return off;
}

void launch_rsa_pow(const LaunchArgs& a, hipStream_t st, bool latency) {
  const PowArgs pw{a.perm, a.n_slots, a.sig, a.signer, a.fold, a.xbuf, a.total + kTotPowGroup};
  if (latency && !lat_off()) {  // a small batch: one block per 64-slot chunk (empty chunks exit at once)
    const uint32_t chunks = (a.n_slots + kLatChunk - 1) / kLatChunk;
    if (chunks) hipLaunchKernelGGL(k_rsa_pow_lat, dim3(chunks), dim3(256), 0, st, pw);
    return;
  }
  const uint32_t blocks = fold_grid(a.n_slots);
  if (blocks) hipLaunchKernelGGL(k_rsa_pow, dim3(blocks), dim3(kBucketAlign), 0, st, pw);
}

}  // namespace mochi
