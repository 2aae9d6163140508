// rsa_final.hip — k_rsa_final: finish the RSA-2048 verify and the
// EMSA-PKCS1-v1_5 check (RFC 8017 §8.2.2 / §9.2, "SHA256withRSA") with one
// product and one matrix-core fold per grant.
//
// k_rsa_pow leaves z = s^(2^16) (mod n), z < 2^2064.  Then per grant
//   t = z * s                                  148 limbs, VALU, one level of
//                                              Karatsuba (3 x 37 x 37 = 4,107
//                                              v_mad_u64_u32, kara_dev.h)
//   D = t_lo + fold(t_hi) + (n - Cpad) - H     the fold of k_rsa_pow (fold_dev.h)
//                                              with the per-key constant
//                                              cnc = cadd + n - Cpad
// so D == s^65537 + n - EM (mod n) with EM = Cpad + H (Cpad: the fixed
// padding + DigestInfo, H: the 256-bit digest), and 0 < D < 2^2064 + n
// (the fold is < 2^2064; n - EM > 0 because EM < 2^2041 < n).  The grant is
// valid iff s < n and s^65537 mod n == EM, i.e. iff D == 0 (mod n).  One
// Montgomery step by 2^28,
//   D' = (D + m n) / 2^28,   m = D * (-n^-1) mod 2^28,
// gives D' == D * 2^-28 (mod n) and 0 < D' < 2^2036 + n/2^28 + n < 2n, so
// valid <=> D' == n exactly.  Cost: 5,476 + 74 mads and 200 MFMAs per 64
// grants, instead of a general Montgomery multiply (10,952 mads) + 1,480.
//
// s < n mirrors OpenSSL's RSA_R_DATA_TOO_LARGE_FOR_MODULUS reject.
//
// Grid: like k_rsa_pow — persistent blocks over the signer's 512-slot groups,
// the signer's fold image in LDS — but one wave per SIMD (256 threads, two
// halves per group): with 512 registers z, s and the 148-limb product stay in
// registers (at 256 the product's peak would spill).
#include "fold_dev.h"
#include "rsa_common.h"

#include <cstdlib>

// A/B: groups from a device counter (fold_dev.h for_groups), as k_rsa_pow's --
// measured 1.6 % slower here (5.29-5.31 vs 5.21 ms), so the contiguous ranges stay
#ifndef MOCHI_FINAL_DYN
#define MOCHI_FINAL_DYN 0
#endif

// MOCHI_FINAL_STAMPS (measurement builds only, `make ab VSRC=rsa_final`): per
// wave, s_memtime cycles in the operand loads (=2: an explicit vmcnt(0) wait
// after them, so their latency is separated from the product), the product,
// the digest load + fold, the final Montgomery step + store, and the whole
// kernel; read back with mochi_debug_final_stamps() (scripts/final_stamps.py)
#ifndef MOCHI_FINAL_STAMPS
#define MOCHI_FINAL_STAMPS 0
#endif

namespace mochi {
#if MOCHI_FINAL_STAMPS
__device__ unsigned long long g_final_stamps[4096][6];
#endif
namespace {

struct FStamps {
  uint64_t load = 0, prod = 0, fold = 0, check = 0, n = 0;
};

__device__ __forceinline__ uint64_t fstamp() {
#if MOCHI_FINAL_STAMPS
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t t = __builtin_amdgcn_s_memtime();
  __builtin_amdgcn_sched_barrier(0);
  return t;
#else
  return 0;
#endif
}

// A/B: an explicit vmcnt(0) wait once a half-group's operands are issued.
// Phase stamps (scripts/final_stamps.py, round 6) showed the product 3.2k
// cycles per item faster behind one wait than with the compiler's waits for
// single limbs interleaved into its first columns.
#ifndef MOCHI_FINAL_WAIT
#define MOCHI_FINAL_WAIT 1
#endif

// One lane's operands, as loaded: the signature's 16-byte rows, z's limbs, and
// -- issued with them, so their latency hides under the product instead of
// stalling the fold and the flag store (stamps: ~2k cycles each per item) --
// the grant's digest (through its distinct-result index) and its parse flags.
struct FinalOps {
  uint4 sr[16];
  uint32_t z[kL];
  uint32_t hw[8];
  uint32_t g, fl, d;
};

__device__ __forceinline__ void final_load(uint32_t slot, uint32_t g_lead, const uint32_t* __restrict__ perm,
                                           uint32_t n_slots, const uint8_t* __restrict__ sig,
                                           const uint32_t* __restrict__ zin, const uint32_t* __restrict__ lead,
                                           const uint8_t* __restrict__ flags, FinalOps& o) {
  o.g = slot < n_slots ? perm[slot] : 0xFFFFFFFFu;
  const uint32_t gg = o.g != 0xFFFFFFFFu ? o.g : g_lead;  // inactive lanes shadow the lead grant
  o.d = lead ? lead[gg] : gg;  // the grant's distinct prep result (kernels.hip); its digest: final_load_digest
  o.fl = flags[gg];
  const uint4* s128 = (const uint4*)(sig + (size_t)gg * MOCHI_RSA_BYTES);
#pragma unroll
  for (int q = 0; q < 16; q++) o.sr[q] = s128[q];
  // z limb j of this slot: a wave-uniform limb base (SGPRs) + the lane's byte
  // offset (one VGPR), so no 64-bit address per limb stays live.  Every slot
  // of a non-empty group is < n_slots (buckets end 512-aligned inside it).
  const gchar* zp = (const gchar*)zin;
  const uint32_t zoff = slot * 4u;
  const size_t zstride = (size_t)n_slots * 4u;
#pragma unroll
  for (int j = 0; j < kL; j++) {
    o.z[j] = *(const guint*)(zp + zoff);
    zp += zstride;
    asm volatile("" : "+s"(zp));  // a running pointer: 74 limb bases would sit in SGPRs and spill
  }
}

// Issued after the operands have landed (o.d with them): the digest arrives
// while the product runs.
__device__ __forceinline__ void final_load_digest(const uint32_t* __restrict__ digest, uint32_t n_dist, FinalOps& o) {
#pragma unroll
  for (int i = 0; i < 8; i++) o.hw[i] = digest[(size_t)(7 - i) * n_dist + o.d];
}

// One wave's worth of grants from their loaded operands.
__device__ __forceinline__ void final_slot(FinalOps& o, uint32_t key, uint32_t g_lead,
                                           const KeyEntry* __restrict__ keys, const FoldKey* __restrict__ fold,
                                           const uint32_t* __restrict__ digest, const uint32_t* __restrict__ lead,
                                           uint32_t n_dist, uint8_t* __restrict__ flags, const v4i* w,
                                           FStamps& st) {
  const uint32_t g = o.g;
  const bool active = g != 0xFFFFFFFFu;
  if (__ballot(active) == 0) return;  // this wave's part of the group is padding
  const uint64_t t1 = fstamp();
  const KeyEntry* ke = keys + key;
  const cptr n = as_const(ke->n);
  uint32_t sv[kL];
  {
    uint32_t wd[64];
#pragma unroll
    for (int q = 0; q < 16; q++) {  // big-endian bytes [16q, 16q+16)
      wd[63 - 4 * q] = bswap32(o.sr[q].x);
      wd[62 - 4 * q] = bswap32(o.sr[q].y);
      wd[61 - 4 * q] = bswap32(o.sr[q].z);
      wd[60 - 4 * q] = bswap32(o.sr[q].w);
    }
    words_to_limbs(wd, sv);
  }
  // s < n on the normalised limbs (borrow chain)
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < kL; j++) br = ((int32_t)sv[j] - (int32_t)n[j] - br) < 0 ? 1 : 0;
  asm volatile("" : "+v"(br));  // decide here (sunk to its use, it keeps s live through the fold)
  const bool s_lt_n = br != 0;
  uint32_t (&x)[kL] = o.z;
  // ---- t = z * s: one level of Karatsuba (kara_dev.h), t_hi biased ----
  uint32_t t[2 * kL];
  kara_product(x, sv, t);
  const uint64_t t2 = fstamp();
  // digest H as 10 limbs (digest word 0 = most significant 4 bytes of H)
  uint32_t hl[kHL];
  {
    const uint32_t (&hw)[8] = o.hw;
#pragma unroll
    for (int j = 0; j < kHL; j++) {
      const int bit = j * kLimbBits, wi = bit >> 5, sh = bit & 31;
      const uint64_t v = ((uint64_t)(wi + 1 < 8 ? hw[wi + 1] : 0u) << 32) | hw[wi];
      hl[j] = (uint32_t)(v >> sh) & kLimbMask;
    }
  }
  // ---- D = t_lo + fold(t_hi) + cadd + n - Cpad - H ----
  fold_reduce<true, true>(t, x, w + (threadIdx.x & 63), as_const(fold[key].cnc), hl);
  const uint64_t t3 = fstamp();
  // ---- D' = (D + m n) / 2^28 == n ? ----
  cptr nn = n;
  asm volatile("" : "+s"(nn));  // reload n here (kept from the s < n check it would sit in SGPRs and spill)
  const uint32_t n0inv = *as_const(&ke->n0inv);
  const uint32_t m = (x[0] * n0inv) & kLimbMask;
  uint64_t c = mad64(m, nn[0], x[0]) >> kLimbBits;  // the low 28 bits cancel
  uint32_t diff = 0;
#pragma unroll
  for (int k = 1; k < kL; k++) {
    const uint64_t acc = mad64(m, nn[k], x[k] + c);
    diff |= ((uint32_t)acc & kLimbMask) ^ nn[k - 1];
    c = acc >> kLimbBits;
  }
  diff |= c != (uint64_t)nn[kL - 1] ? 1u : 0u;
  if (active) {
    const bool ok = s_lt_n && diff == 0;
    flags[g] = (uint8_t)(o.fl | (ok ? MOCHI_GRANT_SIG_OK : 0));
  }
#if MOCHI_FINAL_STAMPS
  const uint64_t t4 = fstamp();
  st.prod += t2 - t1;
  st.fold += t3 - t2;
  st.check += t4 - t3;
  st.n++;
#else
  (void)t1, (void)t2, (void)t3, (void)st;
#endif
}

// 256 threads (one wave per SIMD, 512 registers: z, s and the whole product
// stay in registers) walk each 512-slot group in two halves.
__global__ __launch_bounds__(256, 1) void k_rsa_final(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                                       const uint8_t* __restrict__ sig,
                                                       const uint16_t* __restrict__ signer,
                                                       const KeyEntry* __restrict__ keys,
                                                       const FoldKey* __restrict__ fold,
                                                       const uint32_t* __restrict__ zin,
                                                       const uint32_t* __restrict__ digest,
                                                       const uint32_t* __restrict__ lead, uint32_t n_dist,
                                                       uint8_t* __restrict__ flags, uint32_t* __restrict__ ctr) {
  __shared__ v4i w[kFoldImgBytes / 16];
  FStamps st;
  const uint64_t t_begin = fstamp();
  for_groups(perm, n_slots, signer, fold, w, [&](uint32_t base, uint32_t key, uint32_t g_lead) {
    // (the next half's operands loaded while this half computes -- into AGPRs,
    // 445 registers, or both halves up front, 483 -- measured 10 % and 18 %
    // slower: DESIGN.md section 9)
#pragma unroll 1
    for (uint32_t h = 0; h < kBucketAlign; h += 256) {
      FinalOps o;
      const uint64_t t0 = fstamp();
      final_load(base + h + threadIdx.x, g_lead, perm, n_slots, sig, zin, lead, flags, o);
#if MOCHI_FINAL_STAMPS == 2 || (MOCHI_FINAL_WAIT && !MOCHI_FINAL_STAMPS)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
      final_load_digest(digest, n_dist, o);
#if MOCHI_FINAL_STAMPS
      st.load += fstamp() - t0;
#endif
      (void)t0;
      final_slot(o, key, g_lead, keys, fold, digest, lead, n_dist, flags, w, st);
    }
  }, MOCHI_FINAL_DYN ? ctr : nullptr);
#if MOCHI_FINAL_STAMPS
  const uint64_t t_end = fstamp();
  const uint32_t wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  if ((threadIdx.x & 63) == 0 && wv < 4096) {
    g_final_stamps[wv][0] = st.load;
    g_final_stamps[wv][1] = st.prod;
    g_final_stamps[wv][2] = st.fold;
    g_final_stamps[wv][3] = st.check;
    g_final_stamps[wv][4] = st.n;
    g_final_stamps[wv][5] = t_end - t_begin;
  }
#else
  (void)t_begin;
#endif
}

// ---------------------------------------------------------------------------
// k_rsa_final_lat — k_rsa_final for a SMALL batch (a batcher flush: one or two
// grants per signer bucket), where one lone wave per 64-slot group spends
// ~22k cycles on the product and ~12k on the fold.  As in k_rsa_pow_lat, a block
// of 4 waves owns one 64-slot chunk and splits the work over the CU's SIMDs:
//   t = z s:  wave 0 L = z_lo s_lo (registers), wave 1 H = z_hi s_hi, wave 2
//             M = (z_lo + z_hi)(s_lo + s_hi) (both to LDS) at once; wave 0
//             combines them (kara_combine) into t in LDS;
//   fold:     wave w folds M-tiles w, w+4, w+8 (fold_dev.h lat_fold, with the
//             final's constant cnc and the digest H subtracted, as
//             fold_reduce<true, true>); the second N-tile only when slots
//             32-63 hold a grant;
//   then wave 0 runs the carry chain, the Montgomery step and the compare with
//             n, and stores the flags -- the arithmetic of final_slot, so the
//             verdicts are bit-exact with k_rsa_final (every small batch of the
//             parity tests runs through it).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256, 1) void k_rsa_final_lat(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                                           const uint8_t* __restrict__ sig,
                                                           const uint16_t* __restrict__ signer,
                                                           const KeyEntry* __restrict__ keys,
                                                           const FoldKey* __restrict__ fold,
                                                           const uint32_t* __restrict__ zin,
                                                           const uint32_t* __restrict__ digest,
                                                           const uint32_t* __restrict__ lead, uint32_t n_dist,
                                                           uint8_t* __restrict__ flags) {
  __shared__ v4i w[kFoldImgBytes / 16];
  __shared__ uint32_t xr[kLatRows][kLatChunk];  // the exchange rows (lane-major)
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t base = blockIdx.x * kLatChunk;
  if (base >= n_slots) return;
  // buckets are filled from their start: a chunk whose first slot is empty is all padding
  const uint32_t g_lead = __builtin_amdgcn_readfirstlane(perm[base]);
  if (g_lead == 0xFFFFFFFFu) return;
  const uint32_t key = __builtin_amdgcn_readfirstlane((uint32_t)signer[g_lead]);
  {
    const v4i* src = (const v4i*)fold[key].img;
    for (uint32_t i = threadIdx.x; i < kFoldImgBytes / 16; i += blockDim.x) w[i] = src[i];
  }
  const bool two = __builtin_amdgcn_readfirstlane(base + 32 < n_slots && perm[base + 32] != 0xFFFFFFFFu);
  const uint32_t slot = base + lane;
  const uint32_t g = slot < n_slots ? perm[slot] : 0xFFFFFFFFu;
  const bool active = g != 0xFFFFFFFFu;
  const uint32_t gg = active ? g : g_lead;  // inactive lanes shadow the lead grant (never stored)
  const uint32_t fl = flags[gg];  // the parse flags (grant prep), OR'd with SIG_OK at the end
  uint32_t z[kL], sv[kL];
#pragma unroll
  for (int j = 0; j < kL; j++) z[j] = zin[(size_t)j * n_slots + (slot < n_slots ? slot : base)];
  {
    uint32_t wd[64];
    load_sig_words(sig, gg, wd);
    words_to_limbs(wd, sv);
  }
  __syncthreads();  // the image is staged
  uint32_t lv[kL];
  if (wv == 0) {  // L = z_lo s_lo, normalised, into registers
    uint64_t carry = 0;
    static_for<0, kL>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      lv[k] = product_col<0, 0, k>(z, sv, carry);
    });
  } else if (wv == 1) {  // H = z_hi s_hi -> rows 0..73
    uint32_t hv[kL];  // stored after the chain (k_rsa_pow_lat)
    uint64_t carry = 0;
    static_for<0, kL>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      hv[k] = product_col<kKH, kKH, k>(z, sv, carry);
    });
#pragma unroll
    for (int k = 0; k < kL; k++) xr[k][lane] = hv[k];
  } else if (wv == 2) {  // M = (z_lo + z_hi)(s_lo + s_hi) -> rows 74..148
    uint32_t sz[kKH], ss[kKH];
#pragma unroll
    for (int i = 0; i < kKH; i++) {
      sz[i] = z[i] + z[kKH + i];
      ss[i] = sv[i] + sv[kKH + i];
    }
    uint32_t mv[kL + 1];
    uint64_t carry = 0;
    static_for<0, kL + 1>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      mv[k] = product_col<0, 0, k>(sz, ss, carry);
    });
#pragma unroll
    for (int k = 0; k <= kL; k++) xr[kL + k][lane] = mv[k];
  }
  __syncthreads();  // barrier 1: H and M written
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
  // the digest H as 10 limbs (digest word 0 = most significant 4 bytes of H)
  uint32_t hl[kHL];
  {
    const uint32_t d = lead ? lead[gg] : gg;
    uint32_t hw[8];
#pragma unroll
    for (int i = 0; i < 8; i++) hw[i] = digest[(size_t)(7 - i) * n_dist + d];
#pragma unroll
    for (int j = 0; j < kHL; j++) {
      const int bit = j * kLimbBits, wi = bit >> 5, sh = bit & 31;
      const uint64_t v = ((uint64_t)(wi + 1 < 8 ? hw[wi + 1] : 0u) << 32) | hw[wi];
      hl[j] = (uint32_t)(v >> sh) & kLimbMask;
    }
  }
  __syncthreads();  // barrier 2: t written
  const v4i* wl = w + lane;
  cptr cn = as_const(fold[key].cnc);
  asm volatile("" : "+s"(cn));
  if (two) {  // each contains barrier 3
    if (wv == 0) lat_fold<0, true, true>(wl, cn, xr, lane, hl);
    else if (wv == 1) lat_fold<1, true, true>(wl, cn, xr, lane, hl);
    else if (wv == 2) lat_fold<2, true, true>(wl, cn, xr, lane, hl);
    else lat_fold<3, true, true>(wl, cn, xr, lane, hl);
  } else {
    if (wv == 0) lat_fold<0, false, true>(wl, cn, xr, lane, hl);
    else if (wv == 1) lat_fold<1, false, true>(wl, cn, xr, lane, hl);
    else if (wv == 2) lat_fold<2, false, true>(wl, cn, xr, lane, hl);
    else lat_fold<3, false, true>(wl, cn, xr, lane, hl);
  }
  __syncthreads();  // barrier 4: every (p, h) pair written
  if (wv != 0) return;
  // D = sum_q (h_q 2^16 + p_q) 2^(28 q), normalised (fold_reduce's carry chain)
  uint32_t x[kL];
  {
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
  // s < n, then D' = (D + m n) / 2^28 == n (final_slot)
  const KeyEntry* ke = keys + key;
  const cptr n = as_const(ke->n);
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < kL; j++) br = ((int32_t)sv[j] - (int32_t)n[j] - br) < 0 ? 1 : 0;
  const uint32_t n0inv = *as_const(&ke->n0inv);
  const uint32_t m = (x[0] * n0inv) & kLimbMask;
  uint64_t c = mad64(m, n[0], x[0]) >> kLimbBits;  // the low 28 bits cancel
  uint32_t diff = 0;
#pragma unroll
  for (int k = 1; k < kL; k++) {
    const uint64_t acc = mad64(m, n[k], x[k] + c);
    diff |= ((uint32_t)acc & kLimbMask) ^ n[k - 1];
    c = acc >> kLimbBits;
  }
  diff |= c != (uint64_t)n[kL - 1] ? 1u : 0u;
  if (active) {
    const bool ok = br != 0 && diff == 0;
    flags[g] = (uint8_t)(fl | (ok ? MOCHI_GRANT_SIG_OK : 0));
  }
}

// MOCHI_NO_FINAL_LAT=1 (A/B): small batches take k_rsa_final as well
static bool final_lat_off() {
  static const bool off = [] {
    const char* e = getenv("MOCHI_NO_FINAL_LAT");
    return e && e[0] == '1';
  }();
  return off;
}

}  // namespace

void launch_rsa_final(const LaunchArgs& a, const uint32_t* lead, uint32_t n_dist, hipStream_t st, bool latency) {
  if (a.dbg_y) {  // mochi_rsa_public_op: materialise s^65537 mod n
    launch_rsa_raw(a, st);
    return;
  }
  if (latency && !final_lat_off()) {  // a small batch: one block per 64-slot chunk (empty chunks exit at once)
    const uint32_t chunks = (a.n_slots + kLatChunk - 1) / kLatChunk;
    if (chunks)
      hipLaunchKernelGGL(k_rsa_final_lat, dim3(chunks), dim3(256), 0, st, a.perm, a.n_slots, a.sig, a.signer, a.keys,
                         a.fold, a.xbuf, a.digest, lead, n_dist, a.flags);
    return;
  }
  const uint32_t blocks = fold_grid(a.n_slots);
  if (!blocks) return;
  hipLaunchKernelGGL(k_rsa_final, dim3(blocks), dim3(256), 0, st, a.perm, a.n_slots, a.sig, a.signer, a.keys, a.fold,
                     a.xbuf, a.digest, lead, n_dist, a.flags, a.total + kTotFinalGroup);
}

}  // namespace mochi

#if MOCHI_FINAL_STAMPS
extern "C" int mochi_debug_final_stamps(unsigned long long* out, unsigned n_waves) {
  if (n_waves > 4096) n_waves = 4096;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mochi::g_final_stamps), 48 * (size_t)n_waves, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
