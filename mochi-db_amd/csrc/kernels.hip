// kernels.hip — the Write2 certificate-verification hot path on gfx950.
//
//   k_grant_prep    per grant (certificate order): proto3 Grant parse
//                   (MochiProtocol.java:7369-7425 semantics) + SHA-256 of the
//                   grant bytes (the signed message)
//   k_bucket_*      counting sort of grants by signer into 512-aligned buckets,
//                   so every k_rsa_pow block (8 waves) has ONE modulus and fold
//                   matrix, and every wave of k_rsa_final one modulus (SGPRs)
//   k_rsa_pow       z = s^(2^16) mod n, 16 squarings, reduction on MFMA (rsa_pow.hip)
//   k_rsa_final     u = MontMul(z, s) = s^65537 R^-1; compare with the
//                   EMSA-PKCS1-v1_5 encoding of SHA-256(grant); s < n check
//   k_tally         per certificate: processMultiGrantsFromAllServers +
//                   write2apply verdict (InMemoryDataStore.java:576-640)
//   k_pack_bits     grant-valid bitmap via wavefront ballot
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "../../include/mochi_hip.h"
#include "kernels.h"
#include "prep_dev.h"
#include "proto_dev.h"

namespace mochi {


// ---------------------------------------------------------------------------
// k_grant_prep: parse + SHA-256, certificate order (lane = grant).
// ---------------------------------------------------------------------------
#ifndef MOCHI_PREP_WAVES
#define MOCHI_PREP_WAVES 4  // amdgpu_waves_per_eu for the prep kernels: k_grant_prep_cert fits 126 VGPRs unspilled
                            // (133 uncapped: 3 waves); prep outside the serial stages 0.86 -> 0.83 ms
#endif
#if MOCHI_PREP_WAVES
#define MOCHI_PREP_ATTR __attribute__((amdgpu_waves_per_eu(MOCHI_PREP_WAVES)))
#else
#define MOCHI_PREP_ATTR
#endif
__global__ __launch_bounds__(256) MOCHI_PREP_ATTR void k_grant_prep(const PrepArgs a) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < a.n) grant_prep_one(a, i);
}

// ---------------------------------------------------------------------------
// Grant prep, each distinct grant of a certificate once.  In an honest
// certificate the R grants of an op key are the same bytes (every replica
// builds the Grant from the same objectId, transaction hash and timestamp,
// InMemoryDataStore.java:131-140), and PrepOut is a function of the bytes.
// k_grant_prep_cert (lane = certificate) preps the first grant of each key slot
// (up to two slots) and hands its result to every later grant of the slot with
// the same bytes -- compared as bytes (equal offsets suffice; wire-path grants
// are separate copies, which the decoder may already have matched: `same`),
// never assumed.  The rest (a grant that differs from its slot's first, a third
// slot) keeps its flag (memset 1) and k_grant_prep_rare preps it.
//
// Results are stored once per DISTINCT grant (prep_dev.h PrepArgs): the first
// slot's digest and hash slice at index c (consecutive lanes, consecutive
// words: coalesced, and k_rsa_final's lanes -- consecutive certificates of one
// signer -- read them coalesced too), a second slot's at d_base + g; every
// grant gets only its own timestamp, flags and lead index (13 bytes, not 53).
// ---------------------------------------------------------------------------
struct PrepCertArgs {
  const uint8_t* grant_key;
  const uint32_t* cert_grant_off;
  const uint32_t* same;  // [N] or null: an earlier grant of the certificate with the same bytes (the decoder's match)
  uint32_t n_certs;
  uint8_t* rare;         // [N]: 1 = prepped by k_grant_prep_rare (preset to 1: a grant outside every certificate too)
  const uint8_t* expected;  // [n_certs][MOCHI_TXN_HASH_BYTES] or null: the leaders' hash checks (kHashChecked)
};

// A slot leader's hash_len word: its transactionHash compared with certificate
// c's expected hash here, where the grant's bytes were just read (L2-warm), so
// k_tally -- a serial stage with nothing to hide its memory round trips -- reads
// one word for g0 instead of hash_off and 2 x 128 bytes.  Every grant reading
// this distinct result through `lead` belongs to certificate c.
__device__ __forceinline__ uint32_t leader_hash_word(const PrepArgs& a, const PrepCertArgs& p, uint32_t c,
                                                     uint64_t og, const PrepOut& o) {
  if (!p.expected || !(o.flags & MOCHI_GRANT_PARSED)) return hash_len_word(o);
  static_assert(MOCHI_TXN_HASH_BYTES == 128, "bytes128_equal");
  const bool eq = o.hash_len == MOCHI_TXN_HASH_BYTES &&
                  bytes128_equal(a.blob + og + o.hash_rel, p.expected + (size_t)c * MOCHI_TXN_HASH_BYTES);
  return kHashChecked | (eq ? kHashEq : 0u);
}

// The block's first-slot per-grant outputs go out through LDS: each lane puts
// its leader's timestamp and flags in `lo` and marks the leader and its
// byte-equal grants in `ref`; then the block stores them grant by grant
// (consecutive lanes, consecutive grants), not lane = certificate at a 4-grant
// stride.  A block whose certificates hold more than kPrepBlockGrants grants,
// and second slots, store directly.
constexpr uint32_t kPrepBlockGrants = 2048;
#ifndef MOCHI_SAME_HINT_CHECK
#define MOCHI_SAME_HINT_CHECK 0
#endif
#ifndef MOCHI_PREP_LDS_STORE
#define MOCHI_PREP_LDS_STORE 1  // A/B
#endif

struct PrepOutLds {  // a leader's per-grant outputs and its byte offset
  uint32_t ts_lo, ts_hi, flags;
  uint32_t goff_lo, goff_hi;
};

// Byte compares of separate copies (a slot's later grants whose offsets differ
// from its first grant's and that the decoder did not match) are not done by
// the certificate's lane: there each compare is one more dependent memory round
// trip per follower (C4 with separate copies: +1.5 ms).  The staged pass marks
// them (rare = 2) with their results stored optimistically and the leader's
// byte offset parked in hash_off[d_base + h] (the follower's own distinct slot,
// unused unless the bytes differ), and k_grant_match compares them 16 lanes per
// grant, coalesced; a mismatch becomes rare = 1 (prepped on its own).
constexpr uint32_t kMatchMaxLen = 256;  // 16 lanes x 16 bytes; longer grants compare in the certificate's lane
constexpr uint16_t kRefMatch = 0x8000u;

__global__ __launch_bounds__(256) MOCHI_PREP_ATTR void k_grant_prep_cert(const PrepArgs a, const PrepCertArgs p) {
#if MOCHI_PREP_LDS_STORE
  __shared__ PrepOutLds lo[256];
  __shared__ uint16_t ref[kPrepBlockGrants];
  const uint32_t c0 = blockIdx.x * blockDim.x;
  const uint32_t c_end = c0 + blockDim.x < p.n_certs ? c0 + blockDim.x : p.n_certs;
  const uint32_t G0 = p.cert_grant_off[c0], G1 = p.cert_grant_off[c_end];
  const bool staged = G1 - G0 <= kPrepBlockGrants;  // block-uniform
  if (staged)
    for (uint32_t i = threadIdx.x; i < G1 - G0; i += blockDim.x) ref[i] = 0xFFFFu;
  __syncthreads();
#else
  const bool staged = false;
  const uint32_t G0 = 0, c0 = 0;
  uint16_t* ref = nullptr;
  PrepOutLds* lo = nullptr;
#endif
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < p.n_certs) {
    const uint32_t g_lo = p.cert_grant_off[c], g_hi = p.cert_grant_off[c + 1];
    uint64_t seen = 0;  // key slots < 64 whose first grant came already (others: a scan back)
    uint32_t leaders = 0;
#pragma unroll 1
    for (uint32_t g = g_lo; g < g_hi; g++) {
      const uint32_t s = p.grant_key[g];
      bool first;
      if (s < 64) {
        first = !((seen >> s) & 1);
        seen |= 1ull << s;
      } else {
        first = true;
#pragma unroll 1
        for (uint32_t q = g_lo; q < g; q++)
          if (p.grant_key[q] == s) {
            first = false;
            break;
          }
      }
      if (!first) continue;  // decided in its slot's first grant's pass
      if (leaders++ == 2) break;  // a third slot: its grants are left to k_grant_prep_rare (rare stays 1)
      // g leads its slot: prep it, store its distinct result, then hand it to every
      // later grant of the slot with the same bytes; a grant that differs stays flagged
      const bool via_lds = staged && leaders == 1;
      PrepOut o;
      const uint64_t og = a.goff[g];
      const uint32_t lg = a.glen[g];
      grant_prep_bytes(a.blob + og, lg, o);
      const uint32_t d = leaders == 1 ? c : a.d_base + g;
      grant_prep_store_dist(a, d, og, o, leader_hash_word(a, p, c, og, o));
      if (via_lds) {
        PrepOutLds& e = lo[threadIdx.x];
        e.ts_lo = (uint32_t)o.ts;
        e.ts_hi = (uint32_t)((uint64_t)o.ts >> 32);
        e.flags = o.flags;
        e.goff_lo = (uint32_t)og;
        e.goff_hi = (uint32_t)(og >> 32);
        ref[g - G0] = (uint16_t)threadIdx.x;
      } else {
        grant_prep_store_grant(a, g, d, o.ts, o.flags);
        p.rare[g] = 0;
      }
#pragma unroll 1
      for (uint32_t h = g + 1; h < g_hi; h++) {
        if (p.grant_key[h] != s) continue;
        if (a.glen[h] != lg) continue;
        const uint64_t oh = a.goff[h];
        // the decoder's match (`same`) is taken only with equal lengths as well; with
        // MOCHI_SAME_HINT_CHECK=1 (a CI build) it must also survive the byte compare
        const bool hinted = p.same && p.same[h] == g && !MOCHI_SAME_HINT_CHECK;
        const bool known = hinted || oh == og;
        if (via_lds && !known && lg <= kMatchMaxLen) {  // compared by k_grant_match
          ref[h - G0] = (uint16_t)threadIdx.x | kRefMatch;
          continue;
        }
        if (!known && !bytes_equal(a.blob + oh, a.blob + og, lg)) continue;
        if (via_lds) {
          ref[h - G0] = (uint16_t)threadIdx.x;
        } else {
          grant_prep_store_grant(a, h, d, o.ts, o.flags);
          p.rare[h] = 0;
        }
      }
    }
  }
#if MOCHI_PREP_LDS_STORE
  __syncthreads();
  if (staged) {
#pragma unroll 1
    for (uint32_t i = threadIdx.x; i < G1 - G0; i += blockDim.x) {
      const uint32_t rr = ref[i];
      if (rr == 0xFFFFu) continue;  // a rare grant, or a second slot's (stored directly)
      const uint32_t r = rr & 0xFFu;
      const PrepOutLds& e = lo[r];
      grant_prep_store_grant(a, G0 + i, c0 + r, (int64_t)(((uint64_t)e.ts_hi << 32) | e.ts_lo), (uint8_t)e.flags);
      if (rr & kRefMatch) {  // optimistic: k_grant_match compares the bytes with the leader's
        a.hash_off[(size_t)a.d_base + G0 + i] = ((uint64_t)e.goff_hi << 32) | e.goff_lo;
        p.rare[G0 + i] = 2;
      } else {
        p.rare[G0 + i] = 0;
      }
    }
  }
#endif
}

// Separate copies marked by k_grant_prep_cert (rare == 2): 16 lanes per grant,
// lane j compares bytes [16j, 16j + 16) of the grant with its slot leader's
// (offset parked in hash_off[d_base + h]).  A wave takes 256 grants at a time:
// one coalesced load of their flags (a dword per lane), and spans without a
// candidate (every one when a certificate's grants share their bytes) are
// skipped; otherwise each lane stages its four grants' length and offsets in
// LDS (coalesced loads), and the wave compares 4 grants per group over the 64
// four-grant groups that hold a candidate, kMatchUnroll groups at a time with
// their window loads issued together -- one memory round trip per
// kMatchUnroll groups.  Equal: rare = 0 (the leader's results stored by
// prep_cert stand); different: rare = 1.
constexpr uint32_t kMatchUnroll = 4;

struct MatchMeta {
  uint64_t off, lead_off;
  uint32_t len, pad;
};

__global__ __launch_bounds__(256) void k_grant_match(const PrepArgs a, uint8_t* __restrict__ rare) {
  __shared__ MatchMeta meta[4][256];
  const uint32_t lane = threadIdx.x & 63, sub = lane >> 4, piece = lane & 15, wv = threadIdx.x >> 6;
  const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_waves = (gridDim.x * blockDim.x) >> 6;
  MatchMeta* m = meta[wv];
#pragma unroll 1
  for (uint64_t base = (uint64_t)wave * 256; base < a.n; base += (uint64_t)n_waves * 256) {
    const uint64_t g4 = base + 4 * lane;  // this lane's four flags
    uint32_t f = 0;
    if (g4 + 4 <= a.n) {
      f = *(const uint32_t*)(rare + g4);  // rare is 256-byte aligned, base and 4 * lane multiples of 4
    } else {
      for (uint32_t b = 0; b < 4; b++)
        if (g4 + b < a.n) f |= (uint32_t)rare[g4 + b] << (8 * b);
    }
    uint64_t todo = __ballot((f & 0x02020202u) != 0);  // flags are 0, 1 or 2
    if (!todo) continue;
    if (f & 0x02020202u) {  // stage the metadata of this lane's candidates
#pragma unroll
      for (uint32_t b = 0; b < 4; b++)
        if (((f >> (8 * b)) & 0xFFu) == 2) {
          const uint64_t h = g4 + b;
          MatchMeta& e = m[4 * lane + b];
          e.off = a.goff[h];
          e.lead_off = a.hash_off[(size_t)a.d_base + h];
          e.len = a.glen[h];
        }
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll 1
    while (todo) {
      uint32_t q[kMatchUnroll];
#pragma unroll
      for (uint32_t u = 0; u < kMatchUnroll; u++) {
        q[u] = todo ? (uint32_t)__builtin_ctzll(todo) : 64u;
        if (todo) todo &= todo - 1;
      }
      bool cand[kMatchUnroll], diff[kMatchUnroll];
#pragma unroll
      for (uint32_t u = 0; u < kMatchUnroll; u++) {
        const uint32_t fq = q[u] < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)f, (int)q[u]) : 0u;
        cand[u] = ((fq >> (8 * sub)) & 0xFFu) == 2;
        diff[u] = false;
      }
      // all kMatchUnroll groups' window loads before any compare: no branch between
      // them (lanes without a byte to compare read a dummy line of `rare`)
      uint32_t x[kMatchUnroll][4], y[kMatchUnroll][4], len[kMatchUnroll];
      const uint32_t pos = 16 * piece;
#pragma unroll
      for (uint32_t u = 0; u < kMatchUnroll; u++) {
        const MatchMeta& e = m[4 * (q[u] & 63) + sub];
        len[u] = cand[u] ? e.len : 0u;
        const bool valid = pos < len[u];
        const uintptr_t ax = valid ? (uintptr_t)(a.blob + e.off + pos) : (uintptr_t)rare;
        const uintptr_t ay = valid ? (uintptr_t)(a.blob + e.lead_off + pos) : (uintptr_t)rare;
        const uint32_t shx = (uint32_t)(ax & 15), shy = (uint32_t)(ay & 15);
        window16_nb(ax, valid && shx != 0 && pos - shx + 16 < len[u], x[u]);
        window16_nb(ay, valid && shy != 0 && pos - shy + 16 < len[u], y[u]);
      }
#pragma unroll
      for (uint32_t u = 0; u < kMatchUnroll; u++) {
        uint32_t d = 0;
#pragma unroll
        for (int t = 0; t < 4; t++) {
          const int32_t left = (int32_t)(len[u] - pos) - 4 * t;  // len <= pos: every mask 0
          const uint32_t mk = left >= 4 ? ~0u : left <= 0 ? 0u : (1u << (8 * left)) - 1u;
          d |= (x[u][t] ^ y[u][t]) & mk;
        }
        diff[u] = d != 0;
      }
#pragma unroll
      for (uint32_t u = 0; u < kMatchUnroll; u++) {
        const uint64_t dm = __ballot(diff[u]);
        if (cand[u] && piece == 0) rare[base + 4 * q[u] + sub] = ((dm >> (16 * sub)) & 0xFFFFull) ? 1 : 0;
      }
    }
    __builtin_amdgcn_wave_barrier();  // the next span's staging overwrites m
  }
}

// The flagged grants, compacted per block: each block scans kRareSpan flags
// (16 per thread, one 16-byte load), queues the flagged ones in LDS and preps
// them with consecutive lanes -- a few per block, so one prep time per block.
constexpr uint32_t kRareSpan = 4096;

__global__ __launch_bounds__(256) MOCHI_PREP_ATTR void k_grant_prep_rare(const PrepArgs a, const uint8_t* __restrict__ rare) {
  __shared__ uint32_t q[kRareSpan];
  __shared__ uint32_t nq;
  if (threadIdx.x == 0) nq = 0;
  __syncthreads();
  const uint32_t g0 = blockIdx.x * kRareSpan + 16 * threadIdx.x;
  if (g0 < a.n) {
    uint32_t f[4];
    if (g0 + 16 <= a.n) {
      const uint4 v = *(const uint4*)(rare + g0);  // g0 is a multiple of 16: aligned
      f[0] = v.x, f[1] = v.y, f[2] = v.z, f[3] = v.w;
    } else {
      for (int k = 0; k < 4; k++) {
        f[k] = 0;
        for (int b = 0; b < 4; b++)
          if (g0 + 4 * k + b < a.n) f[k] |= (uint32_t)rare[g0 + 4 * k + b] << (8 * b);
      }
    }
    if (f[0] | f[1] | f[2] | f[3]) {
#pragma unroll
      for (int j = 0; j < 16; j++)
        if ((f[j >> 2] >> (8 * (j & 3))) & 0xFFu) q[atomicAdd(&nq, 1u)] = g0 + j;
    }
  }
  __syncthreads();
  const uint32_t n = nq;
#pragma unroll 1
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) grant_prep_one(a, q[i]);
}

// ---------------------------------------------------------------------------
// Signer buckets (kBucketAlign = 512-aligned: one k_rsa_pow block) — counting sort.
// ---------------------------------------------------------------------------
// Wave-aggregated LDS counter add: the lanes of a wave that share a key are
// ranked by ballot and their leader adds the group's size once, so a batch
// with few signers (R = 4) costs a handful of LDS atomics per wave instead of
// 64 same-address ones.  Returns this lane's slot (base + rank in the wave);
// lanes with key == 0xFFFFFFFF take no part.  Must be reached by the whole wave.
__device__ __forceinline__ uint32_t wave_counted_add(uint32_t* __restrict__ lcount, uint32_t key) {
  bool pending = key != 0xFFFFFFFFu;
  uint32_t slot = 0;
  while (true) {
    const uint64_t pm = __ballot(pending);
    if (pm == 0) break;
    const int leader = __ffsll((unsigned long long)pm) - 1;
    const uint32_t k = (uint32_t)__builtin_amdgcn_readlane((int)key, leader);  // scalar, no LDS round trip
    const bool mine = pending && key == k;
    const uint64_t mm = __ballot(mine);
    uint32_t base = 0;
    if ((int)__lane_id() == leader) base = atomicAdd(&lcount[k], (uint32_t)__popcll(mm));
    base = (uint32_t)__builtin_amdgcn_readlane((int)base, leader);
    if (mine) {
      const uint32_t below = __builtin_amdgcn_mbcnt_hi((uint32_t)(mm >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mm, 0u));
      slot = base + below;
      pending = false;
    }
  }
  return slot;
}

__global__ __launch_bounds__(256) void k_bucket_count(const uint16_t* __restrict__ signer, uint32_t n, uint32_t n_keys,
                                                      uint32_t* __restrict__ count) {
  extern __shared__ uint32_t hist[];
  for (uint32_t k = threadIdx.x; k < n_keys; k += blockDim.x) hist[k] = 0;
  __syncthreads();
  // no-return LDS atomics pipeline; the wave-aggregated form (wave_counted_add)
  // measured 65 us vs 17 us here at C2
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t s = signer[i];
    if (s < n_keys) atomicAdd(&hist[s], 1u);
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < n_keys; k += blockDim.x)
    if (hist[k]) atomicAdd(&count[k], hist[k]);
}

// Single block: exclusive scan of round_up(count, kBucketAlign); cursor[k] = start[k].
__global__ __launch_bounds__(256) void k_bucket_scan(const uint32_t* __restrict__ count, uint32_t n_keys,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ total) {
  __shared__ uint32_t part[256];
  const uint32_t per = (n_keys + 255) / 256;
  const uint32_t b = threadIdx.x * per;
  uint32_t s = 0;
  for (uint32_t k = b; k < b + per && k < n_keys; k++) s += (count[k] + kBucketAlign - 1) & ~(kBucketAlign - 1);
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (int t = 0; t < 256; t++) {
      const uint32_t v = part[t];
      part[t] = run;
      run += v;
    }
    total[0] = run;
#pragma unroll
    for (int i = 1; i < kTotalWords; i++) total[i] = 0;  // the counters of this call's later kernels (kernels.h)
  }
  __syncthreads();
  uint32_t run = part[threadIdx.x];
  for (uint32_t k = b; k < b + per && k < n_keys; k++) {
    cursor[k] = run;
    run += (count[k] + kBucketAlign - 1) & ~(kBucketAlign - 1);
  }
}

// Each block places kScatterPer x 256 grants: ranks within the block come from
// wave_counted_add, then ONE global cursor add per (block, signer).  16 per
// thread (3,902 blocks x R cursor adds at C4): the bucket stage 0.175 -> 0.140
// ms against 8 per thread (7,804 blocks), 0.147 at 32 (alternated A/B)
#ifndef MOCHI_SCATTER_PER
#define MOCHI_SCATTER_PER 16
#endif
constexpr uint32_t kScatterPer = MOCHI_SCATTER_PER;

__global__ __launch_bounds__(256) void k_bucket_scatter(const uint16_t* __restrict__ signer, uint32_t n, uint32_t n_keys,
                                                        uint32_t* __restrict__ cursor, uint32_t* __restrict__ perm) {
  extern __shared__ uint32_t lds[];  // [n_keys] local count, then [n_keys] base
  uint32_t* lcount = lds;
  uint32_t* lbase = lds + n_keys;
  for (uint32_t k = threadIdx.x; k < n_keys; k += blockDim.x) lcount[k] = 0;
  __syncthreads();
  const uint32_t i0 = blockIdx.x * (blockDim.x * kScatterPer) + threadIdx.x;
  uint32_t s[kScatterPer], rank[kScatterPer];
#pragma unroll
  for (uint32_t j = 0; j < kScatterPer; j++) {
    const uint32_t i = i0 + j * blockDim.x;
    uint32_t v = i < n ? (uint32_t)signer[i] : 0xFFFFFFFFu;
    s[j] = v < n_keys ? v : 0xFFFFFFFFu;
  }
#pragma unroll
  for (uint32_t j = 0; j < kScatterPer; j++) rank[j] = wave_counted_add(lcount, s[j]);
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < n_keys; k += blockDim.x)
    lbase[k] = lcount[k] ? atomicAdd(&cursor[k], lcount[k]) : 0u;
  __syncthreads();
#pragma unroll
  for (uint32_t j = 0; j < kScatterPer; j++)
    if (s[j] != 0xFFFFFFFFu) perm[lbase[s[j]] + rank[j]] = i0 + j * blockDim.x;
}

// A small batch (a batcher flush: a few messages) in ONE kernel of one block:
// perm cleared, counts, bucket starts, totals and the scatter -- instead of two
// memsets and three kernels, each ~5 us of dispatch on an otherwise idle GPU.
constexpr uint32_t kSmallGrants = 4096;

// prep (n <= kSmallPrepFused): then the per-grant prep of the n grants as
// well, in the same block (one launch fewer; nothing reads the prep's outputs
// before k_rsa_final).
constexpr uint32_t kSmallPrepFused = 1024;

__global__ __launch_bounds__(1024) void k_bucket_small(const uint16_t* __restrict__ signer, uint32_t n, uint32_t n_keys,
                                                       uint32_t n_slots, uint32_t* __restrict__ perm,
                                                       uint32_t* __restrict__ total, const PrepArgs pa,
                                                       uint32_t prep) {
  extern __shared__ uint32_t lds[];  // [n_keys] count, then [n_keys] cursor
  uint32_t* cnt = lds;
  uint32_t* cur = lds + n_keys;
  __shared__ uint32_t part[1024];
  for (uint32_t k = threadIdx.x; k < n_keys; k += blockDim.x) cnt[k] = 0;
  for (uint32_t i = threadIdx.x; i < n_slots; i += blockDim.x) perm[i] = 0xFFFFFFFFu;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t k = signer[i];
    if (k < n_keys) atomicAdd(&cnt[k], 1u);
  }
  __syncthreads();
  // exclusive scan of the 512-aligned bucket sizes: per-thread runs, a shuffle
  // scan per wave, then one over the 16 wave totals (a serial pass of thread 0
  // over the 1024 partials was most of this kernel's time)
  const uint32_t per = (n_keys + blockDim.x - 1) / blockDim.x, b = threadIdx.x * per;
  uint32_t sum = 0;
  for (uint32_t k = b; k < b + per && k < n_keys; k++) sum += (cnt[k] + kBucketAlign - 1) & ~(kBucketAlign - 1);
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t incl = sum;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  if (lane == 63) part[wid] = incl;
  __syncthreads();
  if (wid == 0) {
    const uint32_t nw = blockDim.x >> 6;  // 16 wave totals
    const uint32_t wt = lane < nw ? part[lane] : 0u;
    uint32_t wi = wt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(wi, d, 64);
      if (lane >= (uint32_t)d) wi += y;
    }
    if (lane < nw) part[64 + lane] = wi - wt;  // exclusive
    if (lane == nw - 1) {
      total[0] = wi;
#pragma unroll
      for (int i = 1; i < kTotalWords; i++) total[i] = 0;  // the counters of this call's later kernels (kernels.h)
    }
  }
  __syncthreads();
  uint32_t run = part[64 + wid] + incl - sum;
  for (uint32_t k = b; k < b + per && k < n_keys; k++) {
    cur[k] = run;
    run += (cnt[k] + kBucketAlign - 1) & ~(kBucketAlign - 1);
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    const uint32_t k = signer[i];
    if (k < n_keys) perm[atomicAdd(&cur[k], 1u)] = i;
  }
  if (prep)
    for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) grant_prep_one(pa, i);
}

// ---------------------------------------------------------------------------
// Certificate tally (lane = certificate).  Restates oracle_tally, i.e.
// InMemoryDataStore.java:613-640 then :576-611 (verdict part).
// ---------------------------------------------------------------------------
// 32 words of a 128-byte string at any byte alignment: 33 (or 32) aligned
// word loads issued back to back and funnel-shifted; never touches a word that
// holds no byte of the string.
__device__ __forceinline__ void load128(const uint8_t* p, uint32_t (&w)[32]) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t* wp = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  uint32_t raw[33];
#pragma unroll
  for (int i = 0; i < 32; i++) raw[i] = wp[i];
  raw[32] = sh ? wp[32] : 0u;
#pragma unroll
  for (int i = 0; i < 32; i++) w[i] = (uint32_t)((((uint64_t)raw[i + 1] << 32) | raw[i]) >> (8 * sh));
}

// g0's transactionHash == the expected hash: two 64-byte windows per side
// (bytes_equal, prep_dev.h: 16-byte-aligned dwordx4 loads) instead of load128's
// 33 dword loads per side -- the tally's lane reads its own cache lines, so the
// number of load instructions is what its time follows
#ifndef MOCHI_TALLY_LOAD128
#define MOCHI_TALLY_LOAD128 0  // A/B: the dword-load compare
#endif
__device__ bool hash_matches(const uint8_t* __restrict__ blob, uint64_t off, uint32_t len,
                             const uint8_t* __restrict__ expected) {
  if (len != MOCHI_TXN_HASH_BYTES) return false;
#if MOCHI_TALLY_LOAD128
  uint32_t a[32], e[32];
  load128(blob + off, a);
  load128(expected, e);
  uint32_t diff = 0;
#pragma unroll
  for (int q = 0; q < 32; q++) diff |= a[q] ^ e[q];
  return diff == 0;
#else
  return bytes_equal(blob + off, expected, MOCHI_TXN_HASH_BYTES);
#endif
}

// Everything k_tally reads, by value (one kernel argument block).
struct TallyArgs {
  const uint32_t* cert_grant_off;
  const uint32_t* cert_op_off;
  const uint32_t* cert_mg_off;   // null: a MultiGrant = a maximal run of equal signers
  const uint32_t* mg_grant_off;
  const uint8_t* grant_key;
  const uint16_t* signer;
  const uint8_t* op_key;
  const uint8_t* op_flags;
  const int64_t* op_object_ts;   // null: no stored certificates
  const uint64_t* op_key_off;    // MOCHI_Q_BIND
  const uint32_t* op_key_len;
  const uint8_t* flags;
  const int64_t* ts;
  const uint8_t* blob;
  const uint64_t* grant_off;
  const uint32_t* grant_len;
  const uint64_t* hash_off;  // distinct results, index lead[g] (g without lead)
  const uint32_t* hash_len;
  const uint32_t* lead;
  const uint8_t* expected;
  uint32_t n_certs, majority, strict_gt, quorum_mode;
  uint32_t* accept_bits;
  uint8_t* reason_out;
  uint8_t* fail_op_out;
  uint8_t* op_decision;
  uint32_t* op_g0;
  int64_t* op_ts;
  const uint32_t* op_out_off;
  const uint8_t* msg_status;  // [n_certs] or null: the wire path's message status
};

// MOCHI_Q_BIND: Grant.objectId == the op key it is filed under (op `o`'s
// operand1) and Grant.transactionHash == expected.  Out of line and called with
// plain values: the bind mode is rare, and its Grant parse inlined into k_tally
// would cost every certificate of every mode registers.
__device__ __noinline__ bool grant_bound_at(const uint8_t* gp, uint32_t glen, const uint8_t* k, uint32_t kl,
                                            const uint8_t* expected) {
  ByteReader r;
  r.init(gp, glen);
  int64_t t;
  uint32_t ho, hl, oo, ol;
  if (!parse_grant(r, t, ho, hl, oo, ol)) return false;
  if (ol != kl) return false;
  const uint8_t* id = gp + oo;
#pragma unroll 1
  for (uint32_t i = 0; i < kl; i++)
    if (id[i] != k[i]) return false;
  return hash_matches(gp, ho, hl, expected);
}

// g0's transactionHash == expected, g0's distinct result at d: the leader's
// check (kHashChecked), else the bytes.  kLean (the launch with
// k_grant_prep_cert's checks, no MOCHI_Q_BIND) compares a grant prepped on its
// own -- rare -- 16 bytes at a time; the two-window compare (the other launches:
// the small-batch sequence, whose per-grant prep checks nothing, and the bind
// mode, whose Grant parse is a call) or a call would set k_tally's register count:
// 118 VGPRs and 4 waves per SIMD against 49 and 8 without (the tally waits on
// memory, so its occupancy is its speed).
__device__ __forceinline__ bool hash_matches_lean(const uint8_t* __restrict__ gp, const uint8_t* __restrict__ e) {
  uint32_t diff = 0;
#pragma unroll 1
  for (uint32_t pos = 0; pos < MOCHI_TXN_HASH_BYTES; pos += 16) {
    uint32_t wa[4], wb[4];
    window16(gp, MOCHI_TXN_HASH_BYTES, pos, wa);
    window16(e, MOCHI_TXN_HASH_BYTES, pos, wb);
#pragma unroll
    for (int t = 0; t < 4; t++) diff |= wa[t] ^ wb[t];
  }
  return diff == 0;
}

template <bool kLean>
__device__ __forceinline__ bool g0_hash_matches(const TallyArgs& a, uint32_t d, const uint8_t* expected) {
  const uint32_t hl = a.hash_len[d];
  if (hl & kHashChecked) return (hl & kHashEq) != 0;
  if (!kLean) return hash_matches(a.blob, a.hash_off[d], hl, expected);
  return hl == MOCHI_TXN_HASH_BYTES && hash_matches_lean(a.blob + a.hash_off[d], expected);
}

__device__ __forceinline__ bool grant_bound(const TallyArgs& a, uint32_t g, uint32_t o, const uint8_t* expected) {
  if (!a.op_key_off || !a.op_key_len) return false;
  return grant_bound_at(a.blob + a.grant_off[g], a.grant_len[g], a.blob + a.op_key_off[o], a.op_key_len[o], expected);
}

// Grant g counts toward its key slot's quorum list (reference parity: its
// signature verified -- invalid => absent, InMemoryDataStore.java:622-624 --
// and an op names its slot); MOCHI_Q_BIND / MOCHI_Q_DISTINCT_SIGNERS exclude
// more.  first_op[] is not kept per lane: the op naming slot s is found by scan.
template <bool kLean>
__device__ bool counts(const TallyArgs& a, uint32_t g, uint32_t g_lo, uint32_t o_lo, uint32_t o_hi,
                       const uint8_t* expected) {
  if (!(a.flags[g] & MOCHI_GRANT_SIG_OK)) return false;
  if (a.quorum_mode == 0) return true;  // callers only ask about slots an op names
  const uint32_t s = a.grant_key[g];
  uint32_t fo = 0xFFFFFFFFu;
#pragma unroll 1
  for (uint32_t o = o_lo; o < o_hi; o++)
    if (a.op_key[o] == s) {
      fo = o;
      break;
    }
  if (fo == 0xFFFFFFFFu) return false;  // no op looks this key up
  const bool bind = !kLean && (a.quorum_mode & MOCHI_Q_BIND);
  if (bind && !grant_bound(a, g, fo, expected)) return false;
  if (a.quorum_mode & MOCHI_Q_DISTINCT_SIGNERS) {
    // the first grant of (slot, signer) that passes the other checks counts
#pragma unroll 1
    for (uint32_t q = g_lo; q < g; q++)
      if (a.grant_key[q] == s && a.signer[q] == a.signer[g] && (a.flags[q] & MOCHI_GRANT_SIG_OK) &&
          (!bind || grant_bound(a, q, fo, expected)))
        return false;
  }
  return true;
}

// getCurrentTimestampFromCurrentCertificate on the INCOMING certificate
// (StoreValueObjectContainer.java:175-198, called by applyOperation after
// setCurrentC(wc), InMemoryDataStore.java:533-534): every MultiGrant must hold a
// grant for the key, all with one timestamp.  Signatures play no part.
__device__ bool incoming_cert_ok(const TallyArgs& a, uint32_t c, uint32_t g_lo, uint32_t g_hi, uint32_t s) {
  bool have = false, ok = true;
  int64_t t0 = 0;
  if (a.cert_mg_off && a.mg_grant_off) {
    const uint32_t m_lo = a.cert_mg_off[c], m_hi = a.cert_mg_off[c + 1];
#pragma unroll 1
    for (uint32_t m = m_lo; m < m_hi && ok; m++) {
      bool found = false;
#pragma unroll 1
      for (uint32_t g = a.mg_grant_off[m]; g < a.mg_grant_off[m + 1]; g++) {
        if (a.grant_key[g] != s) continue;
        found = true;
        const int64_t t = a.ts[g];
        if (!have) {
          have = true;
          t0 = t;
        } else if (t != t0) {
          ok = false;
        }
      }
      ok = ok && found;
    }
  } else {
    bool found = true;  // vacuous before the first run
#pragma unroll 1
    for (uint32_t g = g_lo; g < g_hi && ok; g++) {
      if (g == g_lo || a.signer[g] != a.signer[g - 1]) {  // a new MultiGrant starts
        ok = found;
        found = false;
      }
      if (a.grant_key[g] != s) continue;
      found = true;
      const int64_t t = a.ts[g];
      if (!have) {
        have = true;
        t0 = t;
      } else if (t != t0) {
        ok = false;
      }
    }
    ok = ok && found;
  }
  return ok && have;  // no MultiGrant at all: null Long unboxed (NPE)
}

// Certificate tally (lane = certificate).  Restates oracle_tally, i.e.
// InMemoryDataStore.java:613-640 then write2apply :576-611 including the
// read/apply step (:594-599, :521-574).
#ifndef MOCHI_TALLY_WAVES
#define MOCHI_TALLY_WAVES 3  // amdgpu_waves_per_eu: at least 3 (the windowed hash compare needs 122 VGPRs: 4 waves
                             // per SIMD; capped for 5 / 6 waves it spills 36 / 51 and takes 0.63 / 0.65 ms vs 0.54
                             // at C4, round 5; with the dword-load compare it needed 181 and 3 waves was best)
#endif
#if MOCHI_TALLY_WAVES
#define MOCHI_TALLY_ATTR __attribute__((amdgpu_waves_per_eu(MOCHI_TALLY_WAVES)))
#else
#define MOCHI_TALLY_ATTR
#endif
template <bool kLean>
__global__ __launch_bounds__(256) MOCHI_TALLY_ATTR void k_tally(const TallyArgs a) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t reason = MOCHI_ACCEPT, fail_op = 0xFF;
  if (c < a.n_certs) {
    const uint32_t g_lo = a.cert_grant_off[c], g_hi = a.cert_grant_off[c + 1];
    const uint32_t o_lo = a.cert_op_off[c], o_hi = a.cert_op_off[c + 1];
    const uint8_t* expected = a.expected + (size_t)c * MOCHI_TXN_HASH_BYTES;
    for (uint32_t g = g_lo; g < g_hi; g++)
      if (!(a.flags[g] & MOCHI_GRANT_PARSED)) reason = MOCHI_REJECT_MALFORMED;
    // processMultiGrantsFromAllServers: per named key slot, every counted
    // grant's ts must equal the first counted grant's ts (wire order).
    if (reason == MOCHI_ACCEPT) {
      for (uint32_t o = o_lo; o < o_hi && reason == MOCHI_ACCEPT; o++) {
        const uint32_t s = a.op_key[o];
        bool dup = false;
        for (uint32_t q = o_lo; q < o; q++) dup |= a.op_key[q] == s;
        if (dup) continue;
        bool seen = false;
        int64_t ts0 = 0;
        for (uint32_t g = g_lo; g < g_hi; g++) {
          if (a.grant_key[g] != s || !counts<kLean>(a, g, g_lo, o_lo, o_hi, expected)) continue;
          if (!seen) {
            seen = true;
            ts0 = a.ts[g];
          } else if (a.ts[g] != ts0) {
            reason = MOCHI_REJECT_TS_MISMATCH;
          }
        }
      }
    }
    // write2apply, ops in txn order
    uint64_t applied = 0, read = 0, wrong = 0;  // per-op decisions (<= 64 ops)
    if (reason == MOCHI_ACCEPT) {
      for (uint32_t o = o_lo; o < o_hi; o++) {
        const uint32_t j = o - o_lo;
        const uint32_t fl = a.op_flags[o];
        if (!(fl & MOCHI_OP_LOCAL)) {  // WRONG_SHARD  :582-587
          wrong |= 1ull << j;
          continue;
        }
        const uint32_t s = a.op_key[o];
        uint32_t mult = 0;
        bool applied_before = false;
        for (uint32_t q = o_lo; q < o_hi; q++) {
          mult += a.op_key[q] == s;
          if (q < o && a.op_key[q] == s && ((applied >> (q - o_lo)) & 1)) applied_before = true;
        }
        uint32_t valid = 0, first = 0xFFFFFFFFu;
        for (uint32_t g = g_lo; g < g_hi; g++) {
          if (a.grant_key[g] != s || !counts<kLean>(a, g, g_lo, o_lo, o_hi, expected)) continue;
          if (first == 0xFFFFFFFFu) first = g;
          valid++;
        }
        const uint32_t cnt = valid * mult;
        uint32_t why = MOCHI_ACCEPT;
        if (first == 0xFFFFFFFFu) why = MOCHI_REJECT_NO_GRANT;                                      // :588
        else if (!(a.strict_gt ? cnt > a.majority : cnt >= a.majority)) why = MOCHI_REJECT_BELOW_QUORUM;  // :590
        else if (!g0_hash_matches<kLean>(a, a.lead ? a.lead[first] : first, expected))
          why = MOCHI_REJECT_HASH_MISMATCH;                                                       // :591,605-607
        else if (!(fl & MOCHI_OP_HAS_SVOC)) why = MOCHI_REJECT_NO_SVOC;                           // :592-593
        else {
          // objectTS = svoc.getCurrentTimestampFromCurrentCertificate()  :594 (stored
          // certificate: wc itself once an earlier op of this txn applied to the key)
          const int64_t g0_ts = a.ts[first];
          const bool has_cc = applied_before || (fl & MOCHI_OP_HAS_CURRENT_C);
          const bool cc_bad = !applied_before && (fl & MOCHI_OP_CURRENT_C_BAD);
          const int64_t obj_ts = applied_before ? g0_ts : (a.op_object_ts ? a.op_object_ts[o] : 0);
          if (cc_bad) why = MOCHI_REJECT_STORED_CERT;
          else if (fl & MOCHI_OP_NOT_WRITE) why = MOCHI_REJECT_NOT_WRITE;  // lock / action checks
          else if (has_cc && obj_ts > g0_ts) read |= 1ull << j;            // readOperation  :596
          else if (!incoming_cert_ok(a, c, g_lo, g_hi, s)) why = MOCHI_REJECT_APPLY_STATE;  // :533-534
          else applied |= 1ull << j;                                        // applyOperation :597
        }
        if (why != MOCHI_ACCEPT) {
          reason = why;
          fail_op = j;
          break;
        }
      }
    }
    // the wire path's undecoded messages (k_w2_fixup's overrides, done here in
    // the same pass): MALFORMED rejected as such, FALLBACK / OPS_MISMATCH left
    // UNDECIDED for the host's fallback, their wire ops not reached
    const uint32_t ms = a.msg_status ? a.msg_status[c] : (uint32_t)MOCHI_MSG_OK;
    if (ms != MOCHI_MSG_OK) {
      reason = ms == MOCHI_MSG_MALFORMED ? MOCHI_REJECT_MALFORMED : MOCHI_UNDECIDED;
      fail_op = 0xFF;
      if (a.op_out_off)
        for (uint32_t o = a.op_out_off[c]; o < a.op_out_off[c + 1]; o++) {
          if (a.op_decision) a.op_decision[o] = MOCHI_OPD_SKIPPED;
          if (a.op_g0) a.op_g0[o] = 0xFFFFFFFFu;
          if (a.op_ts) a.op_ts[o] = 0;
        }
    }
    if (a.reason_out) a.reason_out[c] = (uint8_t)reason;
    if (a.fail_op_out) a.fail_op_out[c] = (uint8_t)fail_op;
    if (a.op_decision || a.op_g0 || a.op_ts) {
      const uint32_t out0 = a.op_out_off ? a.op_out_off[c] : o_lo;
      for (uint32_t o = o_lo; o < o_hi; o++) {
        const uint32_t j = o - o_lo, s = a.op_key[o];
        uint32_t first = 0xFFFFFFFFu;
        for (uint32_t g = g_lo; g < g_hi && first == 0xFFFFFFFFu; g++)
          if (a.grant_key[g] == s && counts<kLean>(a, g, g_lo, o_lo, o_hi, expected)) first = g;
        uint32_t d = MOCHI_OPD_SKIPPED;
        if ((applied >> j) & 1) d = MOCHI_OPD_APPLY;
        else if ((read >> j) & 1) d = MOCHI_OPD_READ;
        else if ((wrong >> j) & 1) d = MOCHI_OPD_WRONG_SHARD;
        else if (j == fail_op) d = MOCHI_OPD_FAILED;
        if (a.op_decision) a.op_decision[out0 + j] = (uint8_t)d;
        if (a.op_g0) a.op_g0[out0 + j] = first == 0xFFFFFFFFu ? first : first - g_lo;
        if (a.op_ts) a.op_ts[out0 + j] = first == 0xFFFFFFFFu ? 0 : a.ts[first];
      }
    }
  }
  // accept bitmap: one ballot per wave covers 64 certificates = 2 words
  const uint64_t acc = __ballot(c < a.n_certs && reason == MOCHI_ACCEPT);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wbase = (c - lane) >> 5;
  const uint32_t nwords = (a.n_certs + 31) >> 5;
  if (lane == 0 && wbase < nwords) a.accept_bits[wbase] = (uint32_t)acc;
  if (lane == 0 && wbase + 1 < nwords) a.accept_bits[wbase + 1] = (uint32_t)(acc >> 32);
}

__global__ __launch_bounds__(256) void k_pack_bits(const uint8_t* __restrict__ flags, uint32_t n, uint8_t mask,
                                                   uint32_t* __restrict__ bits) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t b = __ballot(i < n && (flags[i] & mask));
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wbase = (i - lane) >> 5;
  const uint32_t nwords = (n + 31) >> 5;
  if (lane == 0 && wbase < nwords) bits[wbase] = (uint32_t)b;
  if (lane == 0 && wbase + 1 < nwords) bits[wbase + 1] = (uint32_t)(b >> 32);
}

// Producer-side fault check: a signature that does not verify under the
// signer's own public key is never released (a faulty RSA-CRT half would leak
// a prime factor: gcd(s^e - EM, n)); it is zeroed and counted.
__global__ __launch_bounds__(256) void k_withhold(const uint8_t* __restrict__ flags, uint32_t n, uint8_t* __restrict__ sig,
                                                  uint32_t* __restrict__ rejected) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || (flags[i] & MOCHI_GRANT_SIG_OK)) return;
  uint4* s = (uint4*)(sig + (size_t)i * MOCHI_RSA_BYTES);
#pragma unroll
  for (int q = 0; q < MOCHI_RSA_BYTES / 16; q++) s[q] = make_uint4(0, 0, 0, 0);
  atomicAdd(rejected, 1u);
}

// ---------------------------------------------------------------------------
// Launchers (host side of this translation unit).
// ---------------------------------------------------------------------------
static inline uint32_t cdiv(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

// MOCHI_NO_DEDUP=1 (A/B): every grant parsed and hashed on its own (k_grant_prep)
static bool dedup_off() {
  static const bool off = [] {
    const char* e = getenv("MOCHI_NO_DEDUP");
    return e && e[0] == '1';
  }();
  return off;
}

// MOCHI_NO_HASH_PRECHECK=1 (A/B): k_tally compares every g0 hash itself
static bool hash_precheck() {
  static const bool on = [] {
    const char* e = getenv("MOCHI_NO_HASH_PRECHECK");
    return !(e && e[0] == '1');
  }();
  return on;
}

// MOCHI_W2_NO_SMALL_SCAN=1 (A/B, with the decoder's): the small-batch prep as a launch of its own
static bool small_scan_off() {
  static const bool off = [] {
    const char* e = getenv("MOCHI_W2_NO_SMALL_SCAN");
    return e && e[0] == '1';
  }();
  return off;
}

// MOCHI_NO_SMALL=1 (A/B): small batches take the large-batch launch sequence
static bool small_off() {
  static const bool off = [] {
    const char* e = getenv("MOCHI_NO_SMALL");
    return e && e[0] == '1';
  }();
  return off;
}

// MOCHI_PREP_FIRST=1 (A/B): grant prep ahead of k_rsa_pow on the main stream
static bool prep_first() {
  static const bool on = [] {
    const char* e = getenv("MOCHI_PREP_FIRST");
    return e && e[0] == '1';
  }();
  return on;
}

hipError_t launch_withhold(const uint8_t* flags, uint32_t n, uint8_t* sig, uint32_t* rejected, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_withhold, dim3(cdiv(n, 256)), dim3(256), 0, st, flags, n, sig, rejected);
  return hipGetLastError();
}

hipError_t launch_pack_bits(const uint8_t* flags, uint32_t n, uint8_t mask, uint32_t* bits, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_pack_bits, dim3(cdiv(n, 256)), dim3(256), 0, st, flags, n, mask, bits);
  return hipGetLastError();
}

hipError_t launch_verify(const LaunchArgs& a, hipStream_t st) {
  const uint32_t N = a.n_grants, C = a.n_certs;
  auto mark = [&](int stage, bool end, hipStream_t s) {
    if (a.prof_events) (void)hipEventRecord(a.prof_events[2 * stage + (end ? 1 : 0)], s);
  };
  // Grant prep (parse + SHA-256) only feeds k_rsa_final and k_tally, so it is
  // forked onto the aux stream after bucketing and joined before k_rsa_final.
  // k_rsa_pow holds every VGPR of the CUs it runs on (2 waves of 256 per SIMD)
  // and is dispatched first, so prep's blocks in fact run in pow's TAIL: on
  // each CU the moment its last pow group is done (the per-CU group counts
  // differ by one) -- measured 0.8 ms a step better than serialised
  // (MOCHI_PREP_SERIAL=1).  Done inside k_rsa_pow's phases instead (one wave
  // per SIMD-half, nothing to hide its latency) it cost the step 5-9 ms
  // (DESIGN.md section 9).  The fork comes after bucketing: beside prep, the
  // short bucket kernels (which gate k_rsa_pow) took ~4x longer.
  // A small batch (<= kSmallGrants): one bucketing kernel, then the per-grant prep
  // on the launch stream -- no fork, no dedup passes (each a dispatch of its own)
  const bool small = N && N <= a.small_grants && N <= kSmallGrants && !small_off();
  // grant dedup (k_grant_prep_cert + k_grant_prep_rare): results stored once per distinct
  // grant, read through `lead`; without it every grant is its own distinct index
  const bool dedup = !small && a.rare && a.lead && a.cert_grant_off && C && !dedup_off();
  const uint32_t nd = a.n_dist ? a.n_dist : N;
  const PrepArgs pa{a.blob,     a.grant_off, a.grant_len, N,        nd,      dedup ? C : 0u,
                    a.digest,   a.ts,        a.hash_off,  a.hash_len, a.flags, dedup ? a.lead : nullptr};
  const uint32_t* lead = dedup ? a.lead : nullptr;
  const bool prep = N && !a.skip_prep_tally;
  const bool fork = prep && a.aux && !small;
  // a small batch of at most kSmallPrepFused grants: the prep inside k_bucket_small
  const bool prep_fused = small && prep && N <= kSmallPrepFused && !small_scan_off();
  hipStream_t ps = fork ? a.aux : st;
  auto bucket = [&](hipStream_t bs) -> hipError_t {
    mark(kStageBucket, false, bs);
    if (small) {
      hipLaunchKernelGGL(k_bucket_small, dim3(1), dim3(1024), 2 * sizeof(uint32_t) * a.n_keys, bs, a.signer, N,
                         a.n_keys, a.n_slots, a.perm, a.total, pa, (uint32_t)prep_fused);
    } else if (N) {
      hipError_t e = hipMemsetAsync(a.count, 0, sizeof(uint32_t) * a.n_keys, bs);
      if (e != hipSuccess) return e;
      e = hipMemsetAsync(a.perm, 0xFF, sizeof(uint32_t) * (size_t)a.n_slots, bs);
      if (e != hipSuccess) return e;
      const uint32_t lds = sizeof(uint32_t) * a.n_keys;
      const uint32_t cblocks = cdiv(N, 256) < 1024 ? cdiv(N, 256) : 1024;
      hipLaunchKernelGGL(k_bucket_count, dim3(cblocks), dim3(256), lds, bs, a.signer, N, a.n_keys, a.count);
      hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(256), 0, bs, a.count, a.n_keys, a.cursor, a.total);
      hipLaunchKernelGGL(k_bucket_scatter, dim3(cdiv(N, 256 * kScatterPer)), dim3(256), 2 * lds, bs, a.signer, N,
                         a.n_keys, a.cursor, a.perm);
    }
    mark(kStageBucket, true, bs);
    return hipSuccess;
  };
  auto grant_prep = [&](hipStream_t ps) -> hipError_t {
    mark(kStagePrep, false, ps);
    if (prep) {
      if (dedup) {
        const PrepCertArgs pc{a.grant_key, a.cert_grant_off, a.grant_same, C, a.rare,
                              hash_precheck() ? a.expected_hash : nullptr};
        hipError_t e = hipMemsetAsync(a.rare, 1, N, ps);
        if (e != hipSuccess) return e;
        hipLaunchKernelGGL(k_grant_prep_cert, dim3(cdiv(C, 256)), dim3(256), 0, ps, pa, pc);
        const uint32_t mblocks = cdiv(N, 4 * 256) < 2048 ? cdiv(N, 4 * 256) : 2048;  // 4 waves x 256 grants
        hipLaunchKernelGGL(k_grant_match, dim3(mblocks), dim3(256), 0, ps, pa, a.rare);
        hipLaunchKernelGGL(k_grant_prep_rare, dim3(cdiv(N, kRareSpan)), dim3(256), 0, ps, pa, (const uint8_t*)a.rare);
      } else if (!prep_fused) {
        hipLaunchKernelGGL(k_grant_prep, dim3(cdiv(N, 256)), dim3(256), 0, ps, pa);
      }
    }
    mark(kStagePrep, true, ps);
    return hipSuccess;
  };
  if (fork && prep_first()) {
    // A/B (MOCHI_PREP_FIRST=1): prep on the main stream ahead of pow, the short
    // bucket kernels beside it on the aux stream
    hipError_t e = hipEventRecord(a.ev_fork, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(a.aux, a.ev_fork, 0);
    if (e == hipSuccess) e = bucket(a.aux);
    if (e == hipSuccess) e = hipEventRecord(a.ev_join, a.aux);
    if (e == hipSuccess) e = grant_prep(st);
    if (e == hipSuccess) e = hipStreamWaitEvent(st, a.ev_join, 0);
    if (e != hipSuccess) return e;
    mark(kStagePow, false, st);
    if (N) launch_rsa_pow(a, st, small);
    mark(kStagePow, true, st);
  } else {
    hipError_t e = bucket(st);
    if (e != hipSuccess) return e;
    if (fork) {
      e = hipEventRecord(a.ev_fork, st);
      if (e == hipSuccess) e = hipStreamWaitEvent(a.aux, a.ev_fork, 0);
      if (e != hipSuccess) return e;
    }
    e = grant_prep(ps);
    if (e != hipSuccess) return e;
    if (fork) {
      e = hipEventRecord(a.ev_join, a.aux);
      if (e != hipSuccess) return e;
    }
    mark(kStagePow, false, st);
    if (N) launch_rsa_pow(a, st, small);
    mark(kStagePow, true, st);
    if (fork) {
      e = hipStreamWaitEvent(st, a.ev_join, 0);
      if (e != hipSuccess) return e;
    }
  }
  mark(kStageFinal, false, st);
  if (N) {
    launch_rsa_final(a, lead, nd, st, small);
    if (a.grant_valid_bits)
      hipLaunchKernelGGL(k_pack_bits, dim3(cdiv(N, 256)), dim3(256), 0, st, a.flags, N, (uint8_t)MOCHI_GRANT_SIG_OK,
                         a.grant_valid_bits);
  }
  mark(kStageFinal, true, st);
  mark(kStageTally, false, st);
  if (C && !a.skip_prep_tally) {
    TallyArgs t;
    t.cert_grant_off = a.cert_grant_off;
    t.cert_op_off = a.cert_op_off;
    t.cert_mg_off = a.cert_mg_off;
    t.mg_grant_off = a.mg_grant_off;
    t.grant_key = a.grant_key;
    t.signer = a.signer;
    t.op_key = a.op_key;
    t.op_flags = a.op_flags;
    t.op_object_ts = a.op_object_ts;
    t.op_key_off = a.op_key_off;
    t.op_key_len = a.op_key_len;
    t.flags = a.flags;
    t.ts = a.ts;
    t.blob = a.blob;
    t.grant_off = a.grant_off;
    t.grant_len = a.grant_len;
    t.hash_off = a.hash_off;
    t.hash_len = a.hash_len;
    t.lead = lead;
    t.expected = a.expected_hash;
    t.n_certs = C;
    t.majority = a.majority;
    t.strict_gt = a.strict_gt;
    t.quorum_mode = a.quorum_mode;
    t.accept_bits = a.cert_accept_bits;
    t.reason_out = a.cert_reason;
    t.fail_op_out = a.cert_fail_op;
    t.op_decision = a.op_decision;
    t.op_g0 = a.op_g0;
    t.op_ts = a.op_ts;
    t.op_out_off = a.op_out_off;
    t.msg_status = a.msg_status;
    // lean: every slot leader's hash checked in k_grant_prep_cert, no bind mode
    if (dedup && hash_precheck() && !(a.quorum_mode & MOCHI_Q_BIND))
      hipLaunchKernelGGL(k_tally<true>, dim3(cdiv(C, 256)), dim3(256), 0, st, t);
    else
      hipLaunchKernelGGL(k_tally<false>, dim3(cdiv(C, 256)), dim3(256), 0, st, t);
  }
  mark(kStageTally, true, st);
  return hipGetLastError();
}

}  // namespace mochi
