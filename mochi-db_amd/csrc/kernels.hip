// kernels.hip — the Write2 certificate-verification hot path on gfx950.
//
//   k_grant_prep    per grant (certificate order): proto3 Grant parse
//                   (MochiProtocol.java:7369-7425 semantics) + SHA-256 of the
//                   grant bytes (the signed message)
//   k_bucket_*      counting sort of grants by signer into 64-aligned buckets,
//                   so every wavefront of the RSA kernels has ONE modulus
//                   (wave-uniform -> scalar loads / SGPR operands)
//   k_rsa_pow       X = (s * R)^(2^16) in Montgomery form (1 mul + 16 sqr)
//   k_rsa_final     Y = X * s * R^-1 = s^65537 mod n; compare with the
//                   EMSA-PKCS1-v1_5 encoding of SHA-256(grant); s < n check
//   k_tally         per certificate: processMultiGrantsFromAllServers +
//                   write2apply verdict (InMemoryDataStore.java:576-640)
//   k_pack_bits     grant-valid bitmap via wavefront ballot
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/mochi_hip.h"
#include "kernels.h"
#include "proto_dev.h"
#include "sha256_dev.h"

namespace mochi {


// ---------------------------------------------------------------------------
// k_grant_prep: parse + SHA-256, certificate order (lane = grant).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_grant_prep(const uint8_t* __restrict__ blob, const uint64_t* __restrict__ goff,
                                                    const uint32_t* __restrict__ glen, uint32_t n,
                                                    uint32_t* __restrict__ digest /* [8][n] */,
                                                    int64_t* __restrict__ ts_out, uint32_t* __restrict__ hash_at /* [n] abs off lo */,
                                                    uint64_t* __restrict__ hash_off_out, uint32_t* __restrict__ hash_len_out,
                                                    uint8_t* __restrict__ flags) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = blob + goff[i];
  const uint32_t l = glen[i];
  ByteReader r;
  r.init(p, l);
  int64_t ts = 0;
  uint32_t hoff = 0, hlen = 0;
  const bool ok = parse_grant(r, ts, hoff, hlen);
  uint32_t h[8];
  sha256(p, l, h);
#pragma unroll
  for (int q = 0; q < 8; q++) digest[(size_t)q * n + i] = h[q];
  ts_out[i] = ok ? ts : 0;
  hash_off_out[i] = goff[i] + hoff;
  hash_len_out[i] = ok ? hlen : 0xFFFFFFFFu;
  flags[i] = ok ? MOCHI_GRANT_PARSED : 0;
  (void)hash_at;
}

// ---------------------------------------------------------------------------
// Signer buckets (64-aligned) — counting sort.
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

// Single block: exclusive scan of round_up(count, 64); cursor[k] = start[k].
__global__ __launch_bounds__(256) void k_bucket_scan(const uint32_t* __restrict__ count, uint32_t n_keys,
                                                     uint32_t* __restrict__ cursor, uint32_t* __restrict__ total) {
  __shared__ uint32_t part[256];
  const uint32_t per = (n_keys + 255) / 256;
  const uint32_t b = threadIdx.x * per;
  uint32_t s = 0;
  for (uint32_t k = b; k < b + per && k < n_keys; k++) s += (count[k] + 63u) & ~63u;
  part[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (int t = 0; t < 256; t++) {
      const uint32_t v = part[t];
      part[t] = run;
      run += v;
    }
    *total = run;
  }
  __syncthreads();
  uint32_t run = part[threadIdx.x];
  for (uint32_t k = b; k < b + per && k < n_keys; k++) {
    cursor[k] = run;
    run += (count[k] + 63u) & ~63u;
  }
}

// Each block places kScatterPer x 256 grants: ranks within the block come from
// wave_counted_add, then ONE global cursor add per (block, signer) — 489
// blocks x R adds at C2 instead of 3,906 x R.
constexpr uint32_t kScatterPer = 8;

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

__device__ bool hash_matches(const uint8_t* __restrict__ blob, uint64_t off, uint32_t len,
                             const uint8_t* __restrict__ expected) {
  if (len != MOCHI_TXN_HASH_BYTES) return false;
  uint32_t a[32], e[32];
  load128(blob + off, a);
  load128(expected, e);
  uint32_t diff = 0;
#pragma unroll
  for (int q = 0; q < 32; q++) diff |= a[q] ^ e[q];
  return diff == 0;
}

__global__ __launch_bounds__(256) void k_tally(const uint32_t* __restrict__ cert_grant_off,
                                               const uint32_t* __restrict__ cert_op_off,
                                               const uint8_t* __restrict__ grant_key, const uint8_t* __restrict__ op_key,
                                               const uint8_t* __restrict__ op_flags, const uint8_t* __restrict__ flags,
                                               const int64_t* __restrict__ ts, const uint8_t* __restrict__ blob,
                                               const uint64_t* __restrict__ hash_off, const uint32_t* __restrict__ hash_len,
                                               const uint8_t* __restrict__ expected, uint32_t n_certs, uint32_t majority,
                                               uint32_t strict_gt, uint32_t* __restrict__ accept_bits,
                                               uint8_t* __restrict__ reason_out, uint8_t* __restrict__ fail_op_out) {
  const uint32_t c = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t reason = MOCHI_ACCEPT, fail_op = 0xFF;
  if (c < n_certs) {
    const uint32_t g_lo = cert_grant_off[c], g_hi = cert_grant_off[c + 1];
    const uint32_t o_lo = cert_op_off[c], o_hi = cert_op_off[c + 1];
    for (uint32_t g = g_lo; g < g_hi; g++)
      if (!(flags[g] & MOCHI_GRANT_PARSED)) reason = MOCHI_REJECT_MALFORMED;
    // processMultiGrantsFromAllServers: per named key slot, every valid grant's
    // ts must equal the first valid grant's ts (wire order).
    if (reason == MOCHI_ACCEPT) {
      for (uint32_t o = o_lo; o < o_hi && reason == MOCHI_ACCEPT; o++) {
        const uint32_t s = op_key[o];
        bool dup = false;
        for (uint32_t q = o_lo; q < o; q++) dup |= op_key[q] == s;
        if (dup) continue;
        bool seen = false;
        int64_t ts0 = 0;
        for (uint32_t g = g_lo; g < g_hi; g++) {
          if (!(flags[g] & MOCHI_GRANT_SIG_OK) || grant_key[g] != s) continue;
          if (!seen) {
            seen = true;
            ts0 = ts[g];
          } else if (ts[g] != ts0) {
            reason = MOCHI_REJECT_TS_MISMATCH;
          }
        }
      }
    }
    // write2apply verdict, ops in txn order
    if (reason == MOCHI_ACCEPT) {
      for (uint32_t o = o_lo; o < o_hi; o++) {
        const uint32_t fl = op_flags[o];
        if (!(fl & MOCHI_OP_LOCAL)) continue;
        const uint32_t s = op_key[o];
        uint32_t mult = 0;
        for (uint32_t q = o_lo; q < o_hi; q++) mult += op_key[q] == s;
        uint32_t valid = 0, first = 0xFFFFFFFFu;
        for (uint32_t g = g_lo; g < g_hi; g++) {
          if (!(flags[g] & MOCHI_GRANT_SIG_OK) || grant_key[g] != s) continue;
          if (first == 0xFFFFFFFFu) first = g;
          valid++;
        }
        const uint32_t cnt = valid * mult;
        uint32_t why = MOCHI_ACCEPT;
        if (first == 0xFFFFFFFFu) why = MOCHI_REJECT_NO_GRANT;
        else if (!(strict_gt ? cnt > majority : cnt >= majority)) why = MOCHI_REJECT_BELOW_QUORUM;
        else if (!hash_matches(blob, hash_off[first], hash_len[first], expected + (size_t)c * MOCHI_TXN_HASH_BYTES))
          why = MOCHI_REJECT_HASH_MISMATCH;
        else if (!(fl & MOCHI_OP_HAS_SVOC)) why = MOCHI_REJECT_NO_SVOC;
        if (why != MOCHI_ACCEPT) {
          reason = why;
          fail_op = o - o_lo;
          break;
        }
      }
    }
    if (reason_out) reason_out[c] = (uint8_t)reason;
    if (fail_op_out) fail_op_out[c] = (uint8_t)fail_op;
  }
  // accept bitmap: one ballot per wave covers 64 certificates = 2 words
  const uint64_t acc = __ballot(c < n_certs && reason == MOCHI_ACCEPT);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wbase = (c - lane) >> 5;
  const uint32_t nwords = (n_certs + 31) >> 5;
  if (lane == 0 && wbase < nwords) accept_bits[wbase] = (uint32_t)acc;
  if (lane == 0 && wbase + 1 < nwords) accept_bits[wbase + 1] = (uint32_t)(acc >> 32);
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

// ---------------------------------------------------------------------------
// Launchers (host side of this translation unit).
// ---------------------------------------------------------------------------
static inline uint32_t cdiv(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

hipError_t launch_pack_bits(const uint8_t* flags, uint32_t n, uint8_t mask, uint32_t* bits, hipStream_t st) {
  if (n) hipLaunchKernelGGL(k_pack_bits, dim3(cdiv(n, 256)), dim3(256), 0, st, flags, n, mask, bits);
  return hipGetLastError();
}

hipError_t launch_verify(const LaunchArgs& a, hipStream_t st) {
  const uint32_t N = a.n_grants, C = a.n_certs;
  auto mark = [&](int stage, bool end, hipStream_t s) {
    if (a.prof_events) (void)hipEventRecord(a.prof_events[2 * stage + (end ? 1 : 0)], s);
  };
  // grant prep (parse + SHA-256) only feeds k_rsa_final and k_tally, so it runs
  // beside k_rsa_pow on the aux stream and fills its idle issue slots (it is
  // latency-bound); the launch stream joins it before k_rsa_final.  It forks
  // AFTER bucketing: run beside prep, the short bucket kernels (which gate
  // k_rsa_pow) took ~4x longer
  const bool prep = N && !a.skip_prep_tally;
  const bool fork = prep && a.aux;
  hipStream_t ps = fork ? a.aux : st;
  mark(kStageBucket, false, st);
  if (N) {
    hipError_t e = hipMemsetAsync(a.count, 0, sizeof(uint32_t) * a.n_keys, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(a.perm, 0xFF, sizeof(uint32_t) * (size_t)a.n_slots, st);
    if (e != hipSuccess) return e;
    const uint32_t lds = sizeof(uint32_t) * a.n_keys;
    const uint32_t cblocks = cdiv(N, 256) < 1024 ? cdiv(N, 256) : 1024;
    hipLaunchKernelGGL(k_bucket_count, dim3(cblocks), dim3(256), lds, st, a.signer, N, a.n_keys, a.count);
    hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(256), 0, st, a.count, a.n_keys, a.cursor, a.total);
    hipLaunchKernelGGL(k_bucket_scatter, dim3(cdiv(N, 256 * kScatterPer)), dim3(256), 2 * lds, st, a.signer, N, a.n_keys, a.cursor,
                       a.perm);
  }
  mark(kStageBucket, true, st);
  if (fork) {
    hipError_t e = hipEventRecord(a.ev_fork, st);
    if (e == hipSuccess) e = hipStreamWaitEvent(a.aux, a.ev_fork, 0);
    if (e != hipSuccess) return e;
  }
  mark(kStagePrep, false, ps);
  if (prep)
    hipLaunchKernelGGL(k_grant_prep, dim3(cdiv(N, 256)), dim3(256), 0, ps, a.blob, a.grant_off, a.grant_len, N,
                       a.digest, a.ts, nullptr, a.hash_off, a.hash_len, a.flags);
  mark(kStagePrep, true, ps);
  if (fork) {
    hipError_t e = hipEventRecord(a.ev_join, a.aux);
    if (e != hipSuccess) return e;
  }
  mark(kStagePow, false, st);
  if (N) launch_rsa_pow(a, st);
  mark(kStagePow, true, st);
  if (fork) {
    hipError_t e = hipStreamWaitEvent(st, a.ev_join, 0);
    if (e != hipSuccess) return e;
  }
  mark(kStageFinal, false, st);
  if (N) {
    launch_rsa_final(a, st);
    if (a.grant_valid_bits)
      hipLaunchKernelGGL(k_pack_bits, dim3(cdiv(N, 256)), dim3(256), 0, st, a.flags, N, (uint8_t)MOCHI_GRANT_SIG_OK,
                         a.grant_valid_bits);
  }
  mark(kStageFinal, true, st);
  mark(kStageTally, false, st);
  if (C && !a.skip_prep_tally)
    hipLaunchKernelGGL(k_tally, dim3(cdiv(C, 256)), dim3(256), 0, st, a.cert_grant_off, a.cert_op_off, a.grant_key,
                       a.op_key, a.op_flags, a.flags, a.ts, a.blob, a.hash_off, a.hash_len, a.expected_hash, C,
                       a.majority, a.strict_gt, a.cert_accept_bits, a.cert_reason, a.cert_fail_op);
  mark(kStageTally, true, st);
  return hipGetLastError();
}

}  // namespace mochi
