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

namespace mochi {

// ---------------------------------------------------------------------------
// SHA-256 (FIPS 180-4) over one lane's grant bytes.
// ---------------------------------------------------------------------------
__constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_bswap32(x); }

// Big-endian message word at byte position p (multiple of 4) of the padded message.
__device__ __forceinline__ uint32_t sha_word(const uint8_t* base, uint32_t p, uint32_t len, uint32_t total) {
  if (p + 4 <= len) {
    const uintptr_t addr = (uintptr_t)(base + p);
    const uint32_t* wp = (const uint32_t*)(addr & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(addr & 3);
    const uint32_t w0 = wp[0];
    const uint32_t w1 = sh ? wp[1] : 0u;  // holds message byte p+3 when sh != 0
    const uint32_t le = (uint32_t)((((uint64_t)w1 << 32) | w0) >> (8 * sh));
    return bswap32(le);
  }
  if (p + 8 == total) return 0;  // high half of the 64-bit bit length (len < 2^29)
  if (p + 4 == total) return len << 3;
  uint32_t v = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t i = p + q;
    uint32_t byte = 0;
    if (i < len) byte = base[i];
    else if (i == len) byte = 0x80;
    v = (v << 8) | byte;
  }
  return v;
}

__device__ void sha256(const uint8_t* base, uint32_t len, uint32_t (&h)[8]) {
  h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
  h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
  const uint32_t nblocks = (len + 9 + 63) >> 6;
  const uint32_t total = nblocks << 6;
#pragma unroll 1
  for (uint32_t blk = 0; blk < nblocks; blk++) {
    uint32_t w[16];
#pragma unroll
    for (int t = 0; t < 16; t++) w[t] = sha_word(base, blk * 64 + 4 * t, len, total);
    uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
    for (int t = 0; t < 64; t++) {
      uint32_t wt;
      if (t < 16) {
        wt = w[t];
      } else {
        const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
        const uint32_t s0 = rotr(w15, 7) ^ rotr(w15, 18) ^ (w15 >> 3);
        const uint32_t s1 = rotr(w2, 17) ^ rotr(w2, 19) ^ (w2 >> 10);
        wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
        w[t & 15] = wt;
      }
      const uint32_t S1 = rotr(e, 6) ^ rotr(e, 11) ^ rotr(e, 25);
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = hh + S1 + ch + kSha256K[t] + wt;
      const uint32_t S0 = rotr(a, 2) ^ rotr(a, 13) ^ rotr(a, 22);
      const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
      const uint32_t t2 = S0 + mj;
      hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
    }
    h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
  }
}

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
__global__ __launch_bounds__(256) void k_bucket_count(const uint16_t* __restrict__ signer, uint32_t n, uint32_t n_keys,
                                                      uint32_t* __restrict__ count) {
  extern __shared__ uint32_t hist[];
  for (uint32_t k = threadIdx.x; k < n_keys; k += blockDim.x) hist[k] = 0;
  __syncthreads();
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

__global__ __launch_bounds__(256) void k_bucket_scatter(const uint16_t* __restrict__ signer, uint32_t n, uint32_t n_keys,
                                                        uint32_t* __restrict__ cursor, uint32_t* __restrict__ perm) {
  extern __shared__ uint32_t lds[];  // [n_keys] local count, then [n_keys] base
  uint32_t* lcount = lds;
  uint32_t* lbase = lds + n_keys;
  for (uint32_t k = threadIdx.x; k < n_keys; k += blockDim.x) lcount[k] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t s = 0xFFFFFFFFu, rank = 0;
  if (i < n) {
    s = signer[i];
    if (s < n_keys) rank = atomicAdd(&lcount[s], 1u);
    else s = 0xFFFFFFFFu;
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < n_keys; k += blockDim.x)
    lbase[k] = lcount[k] ? atomicAdd(&cursor[k], lcount[k]) : 0u;
  __syncthreads();
  if (s != 0xFFFFFFFFu) perm[lbase[s] + rank] = i;
}

// ---------------------------------------------------------------------------
// Certificate tally (lane = certificate).  Restates oracle_tally, i.e.
// InMemoryDataStore.java:613-640 then :576-611 (verdict part).
// ---------------------------------------------------------------------------
__device__ bool hash_matches(const uint8_t* __restrict__ blob, uint64_t off, uint32_t len,
                             const uint8_t* __restrict__ expected) {
  if (len != MOCHI_TXN_HASH_BYTES) return false;
  const uint8_t* p = blob + off;
  uint32_t diff = 0;
#pragma unroll 4
  for (int q = 0; q < MOCHI_TXN_HASH_BYTES / 4; q++) {
    const uint32_t a = sha_word(p, 4 * q, MOCHI_TXN_HASH_BYTES, 0xFFFFFFFFu);
    const uint32_t e = sha_word(expected, 4 * q, MOCHI_TXN_HASH_BYTES, 0xFFFFFFFFu);
    diff |= a ^ e;
  }
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
  auto mark = [&](int i) {
    if (a.prof_events) (void)hipEventRecord(a.prof_events[i], st);
  };
  mark(0);
  if (N && !a.skip_prep_tally)
    hipLaunchKernelGGL(k_grant_prep, dim3(cdiv(N, 256)), dim3(256), 0, st, a.blob, a.grant_off, a.grant_len, N,
                       a.digest, a.ts, nullptr, a.hash_off, a.hash_len, a.flags);
  mark(1 + kStagePrep);
  if (N) {
    hipError_t e = hipMemsetAsync(a.count, 0, sizeof(uint32_t) * a.n_keys, st);
    if (e != hipSuccess) return e;
    e = hipMemsetAsync(a.perm, 0xFF, sizeof(uint32_t) * (size_t)a.n_slots, st);
    if (e != hipSuccess) return e;
    const uint32_t lds = sizeof(uint32_t) * a.n_keys;
    const uint32_t cblocks = cdiv(N, 256) < 1024 ? cdiv(N, 256) : 1024;
    hipLaunchKernelGGL(k_bucket_count, dim3(cblocks), dim3(256), lds, st, a.signer, N, a.n_keys, a.count);
    hipLaunchKernelGGL(k_bucket_scan, dim3(1), dim3(256), 0, st, a.count, a.n_keys, a.cursor, a.total);
    hipLaunchKernelGGL(k_bucket_scatter, dim3(cdiv(N, 256)), dim3(256), 2 * lds, st, a.signer, N, a.n_keys, a.cursor,
                       a.perm);
  }
  mark(1 + kStageBucket);
  if (N) launch_rsa_pow(a, st);
  mark(1 + kStagePow);
  if (N) {
    launch_rsa_final(a, st);
    if (a.grant_valid_bits)
      hipLaunchKernelGGL(k_pack_bits, dim3(cdiv(N, 256)), dim3(256), 0, st, a.flags, N, (uint8_t)MOCHI_GRANT_SIG_OK,
                         a.grant_valid_bits);
  }
  mark(1 + kStageFinal);
  if (C && !a.skip_prep_tally)
    hipLaunchKernelGGL(k_tally, dim3(cdiv(C, 256)), dim3(256), 0, st, a.cert_grant_off, a.cert_op_off, a.grant_key,
                       a.op_key, a.op_flags, a.flags, a.ts, a.blob, a.hash_off, a.hash_len, a.expected_hash, C,
                       a.majority, a.strict_gt, a.cert_accept_bits, a.cert_reason, a.cert_fail_op);
  mark(1 + kStageTally);
  return hipGetLastError();
}

}  // namespace mochi
