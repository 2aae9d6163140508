// sha256_dev.h — SHA-256 (FIPS 180-4) of one lane's byte string, shared by the
// grant-prep kernel (kernels.hip) and the device signer (rsa_sign.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mochi {

// ---------------------------------------------------------------------------
// SHA-256 (FIPS 180-4) over one lane's grant bytes.
// ---------------------------------------------------------------------------
static __constant__ uint32_t kSha256K[64] = {
    0x428a2f98, 0x71374491, 0xb5c0fbcf, 0xe9b5dba5, 0x3956c25b, 0x59f111f1, 0x923f82a4, 0xab1c5ed5,
    0xd807aa98, 0x12835b01, 0x243185be, 0x550c7dc3, 0x72be5d74, 0x80deb1fe, 0x9bdc06a7, 0xc19bf174,
    0xe49b69c1, 0xefbe4786, 0x0fc19dc6, 0x240ca1cc, 0x2de92c6f, 0x4a7484aa, 0x5cb0a9dc, 0x76f988da,
    0x983e5152, 0xa831c66d, 0xb00327c8, 0xbf597fc7, 0xc6e00bf3, 0xd5a79147, 0x06ca6351, 0x14292967,
    0x27b70a85, 0x2e1b2138, 0x4d2c6dfc, 0x53380d13, 0x650a7354, 0x766a0abb, 0x81c2c92e, 0x92722c85,
    0xa2bfe8a1, 0xa81a664b, 0xc24b8b70, 0xc76c51a3, 0xd192e819, 0xd6990624, 0xf40e3585, 0x106aa070,
    0x19a4c116, 0x1e376c08, 0x2748774c, 0x34b0bcb5, 0x391c0cb3, 0x4ed8aa4a, 0x5b9cca4f, 0x682e6ff3,
    0x748f82ee, 0x78a5636f, 0x84c87814, 0x8cc70208, 0x90befffa, 0xa4506ceb, 0xbef9a3f7, 0xc67178f2};

__device__ __forceinline__ uint32_t sha_rotr(uint32_t x, int n) { return __builtin_amdgcn_alignbit(x, x, n); }
// a ^ b ^ c in one v_bitop3_b32 (truth table 0x96; hipcc forms bitop3 for
// ch / maj but leaves a three-way XOR as two v_xor_b32)
__device__ __forceinline__ uint32_t sha_xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// One compression of the 16 big-endian words w into h.
__device__ __forceinline__ void sha256_compress(uint32_t (&h)[8], uint32_t (&w)[16]) {
  uint32_t a = h[0], b = h[1], c = h[2], d = h[3], e = h[4], f = h[5], g = h[6], hh = h[7];
#pragma unroll
  for (int t = 0; t < 64; t++) {
    uint32_t wt;
    if (t < 16) {
      wt = w[t];
    } else {
      const uint32_t w15 = w[(t - 15) & 15], w2 = w[(t - 2) & 15];
      const uint32_t s0 = sha_xor3(sha_rotr(w15, 7), sha_rotr(w15, 18), w15 >> 3);
      const uint32_t s1 = sha_xor3(sha_rotr(w2, 17), sha_rotr(w2, 19), w2 >> 10);
      wt = w[t & 15] + s0 + w[(t - 7) & 15] + s1;
      w[t & 15] = wt;
    }
    const uint32_t S1 = sha_xor3(sha_rotr(e, 6), sha_rotr(e, 11), sha_rotr(e, 25));
    const uint32_t ch = (e & f) ^ (~e & g);
    const uint32_t t1 = hh + S1 + ch + kSha256K[t] + wt;
    const uint32_t S0 = sha_xor3(sha_rotr(a, 2), sha_rotr(a, 13), sha_rotr(a, 22));
    const uint32_t mj = (a & b) ^ (a & c) ^ (b & c);
    const uint32_t t2 = S0 + mj;
    hh = g; g = f; f = e; e = d + t1; d = c; c = b; b = a; a = t1 + t2;
  }
  h[0] += a; h[1] += b; h[2] += c; h[3] += d; h[4] += e; h[5] += f; h[6] += g; h[7] += hh;
}

// The 16 message words of block `blk` of the padded message (FIPS 180-4 5.1.1)
// of the `len` bytes at `base` (any alignment).  The block's bytes come from
// 16-byte-aligned dwordx4 loads -- 4 or 5 per block instead of two dword loads
// and a branch per word -- each issued only if its 16 bytes hold a message
// byte (so it stays inside the page of a valid byte: the blob may be a slice
// of a wire buffer), then a per-lane dword rotation (two selects per word,
// base & 15 is the same for every block), a funnel shift and a byte swap.
// Words at or past the end take the padding: data bytes, 0x80, zeros, and
// the 64-bit bit length (len < 2^29) in the last two words of the last block.
// hib (optional): += the bytes with their high bit set among the 64 (padding
// included: the 0x80 byte and the bit length count too) -- the grant prep's
// ASCII check rides on these words (prep_dev.h grant_prep_fast)
__device__ __forceinline__ void sha256_block_words(const uint8_t* base, uint32_t len, uint32_t blk, uint32_t total,
                                                   uint32_t (&w)[16], uint32_t* hib = nullptr) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const uintptr_t addr = (uintptr_t)base + 64u * blk;
  const v4u* a16 = (const v4u*)(addr & ~(uintptr_t)15);
  const uint32_t sh = (uint32_t)(addr & 15);
  const int64_t p0 = (int64_t)(64u * blk) - sh;  // message position of the first loaded byte
  uint32_t d[20];
#pragma unroll
  for (int c = 0; c < 5; c++) {
    v4u v = {0u, 0u, 0u, 0u};
    if (len != 0 && p0 + 16 * c < (int64_t)len && (c < 4 || sh != 0)) v = a16[c];
    d[4 * c] = v.x;
    d[4 * c + 1] = v.y;
    d[4 * c + 2] = v.z;
    d[4 * c + 3] = v.w;
  }
  // e[j] = d[j + (sh >> 2)], j = 0..16, as two rounds of mask selects (a
  // ternary here is turned into a dynamically indexed array in scratch)
  const uint32_t m4 = 0u - ((sh >> 2) & 1u), m8 = 0u - ((sh >> 3) & 1u);
  uint32_t e1[19], e[17];
#pragma unroll
  for (int j = 0; j < 19; j++) e1[j] = (d[j + 1] & m4) | (d[j] & ~m4);
#pragma unroll
  for (int j = 0; j < 17; j++) e[j] = (e1[j + 2] & m8) | (e1[j] & ~m8);
  const uint32_t r = 8 * (sh & 3);
  // every lane's block is all message bytes (the common case): no padding work
  const bool full = __ballot(64u * blk + 64 > len) == 0;
#pragma unroll
  for (int t = 0; t < 16; t++) {
    const uint32_t le = __builtin_amdgcn_alignbit(e[t + 1], e[t], r);
    uint32_t v = __builtin_bswap32(le);
    if (!full) {
      const uint32_t p = 64u * blk + 4u * t;
      if (p + 8 == total) {
        v = 0;  // high half of the bit length
      } else if (p + 4 == total) {
        v = len << 3;
      } else if (p + 4 > len) {
        // n data bytes (0..3), then 0x80 if the message ends inside this word
        const uint32_t n = p < len ? len - p : 0;
        const uint32_t keep = n ? ~0u << (32 - 8 * n) : 0u;
        v = (v & keep) | (p + n == len ? 0x80u << (24 - 8 * n) : 0u);
      }
    }
    w[t] = v;
    if (hib) *hib = __builtin_popcount(v & 0x80808080u) + *hib;  // v_bcnt_u32_b32 with its add
  }
}

__device__ inline void sha256(const uint8_t* base, uint32_t len, uint32_t (&h)[8], uint32_t* hib = nullptr) {
  h[0] = 0x6a09e667; h[1] = 0xbb67ae85; h[2] = 0x3c6ef372; h[3] = 0xa54ff53a;
  h[4] = 0x510e527f; h[5] = 0x9b05688c; h[6] = 0x1f83d9ab; h[7] = 0x5be0cd19;
  const uint32_t nblocks = (len + 9 + 63) >> 6;
  const uint32_t total = nblocks << 6;
#pragma unroll 1
  for (uint32_t blk = 0; blk < nblocks; blk++) {
    uint32_t w[16];
    sha256_block_words(base, len, blk, total, w, hib);
    sha256_compress(h, w);
  }
}

}  // namespace mochi
