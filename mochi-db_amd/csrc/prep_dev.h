// prep_dev.h — the per-grant prep of k_grant_prep (kernels.hip): proto3 Grant parse
// (MochiProtocol.java:7369-7425 semantics) and SHA-256 of the grant bytes (the
// signed message).  Outputs feed k_rsa_final (digest) and
// k_tally (timestamp, hash slice, PARSED flag).
#pragma once
#include "../../include/mochi_hip.h"
#include "proto_dev.h"
#include "sha256_dev.h"

namespace mochi {

struct PrepArgs {
  const uint8_t* blob;
  const uint64_t* goff;
  const uint32_t* glen;
  uint32_t n;           // grants to prep (0 = none)
  uint32_t* digest;     // [8][n]
  int64_t* ts;          // [n]
  uint64_t* hash_off;   // [n]
  uint32_t* hash_len;   // [n]
  uint8_t* flags;       // [n]
};

// What the prep of one grant's bytes yields; a pure function of the bytes, so
// it holds for every grant with the same bytes (hash_rel is relative to the
// grant's first byte).
struct PrepOut {
  uint32_t h[8];
  int64_t ts;
  uint32_t hash_rel, hash_len;
  uint8_t flags;
};

__device__ __forceinline__ void grant_prep_bytes(const uint8_t* p, uint32_t l, PrepOut& o) {
  ByteReader r;
  r.init(p, l);
  int64_t ts = 0;
  uint32_t hoff = 0, hlen = 0;
  const bool ok = parse_grant(r, ts, hoff, hlen);
  sha256(p, l, o.h);
  o.ts = ok ? ts : 0;
  o.hash_rel = hoff;
  o.hash_len = ok ? hlen : 0xFFFFFFFFu;
  o.flags = ok ? MOCHI_GRANT_PARSED : 0;
}

__device__ __forceinline__ void grant_prep_store(const PrepArgs& a, uint32_t i, const PrepOut& o) {
#pragma unroll
  for (int q = 0; q < 8; q++) a.digest[(size_t)q * a.n + i] = o.h[q];
  a.ts[i] = o.ts;
  a.hash_off[i] = a.goff[i] + o.hash_rel;
  a.hash_len[i] = o.hash_len;
  a.flags[i] = o.flags;
}

__device__ __forceinline__ void grant_prep_one(const PrepArgs& a, uint32_t i) {
  PrepOut o;
  grant_prep_bytes(a.blob + a.goff[i], a.glen[i], o);
  grant_prep_store(a, i, o);
}

// n bytes at a and at b equal?  Aligned dword loads funnel-shifted into place
// (v_alignbyte); every word read holds a byte of its string, so nothing past
// either grant's last byte is touched (the bytes may be a slice of a wire
// buffer).
__device__ inline bool bytes_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
  const uintptr_t pa = (uintptr_t)a, pb = (uintptr_t)b;
  const uint32_t* wa = (const uint32_t*)(pa & ~(uintptr_t)3);
  const uint32_t* wb = (const uint32_t*)(pb & ~(uintptr_t)3);
  const uint32_t sa = (uint32_t)(pa & 3), sb = (uint32_t)(pb & 3);
  uint32_t diff = 0, i = 0;
#pragma unroll 1
  for (; i + 16 <= n; i += 16) {
    const uint32_t k = i >> 2;
    uint32_t xa[5], xb[5];
#pragma unroll
    for (int j = 0; j < 4; j++) {
      xa[j] = wa[k + j];
      xb[j] = wb[k + j];
    }
    xa[4] = sa ? wa[k + 4] : 0u;  // holds byte i + 15 when sa > 0
    xb[4] = sb ? wb[k + 4] : 0u;
#pragma unroll
    for (int j = 0; j < 4; j++)
      diff |= __builtin_amdgcn_alignbyte(xa[j + 1], xa[j], sa) ^ __builtin_amdgcn_alignbyte(xb[j + 1], xb[j], sb);
    if (diff) return false;
  }
#pragma unroll 1
  for (; i < n; i++) {
    const uint32_t ia = i + sa, ib = i + sb;
    diff |= ((wa[ia >> 2] >> (8 * (ia & 3))) ^ (wb[ib >> 2] >> (8 * (ib & 3)))) & 0xFFu;
  }
  return diff == 0;
}

}  // namespace mochi
