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

__device__ __forceinline__ void grant_prep_one(const PrepArgs& a, uint32_t i) {
  const uint8_t* p = a.blob + a.goff[i];
  const uint32_t l = a.glen[i];
  ByteReader r;
  r.init(p, l);
  int64_t ts = 0;
  uint32_t hoff = 0, hlen = 0;
  const bool ok = parse_grant(r, ts, hoff, hlen);
  uint32_t h[8];
  sha256(p, l, h);
#pragma unroll
  for (int q = 0; q < 8; q++) a.digest[(size_t)q * a.n + i] = h[q];
  a.ts[i] = ok ? ts : 0;
  a.hash_off[i] = a.goff[i] + hoff;
  a.hash_len[i] = ok ? hlen : 0xFFFFFFFFu;
  a.flags[i] = ok ? MOCHI_GRANT_PARSED : 0;
}

}  // namespace mochi
