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

// A grant nested deeper than the parse's register stack (kMaxGroupDepth) is
// marked kPrepDeep and finished by k_grant_deep: a call to the out-of-line
// deep parser here would cost k_grant_prep the call ABI's registers and
// scratch (168 VGPRs instead of ~140).
constexpr uint8_t kPrepDeep = 0x80;

// Grant i of the batch, its bytes read through `r` (HBM, or the copy
// k_grant_prep staged in LDS).
template <class R>
__device__ __forceinline__ void grant_prep_one(const PrepArgs& a, uint32_t i, R& r) {
  int64_t ts = 0;
  uint32_t hoff = 0, hlen = 0, ooff, olen;
  bool too_deep = false;
  const bool ok = parse_grant_t<kMaxGroupDepth>(r, ts, hoff, hlen, ooff, olen, too_deep);
  uint32_t h[8];
  sha256_at<typename R::mem>(r.abase + r.shift, r.len, h);
#pragma unroll
  for (int q = 0; q < 8; q++) a.digest[(size_t)q * a.n + i] = h[q];
  a.ts[i] = ok ? ts : 0;
  a.hash_off[i] = a.goff[i] + hoff;
  a.hash_len[i] = ok ? hlen : 0xFFFFFFFFu;
  a.flags[i] = ok ? MOCHI_GRANT_PARSED : too_deep ? kPrepDeep : 0;
}

}  // namespace mochi
