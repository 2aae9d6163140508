// prep_dev.h — the per-grant prep of k_grant_prep (kernels.hip): proto3 Grant parse
// (MochiProtocol.java:7369-7425 semantics) and SHA-256 of the grant bytes (the
// signed message).  Outputs feed k_rsa_final (digest) and
// k_tally (timestamp, hash slice, PARSED flag).
#pragma once
#include "../../include/mochi_hip.h"
#include "proto_dev.h"
#include "sha256_dev.h"

namespace mochi {

// Per grant: its timestamp and parse flags (outputs of the call) and, with
// grant dedup, `lead` = the index of its DISTINCT result -- the digest and the
// transactionHash slice, stored once per distinct grant (k_rsa_final and
// k_tally read them through lead).  Distinct index d: certificate c's first key
// slot -> c; any other grant prepped on its own -> d_base + g (d_base = the
// number of certificates; 0 and no lead array without dedup: d = g).
struct PrepArgs {
  const uint8_t* blob;
  const uint64_t* goff;
  const uint32_t* glen;
  uint32_t n;           // grants to prep (0 = none)
  uint32_t nd;          // stride of the distinct arrays (>= d_base + n)
  uint32_t d_base;
  uint32_t* digest;     // [8][nd]   distinct
  int64_t* ts;          // [n]       per grant
  uint64_t* hash_off;   // [nd]      distinct
  uint32_t* hash_len;   // [nd]      distinct
  uint8_t* flags;       // [n]       per grant
  uint32_t* lead;       // [n] per grant, or null (d = g)
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

// 16 bytes at p + pos (any alignment) as 4 little-endian words; bytes past l
// are garbage.  One or two 16-byte-aligned dwordx4 loads, each only if it holds
// a byte of the string, then a dword rotation by mask selects and a funnel.
__device__ __forceinline__ void window16(const uint8_t* p, uint32_t l, uint32_t pos, uint32_t (&w)[4]) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const uintptr_t addr = (uintptr_t)p + pos;
  const v4u* a16 = (const v4u*)(addr & ~(uintptr_t)15);
  const uint32_t sh = (uint32_t)(addr & 15);
  const v4u c0 = a16[0];  // holds byte pos (< l)
  v4u c1 = {0u, 0u, 0u, 0u};
  if (sh != 0 && pos - sh + 16 < l) c1 = a16[1];
  const uint32_t d[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  const uint32_t m4 = 0u - ((sh >> 2) & 1u), m8 = 0u - ((sh >> 3) & 1u);
  uint32_t e1[7], e[5];
#pragma unroll
  for (int j = 0; j < 7; j++) e1[j] = (d[j + 1] & m4) | (d[j] & ~m4);
#pragma unroll
  for (int j = 0; j < 5; j++) e[j] = (e1[j + 2] & m8) | (e1[j] & ~m8);
  const uint32_t r = 8 * (sh & 3);
#pragma unroll
  for (int t = 0; t < 4; t++) w[t] = __builtin_amdgcn_alignbit(e[t + 1], e[t], r);
}

// window16 without branches (a batch of them can be issued together): 16 bytes
// at addr; `two` = the second aligned chunk holds a wanted byte (else the first
// is loaded twice).  addr must be readable (callers pass a dummy when unused).
__device__ __forceinline__ void window16_nb(uintptr_t addr, bool two, uint32_t (&w)[4]) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const v4u* a16 = (const v4u*)(addr & ~(uintptr_t)15);
  const uint32_t sh = (uint32_t)(addr & 15);
  const v4u c0 = a16[0];
  const v4u c1 = a16[two ? 1 : 0];
  const uint32_t d[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
  const uint32_t m4 = 0u - ((sh >> 2) & 1u), m8 = 0u - ((sh >> 3) & 1u);
  uint32_t e1[7], e[5];
#pragma unroll
  for (int j = 0; j < 7; j++) e1[j] = (d[j + 1] & m4) | (d[j] & ~m4);
#pragma unroll
  for (int j = 0; j < 5; j++) e[j] = (e1[j + 2] & m8) | (e1[j] & ~m8);
  const uint32_t r = 8 * (sh & 3);
#pragma unroll
  for (int t = 0; t < 4; t++) w[t] = __builtin_amdgcn_alignbit(e[t + 1], e[t], r);
}

// The common Grant shape, as protobuf-java writes it (fields in number order,
// MochiProtocol.java:7556-7574): 0x0A L objectId 0x10 ts 0x22 H transactionHash,
// L < 128, ts a varint of at most 5 bytes, nothing after the hash.  Its header
// comes from two 16-byte windows (at 0 and at the timestamp's tag), and its two
// strings are UTF-8 (valid_utf8's verdict) exactly when they are ASCII: the
// SHA-256 message words count the bytes with their high bit set, and that
// count must be the header's own (varint continuation bytes) plus the
// padding's.  Same outputs as parse_grant for every grant it accepts; false
// (the generic parse decides) for any other shape or a non-ASCII string.
// No per-byte loads: the parse's word-by-word reads and the UTF-8 windows were
// most of the prep's memory requests (lane = certificate: every lane's grant
// sits in its own cache lines).
__device__ __forceinline__ bool grant_prep_fast(const uint8_t* p, uint32_t l, PrepOut& o) {
  if (l < 8) return false;
  uint32_t w0[4];
  window16(p, l, 0, w0);
  const uint32_t L = (w0[0] >> 8) & 0xFFu;
  if ((w0[0] & 0xFFu) != 0x0Au || L >= 0x80u) return false;
  const uint32_t q = 2 + L;  // the timestamp's tag
  if (q + 4 > l) return false;
  uint32_t hw[4];
  window16(p, l, q, hw);
  const uint64_t lo = ((uint64_t)hw[1] << 32) | hw[0], hi = ((uint64_t)hw[3] << 32) | hw[2];
  auto byte = [&](uint32_t k) -> uint32_t {  // k < 16, relative to q
    return (uint32_t)((k < 8 ? lo >> (8 * k) : hi >> (8 * (k - 8))) & 0xFFu);
  };
  if (byte(0) != 0x10u) return false;
  uint64_t ts = 0;
  uint32_t k = 1, hib_hdr = 0;
  bool end = false;
#pragma unroll
  for (int i = 0; i < 5; i++) {
    if (!end) {
      const uint32_t c = byte(k++);
      ts |= (uint64_t)(c & 0x7Fu) << (7 * i);
      end = c < 0x80u;
      hib_hdr += c >> 7;
    }
  }
  if (!end || byte(k) != 0x22u) return false;
  const uint32_t c1 = byte(k + 1), c2 = byte(k + 2);
  uint32_t hl, hp;
  if (c1 < 0x80u) {
    hl = c1;
    hp = q + k + 2;
  } else if (c2 < 0x80u) {
    hl = (c1 & 0x7Fu) | (c2 << 7);
    hp = q + k + 3;
    hib_hdr += 1;
  } else {
    return false;
  }
  if (hp > l || hl != l - hp) return false;  // the hash ends the grant
  uint32_t hib = 0;
  sha256(p, l, o.h, &hib);
  const uint32_t bits = 8 * l;  // the padding: 0x80, then the 64-bit bit length (its low two bytes here)
  if (hib != hib_hdr + 1 + ((bits >> 15) & 1u) + ((bits >> 7) & 1u) + ((bits >> 23) & 1u)) return false;
  o.ts = (int64_t)ts;
  o.hash_rel = hp;
  o.hash_len = hl;
  o.flags = MOCHI_GRANT_PARSED;
  return true;
}

__device__ __forceinline__ void grant_prep_bytes(const uint8_t* p, uint32_t l, PrepOut& o) {
  if (grant_prep_fast(p, l, o)) return;
  ByteReader r;
  r.init(p, l);
  int64_t ts = 0;
  uint32_t hoff = 0, hlen = 0;
  const bool ok = parse_grant(r, ts, hoff, hlen);
  sha256(p, l, o.h);
  o.ts = ok ? ts : 0;
  o.hash_rel = hoff;
  o.hash_len = ok ? hlen : 0u;  // unparsed: k_tally rejects the certificate before its hash check
  o.flags = ok ? MOCHI_GRANT_PARSED : 0;
}

// hash_len[d] with kHashChecked set: k_grant_prep_cert already compared the
// transactionHash with its certificate's expected hash (kHashEq = equal), so
// k_tally reads this word instead of both hashes.  A plain length is kept below
// kHashEq (a length that large is never MOCHI_TXN_HASH_BYTES: same verdict).
constexpr uint32_t kHashChecked = 0x80000000u, kHashEq = 0x40000000u;

__device__ __forceinline__ uint32_t hash_len_word(const PrepOut& o) {
  return o.hash_len < kHashEq ? o.hash_len : kHashEq - 1u;
}

// The distinct result d of grant bytes at offset `goff` (hash_off is absolute).
__device__ __forceinline__ void grant_prep_store_dist(const PrepArgs& a, uint32_t d, uint64_t goff, const PrepOut& o,
                                                      uint32_t hash_word) {
#pragma unroll
  for (int q = 0; q < 8; q++) a.digest[(size_t)q * a.nd + d] = o.h[q];
  a.hash_off[d] = goff + o.hash_rel;
  a.hash_len[d] = hash_word;
}

__device__ __forceinline__ void grant_prep_store_dist(const PrepArgs& a, uint32_t d, uint64_t goff, const PrepOut& o) {
  grant_prep_store_dist(a, d, goff, o, hash_len_word(o));
}

// Grant g's own outputs, its result at distinct index d.
__device__ __forceinline__ void grant_prep_store_grant(const PrepArgs& a, uint32_t g, uint32_t d, int64_t ts,
                                                       uint8_t flags) {
  a.ts[g] = ts;
  a.flags[g] = flags;
  if (a.lead) a.lead[g] = d;
}

__device__ __forceinline__ void grant_prep_one(const PrepArgs& a, uint32_t i) {
  PrepOut o;
  const uint64_t goff = a.goff[i];
  grant_prep_bytes(a.blob + goff, a.glen[i], o);
  const uint32_t d = a.d_base + i;
  grant_prep_store_dist(a, d, goff, o);
  grant_prep_store_grant(a, i, d, o.ts, o.flags);
}

// Bytes [pos, pos + 64) of the `len` bytes at `base` (any alignment) as 16
// little-endian words (words past len hold garbage: callers mask them).  Like
// sha256_block_words: 16-byte-aligned dwordx4 loads, each issued only if its 16
// bytes hold a byte of the string, a per-lane dword rotation by mask selects
// and a funnel shift -- 4 or 5 loads per 64 bytes instead of 16 + 16 dword loads
// (every load of a lane gathered from its own cache line).
__device__ __forceinline__ void window64(const uint8_t* base, uint32_t len, uint32_t pos, uint32_t (&w)[16]) {
  typedef uint32_t v4u __attribute__((ext_vector_type(4)));
  const uintptr_t addr = (uintptr_t)base + pos;
  const v4u* a16 = (const v4u*)(addr & ~(uintptr_t)15);
  const uint32_t sh = (uint32_t)(addr & 15);
  const int64_t p0 = (int64_t)pos - sh;  // string position of the first loaded byte
  uint32_t d[20];
#pragma unroll
  for (int c = 0; c < 5; c++) {
    v4u v = {0u, 0u, 0u, 0u};
    if (p0 + 16 * c < (int64_t)len && (c < 4 || sh != 0)) v = a16[c];
    d[4 * c] = v.x;
    d[4 * c + 1] = v.y;
    d[4 * c + 2] = v.z;
    d[4 * c + 3] = v.w;
  }
  const uint32_t m4 = 0u - ((sh >> 2) & 1u), m8 = 0u - ((sh >> 3) & 1u);
  uint32_t e1[19], e[17];
#pragma unroll
  for (int j = 0; j < 19; j++) e1[j] = (d[j + 1] & m4) | (d[j] & ~m4);
#pragma unroll
  for (int j = 0; j < 17; j++) e[j] = (e1[j + 2] & m8) | (e1[j] & ~m8);
  const uint32_t r = 8 * (sh & 3);
#pragma unroll
  for (int t = 0; t < 16; t++) w[t] = __builtin_amdgcn_alignbit(e[t + 1], e[t], r);
}

// n bytes at a and at b equal?  64 bytes per step (window64); nothing past
// either string's last byte is read (the bytes may be a slice of a wire buffer).
__device__ inline bool bytes_equal(const uint8_t* a, const uint8_t* b, uint32_t n) {
#pragma unroll 1
  for (uint32_t pos = 0; pos < n; pos += 64) {
    uint32_t wa[16], wb[16];
    window64(a, n, pos, wa);
    window64(b, n, pos, wb);
    uint32_t diff = 0;
#pragma unroll
    for (int t = 0; t < 16; t++) {
      const int32_t left = (int32_t)(n - pos) - 4 * t;  // bytes of word t inside the strings
      const uint32_t m = left >= 4 ? ~0u : left <= 0 ? 0u : (1u << (8 * left)) - 1u;
      diff |= (wa[t] ^ wb[t]) & m;
    }
    if (diff) return false;
  }
  return true;
}

// 128 bytes at a and at b (any alignment) equal: all four 64-byte windows
// issued before the compare -- one memory round trip, not bytes_equal's one per
// window (callers that have the registers: k_grant_prep_cert after its SHA-256)
__device__ __forceinline__ bool bytes128_equal(const uint8_t* a, const uint8_t* b) {
  uint32_t a0[16], a1[16], b0[16], b1[16];
  window64(a, 128, 0, a0);
  window64(a, 128, 64, a1);
  window64(b, 128, 0, b0);
  window64(b, 128, 64, b1);
  uint32_t diff = 0;
#pragma unroll
  for (int t = 0; t < 16; t++) diff |= (a0[t] ^ b0[t]) | (a1[t] ^ b1[t]);
  return diff == 0;
}

}  // namespace mochi
