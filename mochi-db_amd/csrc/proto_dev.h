// proto_dev.h — device-side protobuf primitives shared by the grant-prep
// kernel (kernels.hip) and the Write2ToServer wire decoder (w2_decode.hip):
// a word-cached byte reader that never touches a word without an in-bounds
// byte, CodedInputStream-style varints, strict UTF-8 (Utf8.isValidUtf8), and
// the proto3 Grant parser (MochiProtocol.java:7369-7425 semantics).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mochi {

// ---------------------------------------------------------------------------
// Byte access into the grant blob (arbitrary alignment, never reads past the
// last byte of the grant: the blob may be a slice of a wire buffer).
// ---------------------------------------------------------------------------
struct ByteReader {
  const uint8_t* base;  // grant start
  uint32_t len;
  uint32_t cached_idx;  // aligned word index (relative to aligned base) held in `w`
  uint32_t w;
  uintptr_t abase;      // base rounded down to 4
  uint32_t shift;       // base & 3

  __device__ __forceinline__ void init(const uint8_t* p, uint32_t l) {
    base = p;
    len = l;
    abase = (uintptr_t)p & ~(uintptr_t)3;
    shift = (uint32_t)((uintptr_t)p & 3);
    cached_idx = 0xFFFFFFFFu;
    w = 0;
  }
  // byte i (i < len)
  __device__ __forceinline__ uint32_t at(uint32_t i) {
    const uint32_t a = i + shift;
    const uint32_t wi = a >> 2;
    if (wi != cached_idx) {
      w = *(const uint32_t*)(abase + 4 * (uintptr_t)wi);  // word holds byte i: in bounds
      cached_idx = wi;
    }
    return (w >> (8 * (a & 3))) & 0xFFu;
  }
};

// ---------------------------------------------------------------------------
// proto3 Grant parse — restates oracle_grant_parse (oracle/mochi_oracle.c),
// which restates MochiProtocol.java:7369-7425 + protobuf-java 3.16.3
// CodedInputStream.  Returns 1 ok / 0 malformed.
// ---------------------------------------------------------------------------
constexpr int kMaxGroupDepth = 16;    // register-resident group stack of the fast path
constexpr int kDeepGroupDepth = 100;  // CodedInputStream's default recursion limit (protobuf-java)

__device__ __forceinline__ bool rd_varint(ByteReader& r, uint32_t& pos, uint64_t& v) {
  uint64_t x = 0;
#pragma unroll 1
  for (int i = 0; i < 10; i++) {
    if (pos >= r.len) return false;
    const uint32_t c = r.at(pos++);
    x |= (uint64_t)(c & 0x7F) << (7 * i);
    if (!(c & 0x80)) {
      v = x;
      return true;
    }
  }
  return false;
}

__device__ inline bool valid_utf8(ByteReader& r, uint32_t off, uint32_t n) {
  uint32_t i = 0;
  // ASCII runs (keys, ids, the 128-char hex transactionHash) 32 bytes per step
  // at any alignment: the 9 aligned words that hold the 32 bytes are loaded
  // together (independent loads: one latency per step, not one per word) and
  // every byte of the window is tested for its high bit.  Each word holds at
  // least one byte of the window, which lies inside the string, so every load
  // stays in bounds (as ByteReader::at's).  A window with a non-ASCII byte
  // falls through to the byte-wise UTF-8 check below.
#pragma unroll 1
  while (i + 32 <= n) {
    const uintptr_t a = r.abase + (uintptr_t)(off + i + r.shift);
    const uint32_t* wp = (const uint32_t*)(a & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(a & 3);
    uint32_t w[9];
#pragma unroll
    for (int k = 0; k < 8; k++) w[k] = wp[k];
    w[8] = sh ? wp[8] : 0u;
    uint32_t hi = w[0] & (0x80808080u << (8 * sh));
#pragma unroll
    for (int k = 1; k < 8; k++) hi |= w[k];
    if (sh) hi |= w[8] & (0x80808080u >> (8 * (4 - sh)));
    if (hi & 0x80808080u) break;
    i += 32;
  }
#pragma unroll 1
  while (i < n) {
    // 16 ASCII bytes per step once the position is 16-byte aligned (all 16
    // bytes lie inside the string, so the load stays in bounds)
    const uintptr_t addr = r.abase + (uintptr_t)(off + i + r.shift);
    if ((addr & 15) == 0 && i + 16 <= n) {
      const uint4 v = *(const uint4*)addr;
      if (((v.x | v.y | v.z | v.w) & 0x80808080u) == 0) {
        i += 16;
        continue;
      }
    }
    const uint32_t c = r.at(off + i);
    if (c < 0x80) {
      // ASCII fast path: skip every remaining byte of the cached word when all
      // of them are ASCII and inside the string (keys and the 128-char hex
      // transactionHash are ASCII, so this is 4 bytes per step)
      const uint32_t sub = (off + i + r.shift) & 3, rest = 4 - sub;
      if (i + rest <= n && ((r.w >> (8 * sub)) & (0x80808080u >> (8 * sub))) == 0) i += rest;
      else i++;
      continue;
    }
    if (c < 0xC2) return false;
    if (c < 0xE0) {
      if (i + 1 >= n || (r.at(off + i + 1) & 0xC0) != 0x80) return false;
      i += 2;
      continue;
    }
    if (c < 0xF0) {
      if (i + 2 >= n) return false;
      const uint32_t c1 = r.at(off + i + 1), c2 = r.at(off + i + 2);
      if ((c1 & 0xC0) != 0x80 || (c2 & 0xC0) != 0x80) return false;
      if (c == 0xE0 && c1 < 0xA0) return false;
      if (c == 0xED && c1 >= 0xA0) return false;
      i += 3;
      continue;
    }
    if (c < 0xF5) {
      if (i + 3 >= n) return false;
      const uint32_t c1 = r.at(off + i + 1), c2 = r.at(off + i + 2), c3 = r.at(off + i + 3);
      if ((c1 & 0xC0) != 0x80 || (c2 & 0xC0) != 0x80 || (c3 & 0xC0) != 0x80) return false;
      if (c == 0xF0 && c1 < 0x90) return false;
      if (c == 0xF4 && c1 >= 0x90) return false;
      i += 4;
      continue;
    }
    return false;
  }
  return true;
}

__device__ __forceinline__ bool rd_string(ByteReader& r, uint32_t& pos, uint32_t& off, uint32_t& len) {
  uint64_t l;
  if (!rd_varint(r, pos, l)) return false;
  const int32_t l32 = (int32_t)(uint32_t)l;
  if (l32 < 0 || (uint32_t)l32 > r.len - pos) return false;
  if (!valid_utf8(r, pos, (uint32_t)l32)) return false;
  off = pos;
  len = (uint32_t)l32;
  pos += (uint32_t)l32;
  return true;
}

// kDepth = size of the unknown-group stack.  The fast instance keeps 16 entries
// in registers and reports a deeper nesting through `too_deep`; parse_grant
// then re-parses with the 100-deep instance, kept out of line (scratch stack).
// bytes of the minimal varint encoding of v
__device__ __forceinline__ uint32_t varint_size(uint64_t v) {
  const uint32_t bits = v ? 64u - (uint32_t)__builtin_clzll(v) : 1u;
  return (bits + 6) / 7;
}

// CANON (the wire decoder): also report in `canon` whether the bytes are
// exactly Grant.toByteArray() of the Grant they parse to
// (MochiProtocol.java:7556-7574): fields 1..5 in order, each at most once,
// none at its default, one-byte tags, minimal varints and lengths, no unknown
// fields, status an int32 (writeEnum sign-extends) -- decided during the parse
// instead of a second walk.
template <int kDepth, bool CANON = false>
__device__ inline bool parse_grant_t(ByteReader& r, int64_t& ts, uint32_t& hash_off, uint32_t& hash_len,
                                     uint32_t& oid_off, uint32_t& oid_len, bool& too_deep, bool* canon = nullptr) {
  uint32_t pos = 0;
  int64_t t = 0;
  uint32_t hoff = 0, hlen = 0, ooff = 0, olen = 0;
  uint32_t stack[kDepth];
  int depth = 0;
  uint32_t last_field = 0;
  bool cn = true;
#pragma unroll 1
  while (pos < r.len) {
    uint64_t tag64;
    const uint32_t p0 = pos;
    if (!rd_varint(r, pos, tag64)) return false;
    const uint32_t tag = (uint32_t)tag64, field = tag >> 3, wt = tag & 7;
    if (field == 0) return false;
    if (CANON) {
      cn = cn && pos - p0 == 1 && field > last_field && depth == 0;
      last_field = field;
    }
    if (depth > 0) {
      if (wt == 4) {
        if (stack[depth - 1] != field) return false;
        depth--;
        continue;
      }
    } else {
      if (tag == 10) {
        const uint32_t p1 = pos;
        if (!rd_string(r, pos, ooff, olen)) return false;
        if (CANON) cn = cn && olen != 0 && ooff - p1 == varint_size(olen);
        continue;
      }
      if (tag == 16 || tag == 24 || tag == 40) {
        uint64_t v;
        const uint32_t p1 = pos;
        if (!rd_varint(r, pos, v)) return false;
        if (tag == 16) t = (int64_t)v;
        // a 10-byte varint carries bit 63 alone in its last byte: rd_varint
        // drops bits past 64, so any other last byte (0x02..0x7F) decodes to
        // the same v but is not what toByteArray() writes
        if (CANON)
          cn = cn && v != 0 && pos - p1 == varint_size(v) && (pos - p1 < 10 || r.at(pos - 1) == 1) &&
               (tag != 40 || (int64_t)v == (int64_t)(int32_t)(uint32_t)v);
        continue;
      }
      if (tag == 34) {
        const uint32_t p1 = pos;
        if (!rd_string(r, pos, hoff, hlen)) return false;
        if (CANON) cn = cn && hlen != 0 && hoff - p1 == varint_size(hlen);
        continue;
      }
    }
    if (CANON) cn = false;  // an unknown field, a known one with a foreign wire type, or a group
    switch (wt) {
      case 0: {
        uint64_t v;
        if (!rd_varint(r, pos, v)) return false;
        break;
      }
      case 1:
        if (r.len - pos < 8) return false;
        pos += 8;
        break;
      case 2: {
        uint64_t l;
        if (!rd_varint(r, pos, l)) return false;
        const int32_t l32 = (int32_t)(uint32_t)l;
        if (l32 < 0 || (uint32_t)l32 > r.len - pos) return false;
        pos += (uint32_t)l32;
        break;
      }
      case 3:
        if (depth >= kDepth) {
          too_deep = kDepth < kDeepGroupDepth;
          return false;
        }
        stack[depth++] = field;
        break;
      case 5:
        if (r.len - pos < 4) return false;
        pos += 4;
        break;
      default:  // 4 (END_GROUP at top level), 6, 7
        return false;
    }
  }
  if (depth != 0) return false;
  ts = t;
  hash_off = hoff;
  hash_len = hlen;
  oid_off = ooff;
  oid_len = olen;
  if (CANON) *canon = cn;
  return true;
}

// The rare > 16-deep case, out of line.  Everything crosses the call by value
// (the bytes' address and length in, the fields back in a struct): a reader or
// output passed by reference would pin the caller's copies to the scratch
// stack for the whole kernel, so the fast path's every byte read would go
// through scratch memory.
struct GrantFields {
  int64_t ts;
  uint32_t hash_off, hash_len, oid_off, oid_len;
  uint32_t ok;
};

__device__ __noinline__ GrantFields parse_grant_deep(const uint8_t* p, uint32_t len) {
  ByteReader r;
  r.init(p, len);
  GrantFields f{0, 0, 0, 0, 0, 0};
  bool unused = false;
  f.ok = parse_grant_t<kDeepGroupDepth>(r, f.ts, f.hash_off, f.hash_len, f.oid_off, f.oid_len, unused) ? 1u : 0u;
  return f;
}

__device__ inline bool parse_grant(ByteReader& r, int64_t& ts, uint32_t& hash_off, uint32_t& hash_len, uint32_t& oid_off,
                                   uint32_t& oid_len) {
  bool too_deep = false;
  if (parse_grant_t<kMaxGroupDepth>(r, ts, hash_off, hash_len, oid_off, oid_len, too_deep)) return true;
  if (!too_deep) return false;
  const GrantFields f = parse_grant_deep(r.base, r.len);
  ts = f.ts;
  hash_off = f.hash_off;
  hash_len = f.hash_len;
  oid_off = f.oid_off;
  oid_len = f.oid_len;
  return f.ok != 0;
}

// parse validity (as parse_grant) + canonical encoding (parse_grant_t CANON).
// A grant that needs the deep parser has a group in it: parsed, never canonical.
__device__ inline bool parse_grant_canon(ByteReader& r, bool& canon) {
  int64_t ts;
  uint32_t ho, hl, oo, ol;
  bool too_deep = false;
  canon = false;
  if (parse_grant_t<kMaxGroupDepth, true>(r, ts, ho, hl, oo, ol, too_deep, &canon)) return true;
  canon = false;
  if (!too_deep) return false;
  return parse_grant_deep(r.base, r.len).ok != 0;
}

__device__ inline bool parse_grant(ByteReader& r, int64_t& ts, uint32_t& hash_off, uint32_t& hash_len) {
  uint32_t oo, ol;
  return parse_grant(r, ts, hash_off, hash_len, oo, ol);
}


}  // namespace mochi
