// w2_decode.hip — Write2ToServer wire messages -> the SoA certificate batch,
// on the device (one lane per message).
//
//   k_w2_msg      level 1, lane = message: top level, operations, the
//                 WriteCertificate's entry framing and keys; messages outside
//                 the level-by-level shape are validated whole here
//   (scan)        certificate-entry offsets
//   k_w2_entries  the certificate entries into a compact list
//   k_w2_mg       level 2, lane = certificate entry: validate the MultiGrant,
//                 resolve map order, count + canonical-check decoded grants
//   k_w2_final    per message: status and decoded counts; (scans) CSR offsets
//   k_w2_emit_mg  lane = certificate entry: grant offsets (zero copy into the
//                 wire blob), signers, key slots, MultiGrant CSR
//   k_w2_ops      lane = message: operations
//   k_w2_sig      signatures gathered 16 lanes per grant (coalesced)
//   k_w2_fixup    after the verify path: MALFORMED / FALLBACK / OPS_MISMATCH
//                 messages get their reason code and no accept bit
//
// Semantics (restated from protobuf-java 3.16.3, pinned by
// tests/golden/write2_vectors.json and oracle/mochi_oracle.c):
//   * message schema MochiProtocol.proto:107-147 + MultiGrant.grantSignatures
//     = 5 (map<string, bytes>);
//   * singular scalar / string fields: last value wins; unknown fields and
//     known fields with a foreign wire type are skipped;
//   * map fields (WriteCertificate.grants, MultiGrant.grants,
//     MultiGrant.grantSignatures): entries go into a LinkedHashMap, a repeated
//     key keeps its FIRST position and takes the LAST value (MapField +
//     MapEntryLite.parseEntry);
//   * proto3 strings and string map keys must be valid UTF-8; every Grant
//     value must parse, including values a later entry replaces.
// Map de-duplication is done by re-scanning (no per-lane tables): messages
// hold a handful of MultiGrants and grants, so O(n^2) short compares are
// cheaper than spilling per-lane maps.
#include <hipcub/hipcub.hpp>

#include "../../include/mochi_hip.h"
#include "prep_dev.h"
#include "proto_dev.h"
#include "w2.h"

namespace mochi {
namespace {

constexpr uint32_t kMaxMG = kW2MaxCertEntries;  // certificate entries per message (fast path)
constexpr uint32_t kMaxGrantsPerMG = 64;  // grants entries per decoded MultiGrant (fast path)
constexpr uint32_t kMaxOps = MOCHI_MAX_OPS_PER_CERT;

struct Fld {
  uint32_t field, wt;
  uint64_t v;
  uint32_t off, len;  // wt 2 payload (message-relative)
};

__device__ __forceinline__ bool vint(ByteReader& r, uint32_t& pos, uint32_t end, uint64_t& v) {
  uint64_t x = 0;
#pragma unroll 1
  for (int i = 0; i < 10; i++) {
    if (pos >= end) return false;
    const uint32_t c = r.at(pos++);
    x |= (uint64_t)(c & 0x7F) << (7 * i);
    if (!(c & 0x80)) {
      v = x;
      return true;
    }
  }
  return false;
}

__device__ __forceinline__ bool vlen(ByteReader& r, uint32_t& pos, uint32_t end, uint32_t& len) {
  uint64_t l;
  if (!vint(r, pos, end, l)) return false;
  const int32_t l32 = (int32_t)(uint32_t)l;  // readRawVarint32
  if (l32 < 0 || (uint32_t)l32 > end - pos) return false;
  len = (uint32_t)l32;
  return true;
}

// Skip an unknown group opened by `field` (skipMessage + checkLastTagWas).
// Rare: kept out of line so its stack does not weigh on the common path, and
// called with plain values -- a reader or position passed by reference would
// pin the callers' copies to the scratch stack, and every byte the common path
// reads would then go through scratch.  Returns the position after the group,
// or kSkipBad.
constexpr uint32_t kSkipBad = 0xFFFFFFFFu;

__device__ __noinline__ uint32_t skip_group(const uint8_t* base, uint32_t len, uint32_t pos, uint32_t end,
                                            uint32_t field) {
  ByteReader r;
  r.init(base, len);
  uint32_t stack[kDeepGroupDepth];
  int depth = 1;
  stack[0] = field;
#pragma unroll 1
  while (depth > 0) {
    uint64_t t64;
    if (!vint(r, pos, end, t64)) return kSkipBad;
    const uint32_t t = (uint32_t)t64, f = t >> 3, wt = t & 7;
    if (f == 0) return kSkipBad;
    uint32_t l;
    switch (wt) {
      case 0: {
        uint64_t v;
        if (!vint(r, pos, end, v)) return kSkipBad;
        break;
      }
      case 1:
        if (end - pos < 8) return kSkipBad;
        pos += 8;
        break;
      case 2:
        if (!vlen(r, pos, end, l)) return kSkipBad;
        pos += l;
        break;
      case 3:
        if (depth >= kDeepGroupDepth) return kSkipBad;
        stack[depth++] = f;
        break;
      case 4:
        if (stack[depth - 1] != f) return kSkipBad;
        depth--;
        break;
      case 5:
        if (end - pos < 4) return kSkipBad;
        pos += 4;
        break;
      default:
        return kSkipBad;
    }
  }
  return pos;
}

// Next field in [pos, end): 1 field, 0 end, -1 malformed.
__device__ int next_fld(ByteReader& r, uint32_t& pos, uint32_t end, Fld& f) {
  if (pos >= end) return 0;
  uint64_t t64;
  if (!vint(r, pos, end, t64)) return -1;
  const uint32_t t = (uint32_t)t64;
  f.field = t >> 3;
  f.wt = t & 7;
  f.off = f.len = 0;
  f.v = 0;
  if (f.field == 0) return -1;
  switch (f.wt) {
    case 0:
      return vint(r, pos, end, f.v) ? 1 : -1;
    case 1:
      if (end - pos < 8) return -1;
      pos += 8;
      return 1;
    case 2:
      if (!vlen(r, pos, end, f.len)) return -1;
      f.off = pos;
      pos += f.len;
      return 1;
    case 3: {
      const uint32_t np = skip_group(r.base, r.len, pos, end, f.field);
      if (np == kSkipBad) return -1;
      pos = np;
      return 1;
    }
    case 5:
      if (end - pos < 4) return -1;
      pos += 4;
      return 1;
    default:
      return -1;  // END_GROUP at message level, wire types 6 and 7
  }
}

// ---- validity: what protobuf-java's parser checks ---------------------------
__device__ bool valid_grant_at(ByteReader& r, uint32_t off, uint32_t len, bool& canon) {
  ByteReader g;
  g.init(r.base + off, len);
  return parse_grant_canon(g, canon);
}

struct Entry {
  uint32_t koff, klen;  // key (last occurrence; default "")
  uint32_t voff, vlen;  // value (last occurrence; default empty)
  uint32_t nval;
  bool canon;           // Grant value (kind 1): the last value is canonical Grant bytes
  bool assumed;         // ... taken as canonical without a parse: its bytes equal the reference grant's
};

// A Grant slice of the message whose validity and canonical form another lane
// decides (k_w2_mg: the first grant of the message's first MultiGrant); ~0 = none.
struct RefGrant {
  uint32_t off = ~0u, len = 0;
};

// map<string, V> entry; kind 0 = bytes value, 1 = Grant value: validated, and
// its key and value read as read_entry reads them (last occurrence of each)
__device__ bool valid_leaf_read(ByteReader& r, uint32_t off, uint32_t len, int kind, Entry& e,
                                const RefGrant ref = RefGrant{}) {
  e.koff = e.klen = e.voff = e.vlen = e.nval = 0;
  e.canon = e.assumed = false;
  uint32_t pos = off, end = off + len;
  Fld f;
  int rc;
#pragma unroll 1
  while ((rc = next_fld(r, pos, end, f)) > 0) {
    if (f.wt != 2) continue;
    if (f.field == 1) {
      if (!valid_utf8(r, f.off, f.len)) return false;
      e.koff = f.off;
      e.klen = f.len;
    } else if (f.field == 2) {
      if (kind == 1) {
        // the same bytes as the reference grant: its lane parses them (an
        // invalid grant makes the whole message MALFORMED there) and reports
        // a non-canonical one (kStFirstNC), so only the byte compare runs here
        e.assumed = ref.off != ~0u && f.len == ref.len && bytes_equal(r.base + f.off, r.base + ref.off, f.len);
        if (e.assumed) e.canon = true;
        else if (!valid_grant_at(r, f.off, f.len, e.canon)) return false;
      }
      e.voff = f.off;
      e.vlen = f.len;
      e.nval++;
    }
  }
  // an entry without a value holds the default Grant, whose toByteArray() is
  // empty: canonical, as a zero-length value is
  if (kind == 1 && e.nval == 0) e.canon = true;
  return rc == 0;
}

__device__ __forceinline__ bool valid_leaf_entry(ByteReader& r, uint32_t off, uint32_t len, int kind) {
  Entry e;
  return valid_leaf_read(r, off, len, kind, e);
}

__device__ bool valid_multigrant(ByteReader& r, uint32_t off, uint32_t len) {
  uint32_t pos = off, end = off + len;
  Fld f;
  int rc;
#pragma unroll 1
  while ((rc = next_fld(r, pos, end, f)) > 0) {
    if (f.wt != 2) continue;
    if (f.field == 1 && !valid_leaf_entry(r, f.off, f.len, 1)) return false;
    if (f.field >= 2 && f.field <= 4 && !valid_utf8(r, f.off, f.len)) return false;
    if (f.field == 5 && !valid_leaf_entry(r, f.off, f.len, 0)) return false;
  }
  return rc == 0;
}

__device__ bool valid_cert_entry(ByteReader& r, uint32_t off, uint32_t len) {
  uint32_t pos = off, end = off + len;
  Fld f;
  int rc;
#pragma unroll 1
  while ((rc = next_fld(r, pos, end, f)) > 0) {
    if (f.wt != 2) continue;
    if (f.field == 1 && !valid_utf8(r, f.off, f.len)) return false;
    if (f.field == 2 && !valid_multigrant(r, f.off, f.len)) return false;
  }
  return rc == 0;
}

// every field of `off,len` numbered `field` with wt 2 must satisfy `ok`
template <typename F>
__device__ bool all_ld(ByteReader& r, uint32_t off, uint32_t len, uint32_t field, F&& ok) {
  uint32_t pos = off, end = off + len;
  Fld f;
  int rc;
#pragma unroll 1
  while ((rc = next_fld(r, pos, end, f)) > 0)
    if (f.field == field && f.wt == 2 && !ok(f)) return false;
  return rc == 0;
}

// (ko, kl): the operation's operand1 as last_string(.., 2, ..) reads it
__device__ bool valid_operation(ByteReader& r, uint32_t off, uint32_t len, uint32_t& ko, uint32_t& kl) {
  uint32_t pos = off, end = off + len;
  Fld f;
  int rc;
  ko = kl = 0;
#pragma unroll 1
  while ((rc = next_fld(r, pos, end, f)) > 0)
    if (f.wt == 2 && f.field >= 2 && f.field <= 4) {
      if (!valid_utf8(r, f.off, f.len)) return false;
      if (f.field == 2) {
        ko = f.off;
        kl = f.len;
      }
    }
  return rc == 0;
}

__device__ __forceinline__ bool valid_operation(ByteReader& r, uint32_t off, uint32_t len) {
  uint32_t ko, kl;
  return valid_operation(r, off, len, ko, kl);
}

__device__ bool valid_write2(ByteReader& r) {
  uint32_t pos = 0, end = r.len;
  Fld f;
  int rc;
#pragma unroll 1
  while ((rc = next_fld(r, pos, end, f)) > 0) {
    if (f.wt != 2) continue;
    if (f.field == 1 &&
        !all_ld(r, f.off, f.len, 1, [&](const Fld& e) { return valid_cert_entry(r, e.off, e.len); }))
      return false;
    if (f.field == 2 &&
        !all_ld(r, f.off, f.len, 1, [&](const Fld& o) { return valid_operation(r, o.off, o.len); }))
      return false;
  }
  return rc == 0;
}

// ---- extraction on a valid message -------------------------------------------

__device__ void read_entry(ByteReader& r, uint32_t off, uint32_t len, Entry& e) {
  e.koff = e.klen = e.voff = e.vlen = e.nval = 0;
  uint32_t pos = off, end = off + len;
  Fld f;
#pragma unroll 1
  while (next_fld(r, pos, end, f) > 0) {
    if (f.wt != 2) continue;
    if (f.field == 1) {
      e.koff = f.off;
      e.klen = f.len;
    } else if (f.field == 2) {
      e.voff = f.off;
      e.vlen = f.len;
      e.nval++;
    }
  }
}

// 4 bytes at message offset o (any alignment; o + 4 <= message length)
__device__ __forceinline__ uint32_t ld4(const uint8_t* base, uint32_t o) {
  const uintptr_t a = (uintptr_t)(base + o);
  const uint32_t* wp = (const uint32_t*)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t w0 = wp[0];
  const uint32_t w1 = sh ? wp[1] : 0u;  // holds byte o+3 when sh != 0
  return (uint32_t)((((uint64_t)w1 << 32) | w0) >> (8 * sh));
}

// bytes [a, a+n) of message A equal bytes [b, b+n) of message B
__device__ bool bytes_eq(const uint8_t* A, uint32_t a, const uint8_t* B, uint32_t b, uint32_t n) {
  uint32_t i = 0;
#pragma unroll 1
  for (; i + 4 <= n; i += 4)
    if (ld4(A, a + i) != ld4(B, b + i)) return false;
#pragma unroll 1
  for (; i < n; i++)
    if (A[a + i] != B[b + i]) return false;
  return true;
}

// Keys of one map mostly share a prefix ("server-" + UUID, "key-" + number):
// compare the last four bytes first, so a mismatch costs one word per side.
__device__ __forceinline__ bool key_eq(ByteReader& r, uint32_t a, uint32_t al, uint32_t b, uint32_t bl) {
  if (al != bl) return false;
  if (a == b) return true;
  if (al >= 4 && ld4(r.base, a + al - 4) != ld4(r.base, b + al - 4)) return false;
  return bytes_eq(r.base, a, r.base, b, al);
}

// Walk the map entries (field `field`, wt 2) of [off, off+len) in wire order.
// For entry i that is the FIRST occurrence of its key, fn(first, last) is
// called with the entry itself and the entry holding the key's final value.
// Returns false if any entry carries its value more than once (fast-path exit).
template <typename F>
__device__ bool for_map(ByteReader& r, uint32_t off, uint32_t len, uint32_t field, F&& fn) {
  uint32_t pos = off, end = off + len;
  Fld f;
#pragma unroll 1
  while (next_fld(r, pos, end, f) > 0) {
    if (f.field != field || f.wt != 2) continue;
    Entry e;
    read_entry(r, f.off, f.len, e);
    if (e.nval > 1) return false;
    // an earlier entry with the same key?
    bool first = true;
    {
      uint32_t p2 = off;
      Fld g;
#pragma unroll 1
      while (p2 < f.off && next_fld(r, p2, end, g) > 0) {
        if (g.field != field || g.wt != 2 || g.off >= f.off) continue;
        Entry x;
        read_entry(r, g.off, g.len, x);
        if (key_eq(r, x.koff, x.klen, e.koff, e.klen)) {
          first = false;
          break;
        }
      }
    }
    if (!first) continue;
    Entry last = e;
    {
      uint32_t p2 = pos;  // entries after this one
      Fld g;
#pragma unroll 1
      while (next_fld(r, p2, end, g) > 0) {
        if (g.field != field || g.wt != 2) continue;
        Entry x;
        read_entry(r, g.off, g.len, x);
        if (key_eq(r, x.koff, x.klen, e.koff, e.klen)) last = x;
      }
    }
    if (!fn(e, last)) return false;
  }
  return true;
}

__device__ void last_string(ByteReader& r, uint32_t off, uint32_t len, uint32_t field, uint32_t& so, uint32_t& sl) {
  so = sl = 0;
  uint32_t pos = off, end = off + len;
  Fld f;
#pragma unroll 1
  while (next_fld(r, pos, end, f) > 0)
    if (f.field == field && f.wt == 2) {
      so = f.off;
      sl = f.len;
    }
}

// Last value of varint field `field` (wire type 0) of [off, off+len); 0 if absent.
__device__ uint64_t last_varint(ByteReader& r, uint32_t off, uint32_t len, uint32_t field) {
  uint64_t v = 0;
  uint32_t pos = off, end = off + len;
  Fld f;
#pragma unroll 1
  while (next_fld(r, pos, end, f) > 0)
    if (f.field == field && f.wt == 0) v = f.v;
  return v;
}

// Varint at [pos, end) is the minimal encoding of its value.
__device__ bool canon_varint(ByteReader& r, uint32_t& pos, uint32_t end, uint64_t& v) {
  const uint32_t p0 = pos;
  if (!vint(r, pos, end, v)) return false;
  const uint32_t n = pos - p0;
  if (n > 1 && r.at(pos - 1) == 0) return false;   // trailing zero group
  if (n == 10 && r.at(pos - 1) > 1) return false;  // bits beyond 64
  return true;
}

// The Grant bytes at [off, off+len) are exactly Grant.toByteArray() of the
// Grant they parse to (MochiProtocol.java:7556-7574): fields 1..5 in order,
// each at most once, none at its default, minimal varints, no unknown fields.
// (Parse validity was checked by valid_write2.)
__device__ bool grant_canonical(ByteReader& r, uint32_t off, uint32_t len) {
  uint32_t pos = off, end = off + len, last = 0;
#pragma unroll 1
  while (pos < end) {
    const uint32_t tag = r.at(pos++);  // fields 1..5 have one-byte tags
    const uint32_t field = tag >> 3, wt = tag & 7;
    if (field <= last || field > 5) return false;
    last = field;
    uint64_t v;
    if (field == 1 || field == 4) {
      if (wt != 2) return false;
      if (!canon_varint(r, pos, end, v) || v == 0 || v > end - pos) return false;
      pos += (uint32_t)v;
    } else {
      if (wt != 0) return false;
      if (!canon_varint(r, pos, end, v) || v == 0) return false;
      // enum status: writeEnum writes the int32 sign-extended
      if (field == 5 && (int64_t)v != (int64_t)(int32_t)(uint32_t)v) return false;
    }
  }
  return true;
}

// Decoder outputs (the SoA batch).  Mirrors oracle/mochi_oracle.c decode_one.
struct W2Out {
  uint64_t* sig_src;  // wire offset of each grant's 256-byte signature, ~0 = none
  uint64_t* grant_off;
  uint32_t* grant_len;
  uint8_t* sig;
  uint16_t* signer;
  uint8_t* grant_key;
  uint8_t* op_key;
  uint8_t* op_flags;
  int64_t* op_object_ts;
  uint64_t* op_key_off;
  uint32_t* op_key_len;
  uint32_t* mg_grant_off;
  uint32_t* grant_same;  // or null
};

// Per-message decode state (W2Args::cnt_ce onwards; cnt_o is W2Args::cnt_o).
struct W2Msg {
  uint32_t *cnt_ce, *ce_base, *st_bits, *wc_off, *wc_len, *tx_off, *tx_len, *cnt_o;
  uint32_t* inl;  // [M][kW2InlEntries][4]: koff, klen, voff, vlen of the first entries
  uint32_t* inl_ops;  // [M][kW2InlOps][2]: operand1 off, len of the first operations
};

// ---- level by level ------------------------------------------------------------
// A Write2ToServer message is decoded in two levels, so no lane walks a whole
// ~2.9 KB message with dependent loads:
//   level 1, lane = message: the top level, every Operation, and the
//     WriteCertificate's entries (framing, key UTF-8, value count) -- not the
//     MultiGrant values;
//   level 2, lane = certificate entry (one MultiGrant): validates the MultiGrant
//     value (its grants, Grant values, signatures, strings), resolves the
//     LinkedHashMap order against its sibling entries and, for the entry that
//     holds a key's final value, counts the distinct grants and checks them
//     canonical; the emit kernel later writes that MultiGrant's grants.
// Messages outside this shape (writeCertificate / transaction repeated, > 32
// certificate entries, an entry carrying two values, > 64 operations) are
// validated whole by their level-1 lane (valid_write2) and leave the fast path
// (MOCHI_MSG_FALLBACK, or MALFORMED).  Status bits per message: level-2 lanes
// OR theirs in; MALFORMED dominates FALLBACK.
constexpr uint32_t kStMal = 1u, kStFb = 2u;
constexpr uint32_t kMaxSigEntries = 64;  // grantSignatures entries per decoded MultiGrant (fast path)

__device__ __noinline__ bool valid_write2_whole(const uint8_t* base, uint32_t len) {
  ByteReader r;
  r.init(base, len);
  return valid_write2(r);
}

// Level 1 for one message; returns status bits.  nce = certificate entries,
// nops = operations (both 0 when the message left the fast path).
__device__ uint32_t msg_level(ByteReader& r, uint32_t& nce, uint32_t& nops, uint32_t& wc_off, uint32_t& wc_len,
                              uint32_t& tx_off, uint32_t& tx_len, uint32_t* __restrict__ inl,
                              uint32_t* __restrict__ inl_ops) {
  uint32_t n_wc = 0, n_tx = 0;
  bool whole = false;
  nce = nops = 0;
  uint32_t pos = 0;
  Fld f;
  int rc;
#pragma unroll 1
  while (!whole && (rc = next_fld(r, pos, r.len, f)) > 0) {
    if (f.wt != 2) continue;
    if (f.field == 1) {
      if (++n_wc > 1) {
        whole = true;
        break;
      }
      wc_off = f.off;
      wc_len = f.len;
      uint32_t p2 = f.off, e2 = f.off + f.len;
      Fld g;
      int rc2;
#pragma unroll 1
      while ((rc2 = next_fld(r, p2, e2, g)) > 0) {
        if (g.field != 1 || g.wt != 2) continue;
        if (++nce > kMaxMG) {
          whole = true;
          break;
        }
        uint32_t p3 = g.off, e3 = g.off + g.len, nval = 0;
        uint32_t ko = 0, kl = 0, vo = 0, vl = 0;  // read_entry's slices (last key, last value)
        Fld h;
        int rc3;
#pragma unroll 1
        while ((rc3 = next_fld(r, p3, e3, h)) > 0) {
          if (h.wt != 2) continue;
          if (h.field == 1) {
            if (!valid_utf8(r, h.off, h.len)) return kStMal;
            ko = h.off;
            kl = h.len;
          }
          if (h.field == 2) {
            nval++;
            vo = h.off;
            vl = h.len;
          }
        }
        if (rc3 < 0) return kStMal;
        if (nce <= kW2InlEntries) ((uint4*)inl)[nce - 1] = make_uint4(ko, kl, vo, vl);
        if (nval > 1) {
          whole = true;
          break;
        }
      }
      if (!whole && rc2 < 0) return kStMal;
    } else if (f.field == 2) {
      if (++n_tx > 1) {
        whole = true;
        break;
      }
      tx_off = f.off;
      tx_len = f.len;
      uint32_t p2 = f.off, e2 = f.off + f.len;
      Fld g;
      int rc2;
#pragma unroll 1
      while ((rc2 = next_fld(r, p2, e2, g)) > 0) {
        if (g.field != 1 || g.wt != 2) continue;
        if (++nops > kMaxOps) {
          whole = true;
          break;
        }
        uint32_t ko, kl;
        if (!valid_operation(r, g.off, g.len, ko, kl)) return kStMal;
        if (nops <= kW2InlOps) ((uint2*)inl_ops)[nops - 1] = make_uint2(ko, kl);
      }
      if (!whole && rc2 < 0) return kStMal;
    }
  }
  if (whole) {
    nce = nops = 0;
    return valid_write2_whole(r.base, r.len) ? kStFb : kStMal;
  }
  return rc < 0 ? kStMal : 0u;
}

__device__ __forceinline__ uint32_t wbyte(const uint32_t* w, uint32_t k) {  // k compile-time after unrolling
  return (w[k >> 2] >> (8 * (k & 3))) & 0xFFu;
}

// bytes [a, b) of a window, as a mask of word t
__device__ __forceinline__ uint32_t span_mask(int t, int a, int b) {
  const int lo = a - 4 * t, hi = b - 4 * t;
  const uint32_t m_hi = hi >= 4 ? ~0u : hi <= 0 ? 0u : (1u << (8 * hi)) - 1u;
  const uint32_t m_lo = lo <= 0 ? 0u : lo >= 4 ? ~0u : (1u << (8 * lo)) - 1u;
  return m_hi & ~m_lo;
}

// The first grant of a MultiGrant value, as first_grant finds it, from its
// first 16 bytes `h` (at `off`) and one word: lengths of one or two varint
// bytes, a key < 128 bytes (otherwise none -- the match is a hint, and only
// equal bytes use it).  ref_head parses the window: the grant's slice and the
// word expected at `gpos` (its tag and length); ref_grant_win loads both.
struct RefHead {
  uint32_t off, len, gpos, word, mask;
  bool ok;
};
__device__ __forceinline__ RefHead ref_head(const uint32_t (&h)[4], uint32_t off, uint32_t len) {
  RefHead g{~0u, 0, 0, 0, 0, false};
  const uint32_t c1 = wbyte(h, 1), c2 = wbyte(h, 2);
  uint32_t n1, L1, et, kl;
  if (c1 < 0x80u) {
    n1 = 1;
    L1 = c1;
    et = c2;
    kl = wbyte(h, 3);
  } else if (c2 < 0x80u) {
    n1 = 2;
    L1 = (c1 & 0x7Fu) | (c2 << 7);
    et = wbyte(h, 3);
    kl = wbyte(h, 4);
  } else {
    return g;
  }
  const uint32_t e1 = off + 1 + n1;
  if (len < 8 || wbyte(h, 0) != 0x0Au || et != 0x0Au || kl >= 0x80u || e1 + L1 > off + len || L1 < kl + 3 + 1 + 3)
    return g;
  const uint32_t rest = L1 - 3 - kl;  // gl + its varint
  if (rest == 129) return g;         // gl = 127 in two bytes
  const uint32_t n2 = rest <= 128 ? 1u : 2u, gl = rest - n2;
  g.gpos = e1 + 2 + kl;  // gpos + 4 <= the grant's end (gl >= 3)
  g.off = g.gpos + 1 + n2;
  g.len = gl;
  g.word = n2 == 1 ? 0x12u | (gl << 8) : 0x12u | (((gl & 0x7Fu) | 0x80u) << 8) | ((gl >> 7) << 16);
  g.mask = n2 == 1 ? 0xFFFFu : 0xFFFFFFu;
  g.ok = true;
  return g;
}

__device__ __forceinline__ RefGrant ref_grant_win(ByteReader& r, uint32_t off, uint32_t len) {
  RefGrant g;
  if (len < 8) return g;
  uint32_t h[4];
  window16(r.base, r.len, off, h);
  const RefHead rh = ref_head(h, off, len);
  if (rh.ok && (ld4(r.base, rh.gpos) & rh.mask) == rh.word) {
    g.off = rh.off;
    g.len = rh.len;
  }
  return g;
}


// One walk of a MultiGrant value: validates it as valid_multigrant does,
// counts its grants / grantSignatures entries on the wire, and records what
// the decode of the common shape needs -- the last entry of each map (its key
// and value as read_entry reads them) and the last serverId -- so that shape
// (one grants entry, at most one signature entry) is decoded without walking
// the value again.
struct MGScan {
  uint32_t nge, nse;
  Entry g, sg;               // last grants / grantSignatures entry
  uint32_t sid_off, sid_len;  // MultiGrant.serverId (last)
  bool first_nc;             // the first grants entry holds one value, parsed and not canonical
  bool same;                 // the grant's bytes equal the reference grant's (prep reuses its results)
  bool sig_key;              // mg_match: the signature entry's key is the grant's
  uint16_t signer;           // mg_match (MOCHI_W2_EARLY): the signer and key slot of the grant
  uint8_t slot;
};

__device__ bool valid_mg_scan(ByteReader& r, uint32_t off, uint32_t len, MGScan& m, const RefGrant ref = RefGrant{}) {
  uint32_t pos = off, end = off + len;
  Fld f;
  int rc;
  m.nge = m.nse = 0;
  m.sid_off = m.sid_len = 0;
  m.first_nc = m.sig_key = false;
#pragma unroll 1
  while ((rc = next_fld(r, pos, end, f)) > 0) {
    if (f.wt != 2) continue;
    if (f.field == 1) {
      m.nge++;
      if (!valid_leaf_read(r, f.off, f.len, 1, m.g, ref)) return false;
      if (m.nge == 1) m.first_nc = m.g.nval == 1 && !m.g.canon && !m.g.assumed;
    } else if (f.field >= 2 && f.field <= 4) {
      if (!valid_utf8(r, f.off, f.len)) return false;
      if (f.field == 4) {
        m.sid_off = f.off;
        m.sid_len = f.len;
      }
    } else if (f.field == 5) {
      m.nse++;
      if (!valid_leaf_read(r, f.off, f.len, 0, m.sg)) return false;
    }
  }
  m.same = m.nge == 1 && m.g.assumed;
  return rc == 0;
}


// signer = index of the key whose server id is the MultiGrant's serverId.
// The ids share their prefix ("server-"): the last word filters the
// candidates (its table-side load is the same address in every lane), and
// only a candidate is compared in full.
// `tab` (optional): the server ids staged in LDS by the block -- lengths, last
// words and the bytes themselves at word-aligned offsets -- so the lookup
// reads the MultiGrant's serverId once (independent word loads) and compares
// it with LDS words (the same address in every lane: a broadcast) instead of
// a byte-compare loop of dependent global loads per candidate.
constexpr uint32_t kIdTab = 64, kIdTabWords = 1024, kIdFast = 16;  // ids, LDS words, words compared from registers
constexpr uint32_t kSidWords = 15;  // serverId words hashed / compared from mg_match's window (<= 60 bytes)
struct IdTab {
  uint32_t len[kIdTab], tail[kIdTab], pos[kIdTab];  // pos: first LDS word, ~0 = not staged
  uint32_t hash[kIdTab];                            // sid_mix over the id's first kSidWords words
  uint32_t w[kIdTabWords];
};

__device__ __forceinline__ uint32_t sid_mix(uint32_t h, uint32_t w) { return (h ^ w) * 0x9E3779B1u; }

__device__ __forceinline__ void stage_ids(IdTab& tab, const uint8_t* __restrict__ ids,
                                          const uint32_t* __restrict__ id_off, uint32_t n_ids) {
  if (threadIdx.x == 0) {  // word positions (tiny: a handful of ids)
    uint32_t p = 0;
    for (uint32_t k = 0; k < n_ids && k < kIdTab; k++) {
      const uint32_t l = id_off[k + 1] - id_off[k], nw = (l + 3) / 4;
      tab.len[k] = l;
      tab.pos[k] = p + nw <= kIdTabWords ? p : ~0u;
      if (p + nw <= kIdTabWords) p += nw;
    }
  }
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < n_ids && k < kIdTab; k += blockDim.x) {
    const uint32_t o = id_off[k], l = tab.len[k];
    tab.tail[k] = l >= 4 ? ld4(ids, o + l - 4) : 0u;
    uint32_t h = 0;
    for (uint32_t t = 0; t < kSidWords; t++) {
      uint32_t v = 0;
      for (uint32_t j = 0; j < 4 && 4 * t + j < l; j++) v |= (uint32_t)ids[o + 4 * t + j] << (8 * j);
      h = sid_mix(h, v);
    }
    tab.hash[k] = h;
    if (tab.pos[k] != ~0u)
      for (uint32_t t = 0; 4 * t < l; t++) {
        uint32_t v = 0;
        for (uint32_t j = 0; j < 4 && 4 * t + j < l; j++) v |= (uint32_t)ids[o + 4 * t + j] << (8 * j);
        tab.w[tab.pos[k] + t] = v;
      }
  }
  __syncthreads();
}

__device__ __forceinline__ uint16_t find_signer(ByteReader& r, uint32_t so, uint32_t sl, const uint8_t* __restrict__ ids,
                                                const uint32_t* __restrict__ id_off, uint32_t n_ids,
                                                const IdTab* tab = nullptr) {
  const uint32_t tail = sl >= 4 ? ld4(r.base, so + sl - 4) : 0u;
  const bool fast = tab && sl >= 4 && sl <= 4 * kIdFast;
  if (fast && n_ids <= kIdTab) {
    // Usually exactly one staged id has this length and last word (server ids
    // end in distinct UUIDs): pick it first, then compare it in full ONCE.  A
    // loop that compares inside the candidate test runs that compare once per
    // distinct candidate among the wave's lanes (R times at R servers).
    uint32_t cand = ~0u, nc = 0;
    bool unstaged = false;
#pragma unroll 1
    for (uint32_t k = 0; k < n_ids; k++) {
      if (tab->len[k] != sl || tab->tail[k] != tail) continue;
      if (tab->pos[k] == ~0u) unstaged = true;
      if (nc++ == 0) cand = k;
    }
    if (nc == 0) return 0xFFFF;
    if (nc == 1 && !unstaged) {
      // the serverId's words from the aligned words that hold its bytes
      const uintptr_t a = (uintptr_t)(r.base + so);
      const uint32_t* wp = (const uint32_t*)(a & ~(uintptr_t)3);
      const uint32_t sh = 8 * (uint32_t)(a & 3);
      const uint32_t nw = (uint32_t)(((a & 3) + sl + 3) >> 2);  // aligned words holding a byte of it
      const uint32_t* w = tab->w + tab->pos[cand];
      uint32_t diff = 0, lo = wp[0];
#pragma unroll
      for (uint32_t t = 0; t < kIdFast; t++) {
        if (4 * t + 4 > sl) break;
        const uint32_t hi = t + 1 < nw ? wp[t + 1] : 0u;
        diff |= (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) ^ w[t];
        lo = hi;
      }
      return diff == 0 ? (uint16_t)cand : (uint16_t)0xFFFF;  // the tail matched already
    }
  }
#pragma unroll 1
  for (uint32_t k = 0; k < n_ids; k++) {
    if (tab && k < kIdTab) {
      if (tab->len[k] != sl || (sl >= 4 && tab->tail[k] != tail)) continue;
      if (fast && tab->pos[k] != ~0u) {
        // a candidate (usually the only one): its whole words against the
        // serverId's, loads independent of each other (no early exit), then
        // the last four bytes, already equal (the filter)
        uint32_t diff = 0;
        const uint32_t* w = tab->w + tab->pos[k];
#pragma unroll
        for (uint32_t t = 0; t < kIdFast; t++)
          if (4 * t + 4 <= sl) diff |= ld4(r.base, so + 4 * t) ^ w[t];
        if (diff == 0) return (uint16_t)k;
        continue;
      }
    } else {
      if (id_off[k + 1] - id_off[k] != sl) continue;
      if (sl >= 4 && ld4(ids, id_off[k] + sl - 4) != tail) continue;
    }
    if (bytes_eq(ids, id_off[k], r.base, so, sl)) return (uint16_t)k;
  }
  return 0xFFFF;
}

// key slot = index of the first op of the transaction naming `key`
__device__ __forceinline__ uint8_t find_key_slot(ByteReader& r, uint32_t tx_off, uint32_t tx_len, uint32_t ko,
                                                 uint32_t kl) {
  uint32_t pos = tx_off, end = tx_off + tx_len, j = 0;
  Fld f;
#pragma unroll 1
  while (next_fld(r, pos, end, f) > 0) {
    if (f.field != 1 || f.wt != 2) continue;
    uint32_t oo, ol;
    last_string(r, f.off, f.len, 2, oo, ol);
    if (key_eq(r, oo, ol, ko, kl)) return (uint8_t)j;
    j++;
  }
  return 0xFF;
}

// find_key_slot from level 1's record of the message's first kW2InlOps
// operations (cnt_o[m] = operations on the wire; more than recorded: the walk)
__device__ __forceinline__ uint8_t find_key_slot_rec(ByteReader& r, const W2Msg& s, uint32_t m, uint32_t ko,
                                                     uint32_t kl) {
  const uint32_t nops = s.cnt_o[m];
  if (nops > kW2InlOps) return find_key_slot(r, s.tx_off[m], s.tx_len[m], ko, kl);
  const uint2* q = (const uint2*)(s.inl_ops + (size_t)2 * kW2InlOps * m);
#pragma unroll 1
  for (uint32_t j = 0; j < nops; j++) {
    const uint2 o = q[j];
    if (key_eq(r, o.x, o.y, ko, kl)) return (uint8_t)j;
  }
  return 0xFF;
}

// find_signer from mg_match's serverId window (0x22 sl serverId, sl <= 60): the
// id of this length and hash (IdTab::hash) is compared word by word with the
// LDS copy -- no load of the message.  Several candidates (equal ids, a hash
// collision), an unstaged id or a table past kIdTab: find_signer.
__device__ __forceinline__ uint16_t signer_from_window(ByteReader& r, uint32_t so, uint32_t sl, const uint32_t (&sw)[16],
                                                       const uint8_t* __restrict__ ids,
                                                       const uint32_t* __restrict__ id_off, uint32_t n_ids,
                                                       const IdTab& tab) {
  uint32_t w[kSidWords], h = 0;
#pragma unroll
  for (int t = 0; t < (int)kSidWords; t++) {
    w[t] = __builtin_amdgcn_alignbit(sw[t + 1], sw[t], 16) & span_mask(t, 0, (int)sl);
    h = sid_mix(h, w[t]);
  }
  if (n_ids <= kIdTab) {
    uint32_t cand = ~0u, nc = 0;
#pragma unroll 1
    for (uint32_t k = 0; k < n_ids; k++)
      if (tab.len[k] == sl && tab.hash[k] == h && nc++ == 0) cand = k;
    if (nc == 0) return 0xFFFF;
    if (nc == 1 && tab.pos[cand] != ~0u) {
      const uint32_t* tw = tab.w + tab.pos[cand];
      uint32_t diff = 0;
#pragma unroll
      for (int t = 0; t < (int)kSidWords; t++)
        if (4u * t < sl) diff |= w[t] ^ tw[t];  // the LDS copy's last word is zero-padded, as w's
      return diff == 0 ? (uint16_t)cand : (uint16_t)0xFFFF;
    }
  }
  return find_signer(r, so, sl, ids, id_off, n_ids, &tab);
}

// find_key_slot_rec from mg_match's key window (0x0A kl key): each recorded
// operation key of this length is loaded as one window from two bytes before
// it (its tag and length) and compared with the key's bytes in registers
__device__ __forceinline__ uint8_t slot_from_window(ByteReader& r, const W2Msg& s, uint32_t m, uint32_t ko, uint32_t kl,
                                                    const uint32_t (&kw)[16]) {
  const uint32_t nops = s.cnt_o[m];
  if (nops > kW2InlOps) return find_key_slot(r, s.tx_off[m], s.tx_len[m], ko, kl);
  const uint2* q = (const uint2*)(s.inl_ops + (size_t)2 * kW2InlOps * m);
  uint8_t slot = 0xFF;
#pragma unroll
  for (uint32_t j = 0; j < kW2InlOps; j++) {
    if (j < nops) {
      const uint2 o = q[j];
      bool eq = o.y == kl;
      if (eq && kl != 0) {  // an operand1 is preceded by its tag and length: o.x >= 2
        uint32_t ow[16], diff = 0;
        window64(r.base, r.len, o.x - 2, ow);
#pragma unroll
        for (int t = 0; t < 16; t++) diff |= (ow[t] ^ kw[t]) & span_mask(t, 2, 2 + (int)kl);
        eq = diff == 0;
      }
      if (eq && slot == 0xFF) slot = (uint8_t)j;
    }
  }
  return slot;
}

// ---- the reference encoder's MultiGrant, matched from a few wide loads ------
// encode_multigrant / protobuf-java (MochiProtocol.proto:117-124 + field 5):
// one grant, fields in number order, each map entry its key then its value,
//   0x0A L1 { 0x0A kl key 0x12 gl Grant } 0x22 sl serverId
//   0x2A L5 { 0x0A kl key 0x12 0x80 0x02 signature[256] }
// the signature entry under the grant's key, key and serverId ASCII (kl, sl <= 60),
// L1 and gl one or two varint bytes, and the Grant itself in its common
// canonical shape 0x0A L objectId 0x10 ts 0x22 H transactionHash (<= 192 bytes,
// ASCII strings).  Every position follows from the first 16 bytes (the
// signature entry's from the value's end), so the loads after the first are
// independent of each other -- a handful of load latencies (header; key,
// serverId and framing windows; the operation key for the slot; the grant's
// windows; its timestamp) where the walk (next_fld / ByteReader::at) paid one
// per field, length and word.  Any difference returns false and valid_mg_scan
// decides; what this accepts, valid_mg_scan accepts with the same MGScan (one
// grants and one grantSignatures entry of one key and one value each, the grant
// parsed and canonical -- parse_grant_t's CANON rules).
#ifndef MOCHI_W2_MATCH
#define MOCHI_W2_MATCH 1  // A/B: 0 = every MultiGrant through valid_mg_scan
#endif
#ifndef MOCHI_W2_EARLY
// signer and key slot inside the match, from the key / serverId windows, and
// the grant's windows loaded only after them: those windows die first, 200 ->
// 161 VGPRs (3 waves per SIMD instead of 2), wire path -0.8 % (3.845 / 3.862
// vs 3.890 / 3.883 ms, alternated)
#define MOCHI_W2_EARLY 1
#endif
#ifndef MOCHI_W2_REFCMP
#define MOCHI_W2_REFCMP 1  // A/B: 0 = the matcher leaves the compare with the first grant to prep (+1.2 %)
#endif

// The common Grant shape, canonical and valid (ASCII strings), from its own
// windows: `hib` = bytes with the high bit set over the whole grant, w0 = its
// first 16 bytes, read from the timestamp's tag on with one more window.
__device__ __forceinline__ bool grant_match(const uint8_t* base, uint32_t mlen, uint32_t g0, uint32_t gl,
                                            const uint32_t (&w0)[16], uint32_t hib) {
  const uint32_t L = wbyte(w0, 1);
  if (wbyte(w0, 0) != 0x0Au || L == 0 || L >= 0x80u || L + 6 > gl) return false;
  uint32_t tb[4];
  window16(base, mlen, g0 + 2 + L, tb);
  if (wbyte(tb, 0) != 0x10u) return false;
  // timestamp: 1..9 varint bytes, minimal (nonzero last byte; a one-byte 0 is the default, never written)
  uint32_t k = 0, last = 0;
  bool end = false;
#pragma unroll
  for (uint32_t i = 1; i <= 9; i++) {
    const uint32_t c = wbyte(tb, i);
    if (!end) {
      k = i;
      last = c;
      end = c < 0x80u;
    }
  }
  if (!end || last == 0) return false;
  uint32_t c1 = 0, c2 = 0, tag = 0;  // the bytes after the timestamp (k + 1 <= 10)
#pragma unroll
  for (uint32_t i = 2; i <= 10; i++) {
    if (i == k + 1) {
      tag = wbyte(tb, i);
      c1 = wbyte(tb, i + 1);
      c2 = wbyte(tb, i + 2);
    }
  }
  if (tag != 0x22u) return false;
  uint32_t hl, nh;
  if (c1 < 0x80u) {
    hl = c1;
    nh = 1;
  } else if (c2 < 0x80u && c2 != 0) {
    hl = (c1 & 0x7Fu) | (c2 << 7);
    nh = 2;
  } else {
    return false;
  }
  const uint32_t hp = 2 + L + 1 + k + 1 + nh;
  return hl != 0 && hp + hl == gl && hib == (k - 1) + (nh - 1);
}

// kw / sw (out): the windows at the grants entry (0x0A kl key) and at the
// serverId (0x22 sl serverId), for the signer and key-slot lookups
// (rvo, rvl): the message's first certificate entry's value (ref_head: the grant
// the prep hint compares with), ~0 = this is that entry
__device__ bool mg_match(ByteReader& r, uint32_t vo, uint32_t vl, uint32_t rvo, uint32_t rvl, MGScan& m,
                         uint32_t (&kw)[16], uint32_t (&sw)[16], const W2Msg& s, uint32_t mi,
                         const uint8_t* __restrict__ ids, const uint32_t* __restrict__ id_off, uint32_t n_ids,
                         const IdTab& tab) {
  const uint8_t* base = r.base;
  const uint32_t mlen = r.len;
  if (vl < 272) return false;
  uint32_t h[4], rh[4] = {0u, 0u, 0u, 0u};
  window16(base, mlen, vo, h);
  if (MOCHI_W2_REFCMP && rvo != ~0u && rvl >= 8) window16(base, mlen, rvo, rh);  // beside this value's header
  const RefHead ref = MOCHI_W2_REFCMP && rvo != ~0u ? ref_head(rh, rvo, rvl) : RefHead{~0u, 0, 0, 0, 0, false};
  const uint32_t c1 = wbyte(h, 1), c2 = wbyte(h, 2);
  uint32_t n1, L1, et, kl;
  if (c1 < 0x80u) {
    n1 = 1;
    L1 = c1;
    et = c2;
    kl = wbyte(h, 3);
  } else if (c2 < 0x80u) {
    n1 = 2;
    L1 = (c1 & 0x7Fu) | (c2 << 7);
    et = wbyte(h, 3);
    kl = wbyte(h, 4);
  } else {
    return false;
  }
  if (wbyte(h, 0) != 0x0Au || et != 0x0Au || kl > 60) return false;
  const uint32_t e1 = vo + 1 + n1, s_tag = e1 + L1, end = vo + vl;
  const uint32_t p5 = end - 264 - kl;  // the signature entry's tag (its key: kl bytes, as the grant's)
  if (L1 < kl + 3 + 1 + 8 || s_tag + 2 > p5 || p5 - s_tag - 2 > 60) return false;
  const uint32_t sl = p5 - s_tag - 2;
  const uint32_t rest = L1 - 3 - kl;  // gl + its varint
  if (rest == 129) return false;     // gl = 127 in two bytes: not minimal
  const uint32_t n2 = rest <= 128 ? 1u : 2u, gl = rest - n2;
  const uint32_t gpos = e1 + 2 + kl, g0 = gpos + 1 + n2;
  if (gl > 192) return false;
  // ---- independent loads: framing words, key / serverId windows, the grant ----
  const uint32_t gh = ld4(base, gpos), t5 = ld4(base, p5), sh = ld4(base, end - 259);
  const bool cmp = ref.ok && ref.len == gl;  // the first grant's header word is checked below
  const uint32_t rgh = cmp ? ld4(base, ref.gpos) : 0u;
  uint32_t(&k1)[16] = kw;
  uint32_t k4[16];
  window64(base, mlen, e1, k1);      // 0x0A kl key
  window64(base, mlen, p5 + 3, k4);  // 0x0A kl key (the signature entry's)
  window64(base, mlen, s_tag, sw);   // 0x22 sl serverId
  const uint32_t L5 = 261 + kl;
  bool ok = (gh & 0xFFu) == 0x12u &&
            (n2 == 1 ? ((gh >> 8) & 0xFFu) == gl : ((gh >> 8) & 0xFFFFu) == (((gl & 0x7Fu) | 0x80u) | ((gl >> 7) << 8))) &&
            t5 == (0x2Au | (((L5 & 0x7Fu) | 0x80u) << 8) | ((L5 >> 7) << 16) | (0x0Au << 24)) &&
            (sh & 0xFFFFFFu) == 0x028012u && (sw[0] & 0xFFFFu) == (0x22u | (sl << 8));
  uint32_t kdiff = 0, hi = 0;
#pragma unroll
  for (int t = 0; t < 16; t++) {
    kdiff |= (k1[t] ^ k4[t]) & span_mask(t, 0, 2 + (int)kl);
    hi |= k1[t] & span_mask(t, 2, 2 + (int)kl);
    hi |= sw[t] & span_mask(t, 2, 2 + (int)sl);
  }
  ok = ok && kdiff == 0 && (hi & 0x80808080u) == 0;
#if MOCHI_W2_EARLY
  m.signer = ok ? signer_from_window(r, s_tag + 2, sl, sw, ids, id_off, n_ids, tab) : (uint16_t)0xFFFF;
  m.slot = ok ? slot_from_window(r, s, mi, e1 + 2, kl, k1) : (uint8_t)0xFF;
  const uint32_t dep = kdiff | hi | m.signer | m.slot;
#else
  const uint32_t dep = kdiff | hi;
#endif
  // ---- the grant: its high-bit count, its first window, and the compare with the reference grant ----
  uint32_t w0[16], hib = 0, gdiff = 0;
  uint32_t ga = g0, ra = ref.off;
#if MOCHI_W2_EARLY  // the grant's windows only after the key / serverId ones are used
  asm volatile("" : "+v"(ga), "+v"(ra) : "v"(dep));
#else
  (void)dep;
#endif
#pragma unroll
  for (int c = 0; c < 3; c++) {
    if (64u * c < gl) {
      uint32_t w[16], v[16];
      window64(base, mlen, ga + 64 * c, w);
      if (cmp) window64(base, mlen, ra + 64 * c, v);
#pragma unroll
      for (int t = 0; t < 16; t++) {
        const uint32_t mk = span_mask(t, 0, (int)gl - 64 * c);
        hib += __builtin_popcount(w[t] & mk & 0x80808080u);
        if (cmp) gdiff |= (w[t] ^ v[t]) & mk;
        if (c == 0) w0[t] = w[t];
      }
    }
  }
  if (!ok || !grant_match(base, mlen, g0, gl, w0, hib)) return false;
  m.nge = m.nse = 1;
  m.g = Entry{e1 + 2, kl, g0, gl, 1, true, false};
  m.sg = Entry{p5 + 5, kl, end - 256, 256, 1, false, false};
  m.sid_off = s_tag + 2;
  m.sid_len = sl;
  m.first_nc = false;
  m.same = cmp && gdiff == 0 && (rgh & ref.mask) == ref.word;
  m.sig_key = true;
  return true;
}

// Certificate entries (compact, in wire order per message): message index,
// key and value slices (message-relative), the index of the entry holding the
// key's final value (~0 unless this entry is the key's first), and the number
// of distinct grants of a final-value entry.
// A decoded MultiGrant with one distinct grant (the common shape) also leaves
// its emit record here -- grant value slice, signature offset (message-
// relative, ~0 = none), signer << 8 | key slot -- written by k_w2_mg while the
// bytes are hot, so k_w2_emit_mg need not walk it again.
struct CE {
  uint32_t *msg, *koff, *klen, *voff, *vlen, *last, *ng;
  uint32_t *r_goff, *r_glen, *r_sig, *r_sk;
};
static_assert(sizeof(CE) == kW2CeArrays * sizeof(uint32_t*), "kW2CeArrays (w2.h) counts the CE arrays");
__host__ __device__ inline CE ce_view(uint32_t* p, uint32_t cap) {
  const size_t c = cap;
  return CE{p, p + c, p + 2 * c, p + 3 * c, p + 4 * c, p + 5 * c, p + 6 * c, p + 7 * c, p + 8 * c, p + 9 * c, p + 10 * c};
}

// The distinct grants of one decoded MultiGrant value [mo, mo+ml), in map
// order: sink(grant value off, len, signer, signature off or ~0, key slot),
// offsets message-relative.
// One pass for k_w2_mg: the distinct grants of the decoded MultiGrant value,
// each canonical (else false: fast-path exit), counted into ng; the first
// one's emit record (grant slice, signer, signature offset, key slot) goes to
// rec(...).  The map is
// resolved once and the signature / key-slot lookups run for the first grant
// only (k_w2_emit_mg redoes them for a MultiGrant with several grants).
template <typename Rec>
__device__ bool mg_decode_first(ByteReader& r, uint32_t mo, uint32_t ml, uint32_t tx_off, uint32_t tx_len,
                                const uint8_t* __restrict__ ids, const uint32_t* __restrict__ id_off, uint32_t n_ids,
                                uint32_t& ng, Rec&& rec) {
  ng = 0;
  return for_map(r, mo, ml, 1, [&](const Entry& ge, const Entry& gv) -> bool {
    if (!grant_canonical(r, gv.voff, gv.vlen)) return false;
    if (ng++ == 0) {
      uint16_t signer;
      {
        uint32_t so, sl;
        last_string(r, mo, ml, 4, so, sl);  // MultiGrant.serverId
        signer = find_signer(r, so, sl, ids, id_off, n_ids);
      }
      uint32_t s_off = 0, s_len = 0;
      bool have = false;
      {
        uint32_t pos = mo, end = mo + ml;
        Fld f;
#pragma unroll 1
        while (next_fld(r, pos, end, f) > 0) {
          if (f.field != 5 || f.wt != 2) continue;
          Entry se;
          read_entry(r, f.off, f.len, se);
          if (key_eq(r, se.koff, se.klen, ge.koff, ge.klen)) {
            have = true;
            s_off = se.voff;
            s_len = se.vlen;
          }
        }
      }
      const uint8_t key = find_key_slot(r, tx_off, tx_len, ge.koff, ge.klen);
      rec(gv.voff, gv.vlen, signer, have && s_len == MOCHI_RSA_BYTES ? s_off : ~0u, key);
    }
    return true;
  });
}

template <typename Sink>
__device__ void walk_mg(ByteReader& r, uint32_t mo, uint32_t ml, uint32_t tx_off, uint32_t tx_len,
                        const uint8_t* __restrict__ ids, const uint32_t* __restrict__ id_off, uint32_t n_ids,
                        Sink&& sink) {
  uint16_t signer;
  {
    uint32_t so, sl;
    last_string(r, mo, ml, 4, so, sl);  // MultiGrant.serverId
    signer = find_signer(r, so, sl, ids, id_off, n_ids);
  }
  for_map(r, mo, ml, 1, [&](const Entry& ge, const Entry& gv) -> bool {
    // grantSignatures[key]: the last entry with this key, its (last) value
    uint32_t s_off = 0, s_len = 0;
    bool have = false;
    {
      uint32_t pos = mo, end = mo + ml;
      Fld f;
#pragma unroll 1
      while (next_fld(r, pos, end, f) > 0) {
        if (f.field != 5 || f.wt != 2) continue;
        Entry se;
        read_entry(r, f.off, f.len, se);
        if (key_eq(r, se.koff, se.klen, ge.koff, ge.klen)) {
          have = true;
          s_off = se.voff;
          s_len = se.vlen;
        }
      }
    }
    // key slot = index of the first op naming this grant's key (that op's own slot)
    uint8_t key = 0xFF;
    {
      uint32_t pos = tx_off, end = tx_off + tx_len, j = 0;
      Fld f;
#pragma unroll 1
      while (next_fld(r, pos, end, f) > 0) {
        if (f.field != 1 || f.wt != 2) continue;
        uint32_t ko, kl;
        last_string(r, f.off, f.len, 2, ko, kl);
        if (key_eq(r, ko, kl, ge.koff, ge.klen)) {
          key = (uint8_t)j;
          break;
        }
        j++;
      }
    }
    sink(gv.voff, gv.vlen, signer, have && s_len == MOCHI_RSA_BYTES ? s_off : ~0u, key);
    return true;
  });
}

__device__ __forceinline__ void emit_grant(const W2Out& out, uint32_t g, uint64_t msg_off, uint32_t goff, uint32_t glen,
                                           uint16_t signer, uint32_t sig_off, uint8_t key, uint32_t same = ~0u) {
  out.grant_off[g] = msg_off + goff;
  if (out.grant_same) out.grant_same[g] = same != ~0u ? same : g;
  out.grant_len[g] = glen;
  out.signer[g] = signer;
  // the 256 signature bytes are gathered by k_w2_sig (coalesced, 16 lanes per grant)
  out.sig_src[g] = sig_off != ~0u ? msg_off + sig_off : ~0ull;
  out.grant_key[g] = key;
}

// A small batch (M < kW2SmallM messages) runs the decode's two scans inside
// one 1024-thread block of the kernel after each (k_w2_entries, k_w2_final)
// instead of as hipcub launches of their own: each launch is ~5 us of dispatch
// on an otherwise idle GPU, a batcher flush carries one or two messages.
constexpr uint32_t kW2SmallM = 1024;

// Exclusive scan of v over the 1024 threads of the block (16 waves): a shuffle
// scan per wave, then one over the wave totals.  lds: 33 words of its own (a
// second scan in the same kernel takes other words); total = the block's sum.
__device__ __forceinline__ uint32_t block_scan_excl(uint32_t v, uint32_t* lds, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += y;
  }
  if (lane == 63) lds[wid] = incl;
  __syncthreads();
  if (wid == 0) {
    const uint32_t wt = lane < nw ? lds[lane] : 0u;
    uint32_t wi = wt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(wi, d, 64);
      if (lane >= (uint32_t)d) wi += y;
    }
    if (lane < nw) lds[16 + lane] = wi - wt;
    if (lane == nw - 1) lds[32] = wi;
  }
  __syncthreads();
  total = lds[32];
  return lds[16 + wid] + incl - v;
}

// Level 1.  cnt_o[m] = operations on the wire (k_w2_final turns it into the
// decoded count).  Element M of cnt_ce is the scan's extra element.
// three waves per SIMD (the register cap keeps the level-1 walk at the occupancy
// it had before the level-2 scan shared its leaf walker)
#ifndef MOCHI_W2MSG_WAVES
#define MOCHI_W2MSG_WAVES 4  // amdgpu_waves_per_eu (126 VGPRs, no spills; 3 waves: wire path 1.2 % slower, 5: 0.4 %)
#endif
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MOCHI_W2MSG_WAVES))) void k_w2_msg(const uint8_t* __restrict__ wire, const uint64_t* __restrict__ moff,
                                                const uint32_t* __restrict__ mlen, uint32_t M, W2Msg s) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m > M) return;
  if (m == M) {
    s.cnt_ce[M] = 0;
    return;
  }
  ByteReader r;
  r.init(wire + moff[m], mlen[m]);
  uint32_t nce = 0, nops = 0, wo = 0, wl = 0, to = 0, tl = 0;
  uint32_t* inl = s.inl + (size_t)4 * kW2InlEntries * m;
  uint32_t* inl_ops = s.inl_ops + (size_t)2 * kW2InlOps * m;
  const uint32_t bits = msg_level(r, nce, nops, wo, wl, to, tl, inl, inl_ops);
  if (bits) nce = nops = 0;
  s.cnt_ce[m] = nce;
  s.cnt_o[m] = nops;
  s.st_bits[m] = bits;
  s.wc_off[m] = wo;
  s.wc_len[m] = wl;
  s.tx_off[m] = to;
  s.tx_len[m] = tl;
}

// Level 1, second walk: the certificate entries into the compact list.
// kSmall: one block, M < kW2SmallM; the entry offsets (ce_base, the scan of
// cnt_ce) are computed here first.
template <bool kSmall>
__global__ __launch_bounds__(kSmall ? 1024 : 256) void k_w2_entries(const uint8_t* __restrict__ wire,
                                                                    const uint64_t* __restrict__ moff,
                                                                    const uint32_t* __restrict__ mlen, uint32_t M,
                                                                    W2Msg s, CE ce) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t e;
  if constexpr (kSmall) {
    __shared__ uint32_t lds[33];
    const uint32_t v = m < M ? s.cnt_ce[m] : 0u;
    uint32_t total;
    e = block_scan_excl(v, lds, total);
    if (m <= M) s.ce_base[m] = e;  // ce_base[M] = the entry total (k_w2_mg, k_w2_emit_mg)
  }
  if (m >= M) return;
  const uint32_t nce = s.cnt_ce[m];
  if (nce == 0) return;
  if constexpr (!kSmall) e = s.ce_base[m];
  if (nce <= kW2InlEntries) {  // recorded by level 1: copy
    const uint4* q = (const uint4*)(s.inl + (size_t)4 * kW2InlEntries * m);
#pragma unroll 4
    for (uint32_t j = 0; j < nce; j++, e++) {
      const uint4 v = q[j];
      ce.msg[e] = m;
      ce.koff[e] = v.x;
      ce.klen[e] = v.y;
      ce.voff[e] = v.z;
      ce.vlen[e] = v.w;
    }
    return;
  }
  ByteReader r;
  r.init(wire + moff[m], mlen[m]);
  uint32_t pos = s.wc_off[m];
  const uint32_t end = pos + s.wc_len[m];
  Fld f;
#pragma unroll 1
  while (next_fld(r, pos, end, f) > 0) {
    if (f.field != 1 || f.wt != 2) continue;
    Entry x;
    read_entry(r, f.off, f.len, x);
    ce.msg[e] = m;
    ce.koff[e] = x.koff;
    ce.klen[e] = x.klen;
    ce.voff[e] = x.voff;
    ce.vlen[e] = x.vlen;
    e++;
  }
}

// The first grant of a MultiGrant value in the reference encoder's layout: its
// first field a grants entry holding exactly a key and one value (0x0A klen key
// 0x12 glen grant).  Only the framing is read; anything else: none.
__device__ RefGrant first_grant(ByteReader& r, uint32_t off, uint32_t len) {
  RefGrant g;
  uint32_t pos = off, end = off + len, l1, kl, gl;
  if (pos >= end || r.at(pos) != 0x0Au) return g;
  pos++;
  if (!vlen(r, pos, end, l1)) return g;
  const uint32_t e1 = pos + l1;
  if (pos >= e1 || r.at(pos) != 0x0Au) return g;
  pos++;
  if (!vlen(r, pos, e1, kl)) return g;
  pos += kl;
  if (pos >= e1 || r.at(pos) != 0x12u) return g;
  pos++;
  if (!vlen(r, pos, e1, gl) || pos + gl != e1) return g;
  g.off = pos;
  g.len = gl;
  return g;
}

// Status bits beside kStMal / kStFb (k_w2_mg): a lane took a grant's canonical
// form from the message's first grant (kStAssume), and that grant is not
// canonical (kStFirstNC): together they make the message FALLBACK (k_w2_final),
// as the lane's own parse would have.
constexpr uint32_t kStAssume = 4u, kStFirstNC = 8u;

// Level 2 (lane = certificate entry; grid-stride over the device-side total).
// MOCHI_W2_STAMPS (measurement builds only, `make ab VSRC=w2_decode`): per
// wave, s_memtime ticks spent between the marks of k_w2_mg (dedup, scan,
// canonical check, signer, key slot, records), read back with
// mochi_debug_w2_stamps() (scripts/w2_stamps.py)
#ifndef MOCHI_W2_STAMPS
#define MOCHI_W2_STAMPS 0
#endif
#if MOCHI_W2_STAMPS
__device__ unsigned long long g_w2_stamps[16384][8];
#endif
struct W2Stamps {
#if MOCHI_W2_STAMPS
  uint64_t acc[7] = {0, 0, 0, 0, 0, 0, 0}, last = 0;
  __device__ __forceinline__ void mark(int i) {
    __builtin_amdgcn_sched_barrier(0);
    const uint64_t t = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    if (i) acc[i] += t - last;
    last = t;
  }
  __device__ __forceinline__ void store() {
    const uint32_t w = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if ((threadIdx.x & 63) == 0 && w < 16384) {
      for (int i = 1; i < 7; i++) g_w2_stamps[w][i] = acc[i];
      g_w2_stamps[w][7] = 1;
    }
  }
#else
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void store() {}
#endif
};

#ifndef MOCHI_W2MG_WAVES
#define MOCHI_W2MG_WAVES 0  // A/B builds: amdgpu_waves_per_eu for k_w2_mg (0 = the compiler's choice)
#endif
#if MOCHI_W2MG_WAVES
#define MOCHI_W2MG_ATTR __attribute__((amdgpu_waves_per_eu(MOCHI_W2MG_WAVES)))
#else
#define MOCHI_W2MG_ATTR
#endif
// (round 3, at 150 registers: capping for 4 or 5 waves per SIMD measured 1.4 %
// and 35 % slower)
__global__ __launch_bounds__(256) MOCHI_W2MG_ATTR void k_w2_mg(
    const uint8_t* __restrict__ wire, const uint64_t* __restrict__ moff, const uint32_t* __restrict__ mlen, uint32_t M,
    W2Msg s, CE ce, const uint8_t* __restrict__ ids, const uint32_t* __restrict__ id_off, uint32_t n_ids) {
  __shared__ IdTab tab;
  stage_ids(tab, ids, id_off, n_ids);
  const uint32_t total = s.ce_base[M];
  W2Stamps stp;
#pragma unroll 1
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x) {
    stp.mark(0);
    const uint32_t m = ce.msg[e];
    ByteReader r;
    r.init(wire + moff[m], mlen[m]);
    const uint32_t b0 = s.ce_base[m], b1 = s.ce_base[m + 1], ko = ce.koff[e], kl = ce.klen[e];
    bool first = true;
    uint32_t last = e;
#pragma unroll 1
    for (uint32_t j = b0; j < b1; j++)
      if (j != e && key_eq(r, ce.koff[j], ce.klen[j], ko, kl)) {
        if (j < e) first = false;
        else last = j;
      }
    const uint32_t vo = ce.voff[e], vl = ce.vlen[e];
    uint32_t bits = 0, ng = 0;
    MGScan sc;
    // the R MultiGrants of an honest certificate carry the same grant bytes:
    // a grant equal to the first MultiGrant's first grant is parsed by that
    // entry's lane only
    const uint32_t rvo = e == b0 ? ~0u : ce.voff[b0], rvl = e == b0 ? 0u : ce.vlen[b0];
    // the emit record, read by k_w2_emit_mg when ng == 1
    auto rec = [&](uint32_t go, uint32_t gl, uint16_t sg, uint32_t so, uint8_t key) {
      ce.r_goff[e] = go;
      ce.r_glen[e] = gl;
      ce.r_sig[e] = so;
      ce.r_sk[e] = (uint32_t)sg << 8 | key;
    };
    stp.mark(1);
    uint32_t kw[16], sw[16];
    const bool fast = MOCHI_W2_MATCH && mg_match(r, vo, vl, rvo, rvl, sc, kw, sw, s, m, ids, id_off, n_ids, tab);
    bool valid = fast;
    if (!fast) {
      const RefGrant ref = rvo == ~0u     ? RefGrant{}
                           : MOCHI_W2_MATCH ? ref_grant_win(r, rvo, rvl)
                                            : first_grant(r, rvo, rvl);
      valid = valid_mg_scan(r, vo, vl, sc, ref);
    }
    stp.mark(2);
    if (valid && e == b0 && sc.first_nc) bits |= kStFirstNC;  // the reference grant of this message's other lanes
    if (!valid) {
      bits = kStMal;
    } else if (last == e) {  // this entry's value is the key's final one: it is decoded
      if (sc.nge == 1 && sc.nse <= 1) {
        // the common shape, from the scan: the one grants entry is its key's
        // first and last; its signature is the signature entry if that entry's
        // key is the grant's (walk_mg's lookup over one entry)
        const bool canon = sc.g.nval <= 1 && sc.g.canon;  // decided by the validating parse
        if (canon && sc.g.assumed) bits |= kStAssume;
        stp.mark(3);
        if (!canon) {
          bits |= kStFb;
        } else {
          ng = 1;
          const bool have = sc.nse == 1 && (sc.sig_key || key_eq(r, sc.sg.koff, sc.sg.klen, sc.g.koff, sc.g.klen));
          const uint16_t signer = fast ? (MOCHI_W2_EARLY ? sc.signer
                                                         : signer_from_window(r, sc.sid_off, sc.sid_len, sw, ids, id_off,
                                                                              n_ids, tab))
                                       : find_signer(r, sc.sid_off, sc.sid_len, ids, id_off, n_ids, &tab);
          stp.mark(4);
          const uint8_t slot = fast ? (MOCHI_W2_EARLY ? sc.slot : slot_from_window(r, s, m, sc.g.koff, sc.g.klen, kw))
                                    : find_key_slot_rec(r, s, m, sc.g.koff, sc.g.klen);
          stp.mark(5);
          rec(sc.g.voff, sc.g.vlen, signer, have && sc.sg.vlen == MOCHI_RSA_BYTES ? sc.sg.voff : ~0u, slot);
          // bit 31: its bytes are the message's first grant's (k_w2_emit_mg); bit 30: the
          // emitted grant IS the value's first grant (one grants entry, one value), so on
          // the first entry it is the grant the other entries were compared with
          ce.r_sk[e] |= (sc.same ? 1u << 31 : 0u) | 1u << 30;
        }
      } else if (sc.nge > kMaxGrantsPerMG || sc.nse > kMaxSigEntries ||
                 !mg_decode_first(r, vo, vl, s.tx_off[m], s.tx_len[m], ids, id_off, n_ids, ng, rec)) {
        bits |= kStFb;
      }
    }
    ce.last[e] = first ? last : ~0u;
    ce.ng[e] = (bits & (kStMal | kStFb)) ? 0u : ng;
    if (bits) atomicOr(s.st_bits + m, bits);
    stp.mark(6);
  }
  stp.store();
}

// Per message: final status and the decoded counts (k_w2_final).
__device__ __forceinline__ void w2_final_msg(uint32_t m, const uint32_t* __restrict__ flags_off, const W2Msg& s,
                                             const CE& ce, uint32_t* __restrict__ cnt_g, uint32_t* __restrict__ cnt_m,
                                             uint8_t* __restrict__ status, uint4* __restrict__ cnt4, uint32_t& ng,
                                             uint32_t& no, uint32_t& nm) {
  uint32_t bits = s.st_bits[m];
  if ((bits & kStAssume) && (bits & kStFirstNC)) bits |= kStFb;  // a lane's assumed-canonical grant was not
  uint32_t st = (bits & kStMal) ? MOCHI_MSG_MALFORMED : (bits & kStFb) ? MOCHI_MSG_FALLBACK : MOCHI_MSG_OK;
  no = s.cnt_o[m];
  ng = 0;
  nm = 0;
  if (st == MOCHI_MSG_OK && flags_off && flags_off[m + 1] - flags_off[m] != no) st = MOCHI_MSG_OPS_MISMATCH;
  if (st == MOCHI_MSG_OK) {
#pragma unroll 1
    for (uint32_t j = s.ce_base[m]; j < s.ce_base[m + 1]; j++) {
      const uint32_t L = ce.last[j];
      if (L != ~0u) {
        nm++;
        ng += ce.ng[L];
      }
    }
  } else {
    no = 0;
  }
  cnt_g[m] = ng;
  s.cnt_o[m] = no;
  cnt_m[m] = nm;
  cnt4[m] = make_uint4(ng, no, nm, 0);
  status[m] = (uint8_t)st;
}

// kSmall: one block, M < kW2SmallM; the packed scan of (grants, ops,
// MultiGrants) into off4 is done here as well.
template <bool kSmall>
__global__ __launch_bounds__(kSmall ? 1024 : 256) void k_w2_final(uint32_t M, const uint32_t* __restrict__ flags_off,
                                                                  W2Msg s, CE ce, uint32_t* __restrict__ cnt_g,
                                                                  uint32_t* __restrict__ cnt_m,
                                                                  uint8_t* __restrict__ status, uint4* __restrict__ cnt4,
                                                                  uint4* __restrict__ off4) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if constexpr (kSmall) {
    __shared__ uint32_t lds[3][33];
    uint32_t ng = 0, no = 0, nm = 0;
    if (m < M) w2_final_msg(m, flags_off, s, ce, cnt_g, cnt_m, status, cnt4, ng, no, nm);
    uint32_t tg, to, tm;
    const uint32_t eg = block_scan_excl(ng, lds[0], tg), eo = block_scan_excl(no, lds[1], to),
                   em = block_scan_excl(nm, lds[2], tm);
    if (m < M) off4[m] = make_uint4(eg, eo, em, 0);
    if (m == M) {
      cnt_g[M] = 0;
      s.cnt_o[M] = 0;
      cnt_m[M] = 0;
      cnt4[M] = make_uint4(0, 0, 0, 0);
      off4[M] = make_uint4(tg, to, tm, 0);  // the totals (the host reads them)
    }
    return;
  }
  if (m > M) return;
  if (m == M) {  // the scan's extra element: totals land at [M]
    cnt_g[M] = 0;
    s.cnt_o[M] = 0;
    cnt_m[M] = 0;
    cnt4[M] = make_uint4(0, 0, 0, 0);
    return;
  }
  uint32_t ng, no, nm;
  w2_final_msg(m, flags_off, s, ce, cnt_g, cnt_m, status, cnt4, ng, no, nm);
}

// Emit, lane = certificate entry: a key's first entry writes its MultiGrant
// (the final value's grants) at the position its predecessors leave.
// Certificate entry e: a key's first entry writes its MultiGrant.
__device__ __forceinline__ void emit_mg_entry(uint32_t e, const uint8_t* __restrict__ wire,
                                              const uint64_t* __restrict__ moff, const uint32_t* __restrict__ mlen,
                                              const W2Msg& s, const CE& ce, const uint8_t* __restrict__ status,
                                              const uint4* __restrict__ off4, const uint8_t* __restrict__ ids,
                                              const uint32_t* __restrict__ id_off, uint32_t n_ids, const W2Out& out) {
  const uint32_t L = ce.last[e];
  if (L == ~0u) return;
  const uint32_t m = ce.msg[e];
  if (status[m] != MOCHI_MSG_OK) return;
  uint32_t idx = 0, gb = 0;
#pragma unroll 1
  for (uint32_t j = s.ce_base[m]; j < e; j++) {
    const uint32_t Lj = ce.last[j];
    if (Lj != ~0u) {
      idx++;
      gb += ce.ng[Lj];
    }
  }
  const uint4 base = off4[m];  // (grants, ops, MultiGrants) before message m
  uint32_t g = base.x + gb;
  out.mg_grant_off[base.z + idx] = g;  // this MultiGrant's first grant
  const uint64_t mo = moff[m];
  if (ce.ng[L] == 1) {  // recorded by k_w2_mg
    const uint32_t sk = ce.r_sk[L];
    // the same bytes as the message's first grant -- the first one emitted
    // (base.x) when the first entry holds its key's final value, one grant
    const uint32_t b0 = s.ce_base[m];
    const bool same = (sk >> 31) && L != b0 && ce.last[b0] == b0 && ce.ng[b0] == 1 && ((ce.r_sk[b0] >> 30) & 1u);
    emit_grant(out, g, mo, ce.r_goff[L], ce.r_glen[L], (uint16_t)(sk >> 8), ce.r_sig[L], (uint8_t)sk,
               same ? base.x : ~0u);
    return;
  }
  ByteReader r;
  r.init(wire + mo, mlen[m]);
  walk_mg(r, ce.voff[L], ce.vlen[L], s.tx_off[m], s.tx_len[m], ids, id_off, n_ids,
          [&](uint32_t go, uint32_t gl, uint16_t sg, uint32_t so, uint8_t key) {
            emit_grant(out, g++, mo, go, gl, sg, so, key);
          });
}

__global__ __launch_bounds__(256) void k_w2_emit_mg(const uint8_t* __restrict__ wire, const uint64_t* __restrict__ moff,
                                                    const uint32_t* __restrict__ mlen, uint32_t M, W2Msg s, CE ce,
                                                    const uint8_t* __restrict__ status,
                                                    const uint4* __restrict__ off4, const uint8_t* __restrict__ ids,
                                                    const uint32_t* __restrict__ id_off, uint32_t n_ids, W2Out out) {
  const uint32_t total = s.ce_base[M];
#pragma unroll 1
  for (uint32_t e = blockIdx.x * blockDim.x + threadIdx.x; e < total; e += gridDim.x * blockDim.x)
    emit_mg_entry(e, wire, moff, mlen, s, ce, status, off4, ids, id_off, n_ids, out);
}

// Emit, lane = message: the operations (key slot = index of the first op
// naming the same operand1) and the MultiGrant CSR terminator.
__device__ __forceinline__ void emit_ops_msg(uint32_t m, const uint8_t* __restrict__ wire,
                                             const uint64_t* __restrict__ moff, const uint32_t* __restrict__ mlen,
                                             uint32_t M, const W2Msg& s, const uint8_t* __restrict__ status,
                                             const uint4* __restrict__ off4, uint32_t* __restrict__ g_base,
                                             uint32_t* __restrict__ o_base, uint32_t* __restrict__ m_base,
                                             const uint32_t* __restrict__ flags_off,
                                             const uint8_t* __restrict__ flags_in, const int64_t* __restrict__ ots_in,
                                             const W2Out& out) {
  // the packed scan unpacked into the batch's three CSR arrays ([M] = totals)
  const uint4 base = off4[m];
  g_base[m] = base.x;
  o_base[m] = base.y;
  m_base[m] = base.z;
  if (m == M) {
    out.mg_grant_off[base.z] = base.x;  // CSR terminator: n_mgs -> N
    return;
  }
  if (status[m] != MOCHI_MSG_OK) return;
  ByteReader r;
  r.init(wire + moff[m], mlen[m]);
  const uint64_t msg_off = moff[m];
  const uint32_t ob = base.y, tx_off = s.tx_off[m], end = tx_off + s.tx_len[m];
  const uint8_t* fl = flags_off ? flags_in + flags_off[m] : nullptr;
  const int64_t* ot = flags_off && ots_in ? ots_in + flags_off[m] : nullptr;
  uint32_t no = 0, pos = tx_off;
  Fld f;
#pragma unroll 1
  while (next_fld(r, pos, end, f) > 0) {
    if (f.field != 1 || f.wt != 2) continue;
    uint32_t ko, kl;
    last_string(r, f.off, f.len, 2, ko, kl);
    uint32_t slot = no, j = 0, p2 = tx_off;
    Fld g;
#pragma unroll 1
    while (j < no && next_fld(r, p2, end, g) > 0) {
      if (g.field != 1 || g.wt != 2) continue;
      uint32_t jo, jl;
      last_string(r, g.off, g.len, 2, jo, jl);
      if (key_eq(r, jo, jl, ko, kl)) {
        slot = j;
        break;
      }
      j++;
    }
    // Operation.action (enum, proto3 open): anything but WRITE = 2 / DELETE = 1
    // fails applyOperation / readOperation (InMemoryDataStore.java:529, :562);
    // an empty operand1 is never write-locked (:339-358)
    const int32_t action = (int32_t)(uint32_t)last_varint(r, f.off, f.len, 1);
    const uint32_t notw = (action != 1 && action != 2) || kl == 0 ? MOCHI_OP_NOT_WRITE : 0;
    out.op_key[ob + no] = (uint8_t)slot;
    out.op_flags[ob + no] = (uint8_t)((fl ? fl[no] : (uint8_t)(MOCHI_OP_LOCAL | MOCHI_OP_HAS_SVOC)) | notw);
    out.op_object_ts[ob + no] = ot ? ot[no] : 0;
    out.op_key_off[ob + no] = msg_off + ko;
    out.op_key_len[ob + no] = kl;
    no++;
  }
}

__global__ __launch_bounds__(256) void k_w2_ops(const uint8_t* __restrict__ wire, const uint64_t* __restrict__ moff,
                                                const uint32_t* __restrict__ mlen, uint32_t M, W2Msg s,
                                                const uint8_t* __restrict__ status, const uint4* __restrict__ off4,
                                                uint32_t* __restrict__ g_base, uint32_t* __restrict__ o_base,
                                                uint32_t* __restrict__ m_base, const uint32_t* __restrict__ flags_off,
                                                const uint8_t* __restrict__ flags_in,
                                                const int64_t* __restrict__ ots_in, W2Out out) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m <= M) emit_ops_msg(m, wire, moff, mlen, M, s, status, off4, g_base, o_base, m_base, flags_off, flags_in, ots_in, out);
}

// sig[g] = wire[sig_src[g] .. +256) (zeros when absent): 16 lanes per grant,
// each moving 16 bytes, so a wave reads 4 signatures' contiguous bytes.
__device__ __forceinline__ void emit_sig_piece(uint64_t t, const uint8_t* __restrict__ wire,
                                               const uint64_t* __restrict__ sig_src, uint8_t* __restrict__ sig) {
  const uint32_t g = (uint32_t)(t >> 4), q = (uint32_t)(t & 15);
  const uint64_t src = sig_src[g];
  uint4 v = make_uint4(0, 0, 0, 0);
  if (src != ~0ull) {
    // the lane's 16 bytes from the one or two 16-byte-aligned chunks holding
    // them (each chunk holds a signature byte: page-safe), shifted by a dword
    // rotation (mask selects) and a funnel shift -- two dwordx4 loads instead
    // of eight dword loads
    const uintptr_t a = (uintptr_t)(wire + src) + 16 * q;
    const uint4* c = (const uint4*)(a & ~(uintptr_t)15);
    const uint32_t sh = (uint32_t)(a & 15);
    const uint4 c0 = c[0];
    const uint4 c1 = sh ? c[1] : make_uint4(0, 0, 0, 0);
    const uint32_t d[8] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
    const uint32_t m4 = 0u - ((sh >> 2) & 1u), m8 = 0u - ((sh >> 3) & 1u);
    uint32_t e1[7], e[5];
#pragma unroll
    for (int j = 0; j < 7; j++) e1[j] = (d[j + 1] & m4) | (d[j] & ~m4);
#pragma unroll
    for (int j = 0; j < 5; j++) e[j] = (e1[j + 2] & m8) | (e1[j] & ~m8);
    const uint32_t r = 8 * (sh & 3);
    v = make_uint4(__builtin_amdgcn_alignbit(e[1], e[0], r), __builtin_amdgcn_alignbit(e[2], e[1], r),
                   __builtin_amdgcn_alignbit(e[3], e[2], r), __builtin_amdgcn_alignbit(e[4], e[3], r));
  }
  ((uint4*)(sig + (size_t)g * MOCHI_RSA_BYTES))[q] = v;
}

__global__ __launch_bounds__(256) void k_w2_sig(const uint8_t* __restrict__ wire, const uint64_t* __restrict__ sig_src,
                                                uint32_t N, uint8_t* __restrict__ sig) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if ((t >> 4) < N) emit_sig_piece(t, wire, sig_src, sig);
}

// A small batch (M < kW2SmallM): the three emit kernels above as one block
// (entries, then messages, then -- once every grant's signature source is
// written -- the signatures), two launches fewer after the host has read the
// decoded totals.
__global__ __launch_bounds__(1024) void k_w2_emit_small(const uint8_t* __restrict__ wire,
                                                         const uint64_t* __restrict__ moff,
                                                         const uint32_t* __restrict__ mlen, uint32_t M, W2Msg s, CE ce,
                                                         const uint8_t* __restrict__ status,
                                                         const uint4* __restrict__ off4,
                                                         const uint8_t* __restrict__ ids,
                                                         const uint32_t* __restrict__ id_off, uint32_t n_ids,
                                                         uint32_t* __restrict__ g_base, uint32_t* __restrict__ o_base,
                                                         uint32_t* __restrict__ m_base,
                                                         const uint32_t* __restrict__ flags_off,
                                                         const uint8_t* __restrict__ flags_in,
                                                         const int64_t* __restrict__ ots_in, uint32_t N, W2Out out) {
  const uint32_t total = s.ce_base[M];
#pragma unroll 1
  for (uint32_t e = threadIdx.x; e < total; e += blockDim.x)
    emit_mg_entry(e, wire, moff, mlen, s, ce, status, off4, ids, id_off, n_ids, out);
#pragma unroll 1
  for (uint32_t m = threadIdx.x; m <= M; m += blockDim.x)
    emit_ops_msg(m, wire, moff, mlen, M, s, status, off4, g_base, o_base, m_base, flags_off, flags_in, ots_in, out);
  __syncthreads();  // sig_src written (emit_grant)
#pragma unroll 1
  for (uint64_t t = threadIdx.x; t < (uint64_t)N * 16; t += blockDim.x) emit_sig_piece(t, wire, out.sig_src, out.sig);
}

__global__ __launch_bounds__(256) void k_w2_fixup(const uint8_t* __restrict__ status, uint32_t M,
                                                  uint32_t* __restrict__ accept_bits, uint8_t* __restrict__ reason,
                                                  uint8_t* __restrict__ fail_op, const uint32_t* __restrict__ op_out_off,
                                                  uint8_t* __restrict__ op_decision, uint32_t* __restrict__ op_g0,
                                                  int64_t* __restrict__ op_ts) {
  const uint32_t m = blockIdx.x * blockDim.x + threadIdx.x;
  const bool bad = m < M && status[m] != MOCHI_MSG_OK;
  const uint64_t badmask = __ballot(bad);
  if (m < M && bad) {
    if (reason) reason[m] = status[m] == MOCHI_MSG_MALFORMED ? MOCHI_REJECT_MALFORMED : MOCHI_UNDECIDED;
    if (fail_op) fail_op[m] = 0xFF;
    if (op_out_off)  // ops of an undecoded message: not reached
      for (uint32_t o = op_out_off[m]; o < op_out_off[m + 1]; o++) {
        if (op_decision) op_decision[o] = MOCHI_OPD_SKIPPED;
        if (op_g0) op_g0[o] = 0xFFFFFFFFu;
        if (op_ts) op_ts[o] = 0;
      }
  }
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wbase = (m - lane) >> 5, nwords = (M + 31) >> 5;
  if (lane == 0 && badmask) {
    if (wbase < nwords) accept_bits[wbase] &= ~(uint32_t)badmask;
    if (wbase + 1 < nwords) accept_bits[wbase + 1] &= ~(uint32_t)(badmask >> 32);
  }
}

inline uint32_t cdiv(uint64_t a, uint32_t b) { return (uint32_t)((a + b - 1) / b); }

W2Msg msg_view(const W2Args& a) {
  const size_t m1 = (size_t)a.M + 1;
  uint32_t* p = a.cnt_ce;
  return W2Msg{p, p + m1, p + 2 * m1, p + 3 * m1, p + 4 * m1, p + 5 * m1, p + 6 * m1, a.cnt_o, a.inl, a.inl_ops};
}

// grid of the grid-stride certificate-entry kernels (the entry total is on the device)
inline uint32_t ce_blocks(const W2Args& a) {
  const uint32_t b = cdiv((uint64_t)a.ce_cap, 256);
  return b < 1 ? 1 : b > 2048 ? 2048 : b;
}

}  // namespace

struct Sum4 {
  __host__ __device__ uint4 operator()(const uint4& a, const uint4& b) const {
    return make_uint4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
  }
};

hipError_t w2_scan_temp_bytes(uint32_t n, size_t* bytes) {
  size_t b1 = 0, b4 = 0;
  hipError_t e = hipcub::DeviceScan::ExclusiveSum(nullptr, b1, (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)n);
  if (e != hipSuccess) return e;
  e = hipcub::DeviceScan::ExclusiveScan(nullptr, b4, (const uint4*)nullptr, (uint4*)nullptr, Sum4{},
                                        make_uint4(0, 0, 0, 0), (int)n);
  *bytes = b1 > b4 ? b1 : b4;
  return e;
}

// MOCHI_W2_NO_SMALL_SCAN=1 (A/B): small batches take the large-batch decode
// launches too (hipcub scans, three emit kernels)
static bool small_scan_off() {
  static const bool off = [] {
    const char* e = getenv("MOCHI_W2_NO_SMALL_SCAN");
    return e && e[0] == '1';
  }();
  return off;
}

bool w2_small(uint32_t M) { return M < kW2SmallM && !small_scan_off(); }

hipError_t launch_w2_count(const W2Args& a, hipStream_t st) {
  const W2Msg s = msg_view(a);
  const CE ce = ce_view(a.ce, a.ce_cap);
  const uint32_t gm1 = cdiv((uint64_t)a.M + 1, 256);
  hipLaunchKernelGGL(k_w2_msg, dim3(gm1), dim3(256), 0, st, a.wire, a.msg_off, a.msg_len, a.M, s);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (w2_small(a.M)) {  // the scans inside single-block kernels
    hipLaunchKernelGGL(k_w2_entries<true>, dim3(1), dim3(1024), 0, st, a.wire, a.msg_off, a.msg_len, a.M, s, ce);
    if (a.M)
      hipLaunchKernelGGL(k_w2_mg, dim3(ce_blocks(a)), dim3(256), 0, st, a.wire, a.msg_off, a.msg_len, a.M, s, ce, a.ids,
                         a.id_off, a.n_ids);
    hipLaunchKernelGGL(k_w2_final<true>, dim3(1), dim3(1024), 0, st, a.M, a.flags_off, s, ce, a.cnt_g, a.cnt_m,
                       a.status, (uint4*)a.cnt4, (uint4*)a.off4);
    return hipGetLastError();
  }
  size_t tb = a.scan_temp_bytes;
  e = hipcub::DeviceScan::ExclusiveSum(a.scan_temp, tb, s.cnt_ce, s.ce_base, (int)(a.M + 1), st);
  if (e != hipSuccess) return e;
  if (a.M) {
    hipLaunchKernelGGL(k_w2_entries<false>, dim3(cdiv(a.M, 256)), dim3(256), 0, st, a.wire, a.msg_off, a.msg_len, a.M,
                       s, ce);
    hipLaunchKernelGGL(k_w2_mg, dim3(ce_blocks(a)), dim3(256), 0, st, a.wire, a.msg_off, a.msg_len, a.M, s, ce, a.ids,
                       a.id_off, a.n_ids);
  }
  hipLaunchKernelGGL(k_w2_final<false>, dim3(gm1), dim3(256), 0, st, a.M, a.flags_off, s, ce, a.cnt_g, a.cnt_m,
                     a.status, (uint4*)a.cnt4, (uint4*)a.off4);
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  // one scan of the packed (grants, ops, MultiGrants) counts instead of three
  tb = a.scan_temp_bytes;
  return hipcub::DeviceScan::ExclusiveScan(a.scan_temp, tb, (const uint4*)a.cnt4, (uint4*)a.off4, Sum4{},
                                           make_uint4(0, 0, 0, 0), (int)(a.M + 1), st);
}

hipError_t launch_w2_emit(const W2Args& a, hipStream_t st) {
  W2Out o{a.sig_src, a.grant_off, a.grant_len, a.sig, a.signer, a.grant_key, a.op_key, a.op_flags,
          a.op_object_ts, a.op_key_off, a.op_key_len, a.mg_grant_off, a.grant_same};
  const W2Msg s = msg_view(a);
  const CE ce = ce_view(a.ce, a.ce_cap);
  if (w2_small(a.M)) {
    hipLaunchKernelGGL(k_w2_emit_small, dim3(1), dim3(1024), 0, st, a.wire, a.msg_off, a.msg_len, a.M, s, ce, a.status,
                       (const uint4*)a.off4, a.ids, a.id_off, a.n_ids, a.cert_grant_off, a.cert_op_off, a.cert_mg_off,
                       a.flags_off, a.flags_in, a.ots_in, a.N, o);
    return hipGetLastError();
  }
  if (a.M)
    hipLaunchKernelGGL(k_w2_emit_mg, dim3(ce_blocks(a)), dim3(256), 0, st, a.wire, a.msg_off, a.msg_len, a.M, s, ce,
                       a.status, (const uint4*)a.off4, a.ids, a.id_off, a.n_ids, o);
  hipLaunchKernelGGL(k_w2_ops, dim3(cdiv((uint64_t)a.M + 1, 256)), dim3(256), 0, st, a.wire, a.msg_off, a.msg_len,
                     a.M, s, a.status, (const uint4*)a.off4, a.cert_grant_off, a.cert_op_off, a.cert_mg_off,
                     a.flags_off, a.flags_in, a.ots_in, o);
  if (a.N) hipLaunchKernelGGL(k_w2_sig, dim3(cdiv((uint64_t)a.N * 16, 256)), dim3(256), 0, st, a.wire, a.sig_src, a.N, a.sig);
  return hipGetLastError();
}

hipError_t launch_w2_fixup(const W2Args& a, uint32_t* accept_bits, uint8_t* reason, uint8_t* fail_op,
                           uint8_t* op_decision, uint32_t* op_g0, int64_t* op_ts, hipStream_t st) {
  if (a.M)
    hipLaunchKernelGGL(k_w2_fixup, dim3(cdiv(a.M, 256)), dim3(256), 0, st, a.status, a.M, accept_bits, reason,
                       fail_op, a.flags_off, op_decision, op_g0, op_ts);
  return hipGetLastError();
}

}  // namespace mochi

#if MOCHI_W2_STAMPS
extern "C" int mochi_debug_w2_stamps(unsigned long long* out, unsigned n_waves) {
  if (n_waves > 16384) n_waves = 16384;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(mochi::g_w2_stamps), 64 * (size_t)n_waves, 0, hipMemcpyDeviceToHost) ==
                 hipSuccess
             ? 0
             : -1;
}
#endif
