// w2_host.cpp — the host side of the Write2ToServer wire path: a complete
// protobuf-java 3.16.3 decode of the messages the device decoder's fast path
// declines (MOCHI_MSG_FALLBACK), so that every certificate -- however it is
// encoded -- still has its signatures checked on the device.
//
// What the device leaves here (w2_decode.hip): writeCertificate / transaction
// given more than once, a map entry carrying its value more than once, Grant
// bytes that are not the canonical encoding, more than 32 MultiGrants or 64
// grants in one MultiGrant.  The semantics restated (MochiProtocol.java's
// generated parsers on protobuf-java 3.16.3):
//   * a singular message field given n times is the merge of the n values,
//     which is the parse of their concatenation (Write2ToServer.writeCertificate
//     / .transaction; a map entry's MultiGrant or Grant value given twice,
//     MapEntryLite.parseField merges message values);
//   * map fields put each entry into a LinkedHashMap: a repeated key keeps its
//     first position and takes the LAST entry's value (replaced, not merged);
//     a bytes value (grantSignatures) given twice in one entry: the last wins;
//   * scalars / strings: last value wins; Operation.action is read as an int32
//     (readEnum), an unknown enum value stays as is;
//   * the signed bytes of a grant are Grant.toByteArray() of the parsed Grant
//     (MochiProtocol.java:7556-7574): known fields 1..5 at non-default values,
//     then the unknown fields the parser retained (proto3 keeps them,
//     parseUnknownFieldProto3), re-serialized as UnknownFieldSet does: by field
//     number, and per number varints, fixed32s, fixed64s, length-delimited
//     values, groups, each in arrival order.
// The message is already known to be parseable (k_w2_valid); any surprise here
// is reported as MALFORMED all the same.
#include <cstdint>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/mochi_hip.h"
#include "w2_host.h"

namespace mochi_host {
namespace {

constexpr int kRecursionLimit = 100;  // CodedInputStream.DEFAULT_RECURSION_LIMIT

struct Span {
  const uint8_t* p;
  size_t n;
};

// One CodedInputStream-style cursor over a byte range.
struct Cursor {
  const uint8_t* p;
  size_t n, i = 0;
  Cursor(const uint8_t* p_, size_t n_) : p(p_), n(n_) {}
  bool done() const { return i >= n; }
  bool varint(uint64_t& v) {
    uint64_t x = 0;
    for (int k = 0; k < 10; k++) {
      if (i >= n) return false;
      const uint8_t c = p[i++];
      x |= (uint64_t)(c & 0x7F) << (7 * k);
      if (!(c & 0x80)) {
        v = x;
        return true;
      }
    }
    return false;
  }
  bool ld(Span& s) {  // length-delimited payload (readRawVarint32 length, >= 0)
    uint64_t l;
    if (!varint(l)) return false;
    const int32_t l32 = (int32_t)(uint32_t)l;
    if (l32 < 0 || (size_t)l32 > n - i) return false;
    s = {p + i, (size_t)l32};
    i += (size_t)l32;
    return true;
  }
  bool fixed(size_t k, uint64_t& v) {
    if (n - i < k) return false;
    v = 0;
    for (size_t b = 0; b < k; b++) v |= (uint64_t)p[i + b] << (8 * b);
    i += k;
    return true;
  }
};

// UnknownFieldSet (TreeMap by field number).
struct Unknown;
struct UField {
  std::vector<uint64_t> varint, f64;
  std::vector<uint32_t> f32;
  std::vector<std::string> ld;
  std::vector<std::unique_ptr<Unknown>> group;
};
struct Unknown {
  std::map<uint32_t, UField> f;
};

bool read_unknown(Cursor& c, uint32_t field, uint32_t wt, Unknown& u, int depth);

// Reads a group body (after its START_GROUP tag) into `u` up to the matching END_GROUP.
bool read_group(Cursor& c, uint32_t field, Unknown& u, int depth) {
  if (depth >= kRecursionLimit) return false;
  for (;;) {
    uint64_t t;
    if (!c.varint(t)) return false;
    const uint32_t tag = (uint32_t)t, fn = tag >> 3, wt = tag & 7;
    if (fn == 0) return false;
    if (wt == 4) return fn == field;
    if (!read_unknown(c, fn, wt, u, depth + 1)) return false;
  }
}

bool read_unknown(Cursor& c, uint32_t field, uint32_t wt, Unknown& u, int depth) {
  UField& f = u.f[field];
  uint64_t v;
  Span s;
  switch (wt) {
    case 0:
      if (!c.varint(v)) return false;
      f.varint.push_back(v);
      return true;
    case 1:
      if (!c.fixed(8, v)) return false;
      f.f64.push_back(v);
      return true;
    case 2:
      if (!c.ld(s)) return false;
      f.ld.emplace_back((const char*)s.p, s.n);
      return true;
    case 3: {
      f.group.emplace_back(new Unknown);
      return read_group(c, field, *f.group.back(), depth);
    }
    case 5:
      if (!c.fixed(4, v)) return false;
      f.f32.push_back((uint32_t)v);
      return true;
    default:
      return false;
  }
}

void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
void put_tag(std::string& o, uint32_t field, uint32_t wt) { put_varint(o, ((uint64_t)field << 3) | wt); }

void write_unknown(std::string& o, const Unknown& u) {
  for (const auto& kv : u.f) {
    const uint32_t fn = kv.first;
    const UField& f = kv.second;
    for (uint64_t v : f.varint) {
      put_tag(o, fn, 0);
      put_varint(o, v);
    }
    for (uint32_t v : f.f32) {
      put_tag(o, fn, 5);
      for (int b = 0; b < 4; b++) o.push_back((char)(v >> (8 * b)));
    }
    for (uint64_t v : f.f64) {
      put_tag(o, fn, 1);
      for (int b = 0; b < 8; b++) o.push_back((char)(v >> (8 * b)));
    }
    for (const std::string& s : f.ld) {
      put_tag(o, fn, 2);
      put_varint(o, s.size());
      o += s;
    }
    for (const auto& g : f.group) {
      put_tag(o, fn, 3);
      write_unknown(o, *g);
      put_tag(o, fn, 4);
    }
  }
}

// Iterate the top-level fields of a byte range; unknown groups are skipped
// (and bounded by the recursion limit).  fn(field, wt, varint, span) -> bool.
template <typename F>
bool for_fields(Span s, F&& fn, int depth = 0) {
  Cursor c(s.p, s.n);
  while (!c.done()) {
    uint64_t t;
    if (!c.varint(t)) return false;
    const uint32_t tag = (uint32_t)t, field = tag >> 3, wt = tag & 7;
    if (field == 0) return false;
    uint64_t v = 0;
    Span p{nullptr, 0};
    switch (wt) {
      case 0:
        if (!c.varint(v)) return false;
        break;
      case 1:
        if (!c.fixed(8, v)) return false;
        break;
      case 2:
        if (!c.ld(p)) return false;
        break;
      case 3: {
        Unknown scratch;
        if (!read_group(c, field, scratch, depth + 1)) return false;
        break;
      }
      case 5:
        if (!c.fixed(4, v)) return false;
        break;
      default:
        return false;
    }
    if (!fn(field, wt, v, p)) return false;
  }
  return true;
}

// Grant (MochiProtocol.java:7369-7425), merged over several byte ranges.
struct Grant {
  std::string oid, hash;
  int64_t ts = 0, cfg = 0;
  int32_t status = 0;
  Unknown unk;
};

bool merge_grant(Grant& g, Span s, int depth) {
  Cursor c(s.p, s.n);
  while (!c.done()) {
    uint64_t t;
    if (!c.varint(t)) return false;
    const uint32_t tag = (uint32_t)t, field = tag >> 3, wt = tag & 7;
    if (field == 0) return false;
    Span p;
    uint64_t v;
    switch (tag) {
      case 10:
        if (!c.ld(p)) return false;
        g.oid.assign((const char*)p.p, p.n);
        continue;
      case 16:
        if (!c.varint(v)) return false;
        g.ts = (int64_t)v;
        continue;
      case 24:
        if (!c.varint(v)) return false;
        g.cfg = (int64_t)v;
        continue;
      case 34:
        if (!c.ld(p)) return false;
        g.hash.assign((const char*)p.p, p.n);
        continue;
      case 40:
        if (!c.varint(v)) return false;
        g.status = (int32_t)(uint32_t)v;
        continue;
      default:
        if (wt == 4) return false;
        if (!read_unknown(c, field, wt, g.unk, depth)) return false;
    }
  }
  return true;
}

// Grant.toByteArray() (MochiProtocol.java:7556-7574).
std::string grant_bytes(const Grant& g) {
  std::string o;
  if (!g.oid.empty()) {
    put_tag(o, 1, 2);
    put_varint(o, g.oid.size());
    o += g.oid;
  }
  if (g.ts) {
    put_tag(o, 2, 0);
    put_varint(o, (uint64_t)g.ts);
  }
  if (g.cfg) {
    put_tag(o, 3, 0);
    put_varint(o, (uint64_t)g.cfg);
  }
  if (!g.hash.empty()) {
    put_tag(o, 4, 2);
    put_varint(o, g.hash.size());
    o += g.hash;
  }
  if (g.status) {
    put_tag(o, 5, 0);
    put_varint(o, (uint64_t)(int64_t)g.status);  // writeEnum: int32, sign-extended
  }
  write_unknown(o, g.unk);
  return o;
}

// LinkedHashMap<String, V> with put(): first position, last value.
template <typename V>
struct LinkedMap {
  std::vector<std::pair<std::string, V>> items;
  std::unordered_map<std::string, size_t> at;
  void put(const std::string& k, V v) {
    auto it = at.find(k);
    if (it == at.end()) {
      at.emplace(k, items.size());
      items.emplace_back(k, std::move(v));
    } else {
      items[it->second].second = std::move(v);
    }
  }
};

// One map entry (key = 1, value = 2) of a byte range: key last, value pieces in order.
bool read_entry(Span e, std::string& key, std::vector<Span>& vals) {
  key.clear();
  vals.clear();
  return for_fields(e, [&](uint32_t f, uint32_t wt, uint64_t, Span p) {
    if (wt == 2 && f == 1) key.assign((const char*)p.p, p.n);
    if (wt == 2 && f == 2) vals.push_back(p);
    return true;
  });
}

}  // namespace

int decode_full(const uint8_t* m, size_t len, const std::vector<std::string>& server_ids, Message& out) {
  out = Message();
  // Write2ToServer: all writeCertificate pieces, all transaction pieces (merge = concatenation)
  std::vector<Span> wc, tx;
  if (!for_fields({m, len}, [&](uint32_t f, uint32_t wt, uint64_t, Span p) {
        if (wt == 2 && f == 1) wc.push_back(p);
        if (wt == 2 && f == 2) tx.push_back(p);
        return true;
      }))
    return MOCHI_MSG_MALFORMED;
  // Transaction.operations: every occurrence is one Operation
  std::vector<std::string> keys;
  for (Span t : tx) {
    const bool ok = for_fields(t, [&](uint32_t f, uint32_t wt, uint64_t, Span p) {
      if (f != 1 || wt != 2) return true;
      int32_t action = 0;
      std::string k;
      if (!for_fields(p, [&](uint32_t f2, uint32_t wt2, uint64_t v, Span q) {
            if (f2 == 1 && wt2 == 0) action = (int32_t)(uint32_t)v;  // readEnum
            if (f2 == 2 && wt2 == 2) k.assign((const char*)q.p, q.n);
            return true;
          }))
        return false;
      Op op;
      op.key_bytes = k;
      op.not_write = (action != 1 && action != 2) || k.empty();  // WRITE = 2, DELETE = 1
      out.ops.push_back(std::move(op));
      keys.push_back(std::move(k));
      return true;
    });
    if (!ok) return MOCHI_MSG_MALFORMED;
  }
  for (size_t j = 0; j < out.ops.size(); j++) {
    uint8_t slot = (uint8_t)(j < 255 ? j : 255);
    for (size_t q = 0; q < j; q++)
      if (keys[q] == keys[j]) {
        slot = out.ops[q].slot;
        break;
      }
    out.ops[j].slot = slot;
  }
  // WriteCertificate.grants: serverId-keyed LinkedHashMap of MultiGrant value pieces
  LinkedMap<std::vector<Span>> certs;
  std::string key;
  std::vector<Span> vals;
  for (Span w : wc) {
    const bool ok = for_fields(w, [&](uint32_t f, uint32_t wt, uint64_t, Span p) {
      if (f != 1 || wt != 2) return true;
      if (!read_entry(p, key, vals)) return false;
      certs.put(key, vals);
      return true;
    });
    if (!ok) return MOCHI_MSG_MALFORMED;
  }
  for (auto& ce : certs.items) {
    MultiGrant mg;
    std::string sid;
    LinkedMap<std::vector<Span>> grants;
    LinkedMap<Span> sigs;
    for (Span piece : ce.second) {
      const bool ok = for_fields(piece, [&](uint32_t f, uint32_t wt, uint64_t, Span p) {
        if (wt != 2) return true;
        if (f == 4) sid.assign((const char*)p.p, p.n);
        if (f == 1) {
          if (!read_entry(p, key, vals)) return false;
          grants.put(key, vals);
        }
        if (f == 5) {
          if (!read_entry(p, key, vals)) return false;
          sigs.put(key, vals.empty() ? Span{nullptr, 0} : vals.back());  // bytes value: last wins
        }
        return true;
      });
      if (!ok) return MOCHI_MSG_MALFORMED;
    }
    mg.signer = 0xFFFF;
    for (size_t k = 0; k < server_ids.size(); k++)
      if (server_ids[k] == sid) {
        mg.signer = (uint16_t)k;
        break;
      }
    for (auto& ge : grants.items) {
      Grant g;
      for (Span piece : ge.second)
        if (!merge_grant(g, piece, 0)) return MOCHI_MSG_MALFORMED;
      GrantOut go;
      go.bytes = grant_bytes(g);
      auto si = sigs.at.find(ge.first);
      if (si != sigs.at.end() && sigs.items[si->second].second.n == MOCHI_RSA_BYTES)
        memcpy(go.sig, sigs.items[si->second].second.p, MOCHI_RSA_BYTES);
      else
        memset(go.sig, 0, MOCHI_RSA_BYTES);
      go.slot = 0xFF;
      for (size_t j = 0; j < keys.size(); j++)
        if (keys[j] == ge.first) {
          go.slot = out.ops[j].slot;
          break;
        }
      mg.grants.push_back(std::move(go));
    }
    out.mgs.push_back(std::move(mg));
  }
  if (out.ops.size() > MOCHI_MAX_OPS_PER_CERT) return MOCHI_MSG_FALLBACK;  // op slots are one byte (< 64)
  return MOCHI_MSG_OK;
}

}  // namespace mochi_host
