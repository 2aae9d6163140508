// config.cpp — the reference's cluster properties file, read the way
// ClusterConfiguration.loadInitialConfigurationFromProperties does
// (ClusterConfiguration.java:138-187), so a server's verifier context gets R,
// the majority M and the replica server-id table from the same file the
// reference boots from (config/sample_config, -DclusterConfig).
//
// Host only.  java.util.Properties.load text rules: logical lines joined on an
// odd run of trailing backslashes, '#' / '!' comment lines, key ended by the
// first unescaped '=', ':' or blank, \t \n \r \f \uXXXX escapes, last
// duplicate wins; the file is ISO-8859-1 and ids reach the wire as UTF-8
// (Utf16ToUtf8 below).  StringUtils.split(s, ',') drops empty fields and trims
// nothing; Integer.parseInt accepts an optional sign and decimal digits only.
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/mochi_hip.h"

namespace mochi {
int set_error(int code, const std::string& msg);  // capi.cpp
}

struct mochi_config {
  std::vector<std::string> ids, urls;  // _CONFIG_SERVERS order
  std::map<long long, uint32_t> token_to_server;  // token VALUE -> server index (tokensToServers)
  uint32_t replication = 0;
};

namespace {

constexpr long long kShardTokens = 1024;                          // ClusterConfiguration.java:25
constexpr long long kTokenRange = 0xffffffffLL / kShardTokens;    // SHARD_TOKEN_VALUE_RANGE (:26)

int cfail(const std::string& msg) { return mochi::set_error(MOCHI_EINVAL, msg); }

void put_utf8(std::string& s, uint32_t cp) {
  if (cp < 0x80) s += (char)cp;
  else if (cp < 0x800) s += (char)(0xC0 | cp >> 6), s += (char)(0x80 | (cp & 0x3F));
  else if (cp < 0x10000)
    s += (char)(0xE0 | cp >> 12), s += (char)(0x80 | ((cp >> 6) & 0x3F)), s += (char)(0x80 | (cp & 0x3F));
  else
    s += (char)(0xF0 | cp >> 18), s += (char)(0x80 | ((cp >> 12) & 0x3F)), s += (char)(0x80 | ((cp >> 6) & 0x3F)),
        s += (char)(0x80 | (cp & 0x3F));
}

// The Java String a Properties value becomes, as the UTF-8 bytes protobuf-java
// puts on the wire for it (CodedOutputStream.writeString): Properties.load(
// InputStream) reads the file as ISO-8859-1, so every raw byte is one UTF-16
// code unit (>= 0x80: a 2-byte UTF-8 sequence), a \uXXXX escape is one code
// unit, a high + low surrogate pair is one supplementary code point, and an
// unpaired surrogate becomes '?' (String.getBytes(UTF_8), protobuf's fallback
// for strings Utf8.encode refuses).
struct Utf16ToUtf8 {
  std::string& o;
  uint32_t hi = 0;  // pending high surrogate
  void unit(uint32_t u) {
    if (hi) {
      if (u >= 0xDC00 && u <= 0xDFFF) {
        put_utf8(o, 0x10000 + ((hi - 0xD800) << 10) + (u - 0xDC00));
        hi = 0;
        return;
      }
      o += '?';
      hi = 0;
    }
    if (u >= 0xD800 && u <= 0xDBFF) hi = u;
    else if (u >= 0xDC00 && u <= 0xDFFF) o += '?';
    else put_utf8(o, u);
  }
  void end() {
    if (hi) o += '?';
    hi = 0;
  }
};

bool is_blank(char c) { return c == ' ' || c == '\t' || c == '\f'; }

// java.util.Properties.load (text form): the key -> value table.
bool parse_properties(const char* text, size_t len, std::map<std::string, std::string>& out, std::string& err) {
  size_t i = 0;
  while (i < len) {
    // one logical line
    std::string line;
    bool first = true;
    for (;;) {
      size_t j = i;
      if (!first)
        while (j < len && is_blank(text[j])) j++;  // continuation lines drop their leading blanks
      size_t e = j;
      while (e < len && text[e] != '\n' && text[e] != '\r') e++;
      std::string phys(text + j, e - j);
      i = e;
      if (i < len && text[i] == '\r') i++;
      if (i < len && text[i] == '\n') i++;
      if (first) {
        size_t k = 0;
        while (k < phys.size() && is_blank(phys[k])) k++;
        if (k == phys.size() || phys[k] == '#' || phys[k] == '!') {
          line.clear();
          break;  // blank or comment line (never continued)
        }
        phys = phys.substr(k);
      }
      size_t bs = 0;
      while (bs < phys.size() && phys[phys.size() - 1 - bs] == '\\') bs++;
      if (bs % 2 == 1 && i <= len) {
        line += phys.substr(0, phys.size() - 1);
        first = false;
        if (i >= len) break;
        continue;
      }
      line += phys;
      break;
    }
    if (line.empty()) continue;
    // key: up to the first unescaped '=', ':' or blank
    std::string key, val;
    size_t k = 0;
    bool esc = false;
    for (; k < line.size(); k++) {
      const char c = line[k];
      if (esc) {
        esc = false;
        continue;
      }
      if (c == '\\') esc = true;
      else if (c == '=' || c == ':' || is_blank(c)) break;
    }
    std::string raw_key = line.substr(0, k);
    while (k < line.size() && is_blank(line[k])) k++;
    if (k < line.size() && (line[k] == '=' || line[k] == ':')) k++;
    while (k < line.size() && is_blank(line[k])) k++;
    std::string raw_val = line.substr(k);
    for (int part = 0; part < 2; part++) {
      const std::string& in = part ? raw_val : raw_key;
      Utf16ToUtf8 o{part ? val : key};
      for (size_t x = 0; x < in.size(); x++) {
        if (in[x] != '\\' || x + 1 >= in.size()) {
          o.unit((uint8_t)in[x]);  // ISO-8859-1: byte = code unit
          continue;
        }
        const char c = in[++x];
        if (c == 't') o.unit('\t');
        else if (c == 'n') o.unit('\n');
        else if (c == 'r') o.unit('\r');
        else if (c == 'f') o.unit('\f');
        else if (c == 'u') {
          if (x + 4 >= in.size()) {
            err = "malformed \\uxxxx encoding";
            return false;
          }
          uint32_t cp = 0;
          for (int h = 1; h <= 4; h++) {
            const char d = in[x + h];
            cp <<= 4;
            if (d >= '0' && d <= '9') cp |= d - '0';
            else if (d >= 'a' && d <= 'f') cp |= d - 'a' + 10;
            else if (d >= 'A' && d <= 'F') cp |= d - 'A' + 10;
            else {
              err = "malformed \\uxxxx encoding";
              return false;
            }
          }
          x += 4;
          o.unit(cp);
        } else o.unit((uint8_t)c);
      }
      o.end();
    }
    out[key] = val;
  }
  return true;
}

// StringUtils.split(s, ','): non-empty fields only, nothing trimmed
std::vector<std::string> split_commas(const std::string& s) {
  std::vector<std::string> v;
  size_t a = 0;
  while (a <= s.size()) {
    size_t b = s.find(',', a);
    if (b == std::string::npos) b = s.size();
    if (b > a) v.push_back(s.substr(a, b - a));
    a = b + 1;
  }
  return v;
}

// Integer.parseInt: optional sign, decimal digits, int32 range
bool parse_int(const std::string& s, long long& v) {
  if (s.empty()) return false;
  size_t i = 0;
  bool neg = false;
  if (s[0] == '-' || s[0] == '+') {
    neg = s[0] == '-';
    i = 1;
    if (s.size() == 1) return false;
  }
  long long x = 0;
  for (; i < s.size(); i++) {
    if (s[i] < '0' || s[i] > '9') return false;
    x = x * 10 + (s[i] - '0');
    if (x > 2147483648LL) return false;
  }
  if (neg) x = -x;
  if (x > 2147483647LL || x < -2147483648LL) return false;
  v = x;
  return true;
}

mochi_config* build(const std::map<std::string, std::string>& props) {
  auto get = [&](const std::string& k, const std::string* def) -> const std::string* {
    auto it = props.find(k);
    return it == props.end() ? def : &it->second;
  };
  const std::string empty;
  mochi_config* c = new mochi_config;
  std::map<std::string, uint32_t> seen;  // servers.put(serverId, ...): a repeated id is one server
  for (const std::string& id : split_commas(*get("_CONFIG_SERVERS", &empty))) {
    const std::string* url = get("_CONFIG_SERVER_" + id + "_URL", nullptr);
    if (!url) {
      cfail("Missing server url for id " + id);
      delete c;
      return nullptr;
    }
    uint32_t idx;
    auto it = seen.find(id);
    if (it == seen.end()) {
      idx = (uint32_t)c->ids.size();
      seen[id] = idx;
      c->ids.push_back(id);
      c->urls.push_back(*url);
    } else {
      idx = it->second;
      c->urls[idx] = *url;
    }
    for (const std::string& t : split_commas(*get("_CONFIG_SERVER_" + id + "_TOKENS", &empty))) {
      long long n;
      if (!parse_int(t, n)) {
        cfail("For input string: \"" + t + "\" (token of " + id + ")");
        delete c;
        return nullptr;
      }
      if (n >= kShardTokens) {
        cfail("Too large shard number");
        delete c;
        return nullptr;
      }
      const long long token = n * kTokenRange;  // tokenNumberToTokenValue
      if (c->token_to_server.count(token)) {
        cfail("Mutple mapping for token: " + std::to_string(token) + " (number " + std::to_string(n) + ")");
        delete c;
        return nullptr;
      }
      c->token_to_server[token] = idx;
    }
  }
  for (long long i = 0; i < kShardTokens; i++)
    if (!c->token_to_server.count(i * kTokenRange)) {
      cfail("Token " + std::to_string(i * kTokenRange) + " (index " + std::to_string(i) + ") is not assigned");
      delete c;
      return nullptr;
    }
  const std::string* bft = get("_CONFIG_BFT_REPLICATION", nullptr);
  long long r;
  if (!bft) {
    cfail("BFT replication factor is non defined");
    delete c;
    return nullptr;
  }
  if (!parse_int(*bft, r)) {
    cfail("For input string: \"" + *bft + "\" (_CONFIG_BFT_REPLICATION)");
    delete c;
    return nullptr;
  }
  if (r < 4) {  // ClusterConfiguration.java:182
    cfail("BFT replication factor should be > 4");
    delete c;
    return nullptr;
  }
  if (r > (long long)c->token_to_server.size()) {  // :183, tokensToServers.values().size()
    cfail("BFT replication factor should be less or equal than number of servers");
    delete c;
    return nullptr;
  }
  c->replication = (uint32_t)r;
  return c;
}

}  // namespace

extern "C" {

mochi_config* mochi_config_parse(const char* text, uint64_t len) {
  if (!text && len) {
    cfail("null text");
    return nullptr;
  }
  std::map<std::string, std::string> props;
  std::string err;
  if (!parse_properties(text ? text : "", (size_t)len, props, err)) {
    cfail(err);
    return nullptr;
  }
  return build(props);
}

mochi_config* mochi_config_load(const char* path) {
  if (!path) {
    cfail("null path");
    return nullptr;
  }
  FILE* f = fopen(path, "rb");
  if (!f) {
    cfail(std::string("cannot open ") + path + ": " + strerror(errno));
    return nullptr;
  }
  std::string text;
  char buf[65536];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) text.append(buf, n);
  fclose(f);
  return mochi_config_parse(text.data(), text.size());
}

void mochi_config_free(mochi_config* c) { delete c; }

uint32_t mochi_config_replication(const mochi_config* c) { return c ? c->replication : 0; }

uint32_t mochi_config_majority(const mochi_config* c) { return c ? 2 * (c->replication / 3) + 1 : 0; }

uint32_t mochi_config_n_servers(const mochi_config* c) { return c ? (uint32_t)c->ids.size() : 0; }

const char* mochi_config_server_id(const mochi_config* c, uint32_t i) {
  return c && i < c->ids.size() ? c->ids[i].c_str() : nullptr;
}

const char* mochi_config_server_url(const mochi_config* c, uint32_t i) {
  return c && i < c->urls.size() ? c->urls[i].c_str() : nullptr;
}

int mochi_config_servers_for_key(const mochi_config* c, const uint8_t* key, uint32_t key_len, uint32_t* idx_out) {
  if (!c || !idx_out || (!key && key_len)) return cfail("null argument");
  // getServersForObjectHashCode (:207-226): the loop takes token i (:215), not
  // (tokenValStart + i) % SHARD_TOKENS, so the key's hash never matters
  std::vector<uint32_t> got;
  for (uint32_t i = 0; i < c->replication; i++) {
    auto it = c->token_to_server.find((long long)i * kTokenRange);
    if (it == c->token_to_server.end()) return cfail("Failed to find server for token " + std::to_string(i));
    for (uint32_t g : got)
      if (g == it->second)
        return cfail("BFT requires all servers to be unique. Found collision for server " + c->ids[g]);
    got.push_back(it->second);
    idx_out[i] = it->second;
  }
  return MOCHI_OK;
}

int64_t mochi_config_replica_ids(const mochi_config* c, const uint8_t* key, uint32_t key_len, uint8_t* ids_out,
                                 uint64_t ids_cap, uint32_t* id_off) {
  if (!c || !id_off) return cfail("null argument");
  std::vector<uint32_t> idx(c->replication);
  const int rc = mochi_config_servers_for_key(c, key, key_len, idx.data());
  if (rc) return rc;
  uint64_t pos = 0;
  id_off[0] = 0;
  for (uint32_t i = 0; i < c->replication; i++) {
    const std::string& s = c->ids[idx[i]];
    if (ids_out && pos + s.size() <= ids_cap) memcpy(ids_out + pos, s.data(), s.size());
    pos += s.size();
    id_off[i + 1] = (uint32_t)pos;
  }
  return (int64_t)pos;
}

}  // extern "C"
