// w2_host.h — full host decode of one Write2ToServer message (w2_host.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace mochi_host {

struct GrantOut {
  std::string bytes;  // Grant.toByteArray() of the parsed (merged) Grant: the signed bytes
  uint8_t sig[256];   // grantSignatures[map key] when exactly 256 bytes, else zeros
  uint8_t slot;       // key slot of the first op naming the map key, 0xFF none
};

struct MultiGrant {
  uint16_t signer;  // key index of MultiGrant.serverId, 0xFFFF unknown
  std::vector<GrantOut> grants;  // LinkedHashMap order
};

struct Op {
  std::string key_bytes;  // Operation.operand1
  uint8_t slot = 0;       // index of the first op with the same operand1
  bool not_write = false; // MOCHI_OP_NOT_WRITE
};

struct Message {
  std::vector<MultiGrant> mgs;  // WriteCertificate.grants values, LinkedHashMap order
  std::vector<Op> ops;
};

// MOCHI_MSG_OK (decoded), MOCHI_MSG_FALLBACK (more than MOCHI_MAX_OPS_PER_CERT
// operations: not expressible as one-byte op slots) or MOCHI_MSG_MALFORMED.
int decode_full(const uint8_t* m, size_t len, const std::vector<std::string>& server_ids, Message& out);

}  // namespace mochi_host
