// w2.h — launch interface between the C-ABI layer (capi.cpp) and the
// Write2ToServer wire decoder (w2_decode.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace mochi {

// Write2ToServer wire decode (w2_decode.hip).  Device pointers.
struct W2Args {
  // input messages
  const uint8_t* wire;
  const uint64_t* msg_off;
  const uint32_t* msg_len;
  uint32_t M;
  const uint32_t* flags_off;  // [M+1] or null
  const uint8_t* flags_in;
  const int64_t* ots_in;      // aligned with flags_in, or null
  const uint8_t* ids;         // server-id table
  const uint32_t* id_off;
  uint32_t n_ids;
  // scratch / outputs
  uint32_t* cnt_g;  // [M+1]
  uint32_t* cnt_o;  // [M+1]
  uint32_t* cnt_m;  // [M+1] MultiGrants
  // level-by-level decode: cnt_ce, ce_base, st_bits, wc_off, wc_len, tx_off,
  // tx_len ([M+1] each, contiguous from cnt_ce) and the certificate-entry list
  // (kW2CeArrays arrays of ce_cap words)
  uint32_t* cnt_ce;
  uint32_t* ce;
  uint32_t ce_cap;
  uint32_t* inl;  // [M+1][kW2InlEntries][4], 16-byte aligned: level 1's first entries (key / value slices)
  uint32_t* inl_ops;  // [M+1][kW2InlOps][2]: level 1's first operations' operand1 slices (key slot lookup)
  uint32_t* cnt4;  // [M+1][4], 16-byte aligned: decoded grants, ops, MultiGrants per message (one scan)
  uint32_t* off4;  // [M+1][4]: their exclusive scan (unpacked into cert_*_off by k_w2_ops)
  uint8_t* status;  // [M]
  void* scan_temp;
  size_t scan_temp_bytes;
  uint32_t* cert_grant_off;  // [M+1]
  uint32_t* cert_op_off;     // [M+1]
  uint32_t* cert_mg_off;     // [M+1]
  uint32_t N;          // decoded grant total (emit)
  uint64_t* sig_src;   // [N] wire offset of each signature (emit -> k_w2_sig)
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
  uint32_t* mg_grant_off;    // [n_mgs+1]
  uint32_t* grant_same;      // [N] or null: an earlier grant of the message with the same bytes (k_w2_mg's match)
};
// Device words of one decode's per-batch scratch: 13 arrays of M+1 (counts,
// CSR offsets, level-1 state) + the certificate-entry list (at most
// kW2MaxCertEntries per message on the fast path, kW2CeArrays words each) +
// level 1's entry records + the packed per-message counts and their scan.
constexpr uint32_t kW2MaxCertEntries = 32;
constexpr int kW2MsgArrays = 13;
constexpr int kW2CeArrays = 11;
// Level 1 records the key / value slices of a message's first kW2InlEntries
// certificate entries, so the compact entry list is copied, not re-parsed.
constexpr uint32_t kW2InlEntries = 4;
// ... and the operand1 (key) slices of its first kW2InlOps operations, so level
// 2's key-slot lookup compares keys instead of re-walking the transaction.
constexpr uint32_t kW2InlOps = 4;
inline size_t w2_scratch_words(uint32_t M) {
  return (size_t)kW2MsgArrays * ((size_t)M + 1) + kW2CeArrays * (size_t)kW2MaxCertEntries * ((size_t)M + 1) +
         4 * (size_t)kW2InlEntries * ((size_t)M + 1) + 2 * (size_t)kW2InlOps * ((size_t)M + 1) + 8 * ((size_t)M + 1) +
         4;  // + 4: 16-byte alignment
}
hipError_t w2_scan_temp_bytes(uint32_t n, size_t* bytes);
// M messages decode without the hipcub scans (single-block kernels; no scan scratch)
bool w2_small(uint32_t M);
hipError_t launch_w2_count(const W2Args& a, hipStream_t stream);  // + exclusive scans
hipError_t launch_w2_emit(const W2Args& a, hipStream_t stream);
hipError_t launch_w2_fixup(const W2Args& a, uint32_t* accept_bits, uint8_t* reason, uint8_t* fail_op,
                           uint8_t* op_decision, uint32_t* op_g0, int64_t* op_ts, hipStream_t stream);

}  // namespace mochi
