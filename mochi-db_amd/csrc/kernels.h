// kernels.h — launch interface between the C-ABI layer (capi.cpp) and the
// HIP kernels (kernels.hip).  All pointers are device pointers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "fold.h"

namespace mochi {

struct KeyEntry;

struct LaunchArgs {
  // batch
  uint32_t n_grants, n_certs, n_keys, n_slots;
  const uint8_t* blob;
  const uint64_t* grant_off;
  const uint32_t* grant_len;
  const uint8_t* sig;
  const uint16_t* signer;
  const uint8_t* grant_key;
  const uint32_t* cert_grant_off;
  const uint32_t* cert_op_off;
  const uint8_t* op_key;
  const uint8_t* op_flags;
  const uint8_t* expected_hash;
  const uint32_t* cert_mg_off;   // [C+1] or null (MultiGrant = signer run)
  const uint32_t* mg_grant_off;  // [n_mgs+1] or null
  const int64_t* op_object_ts;   // [O] or null
  const uint64_t* op_key_off;    // [O] or null (MOCHI_Q_BIND)
  const uint32_t* op_key_len;    // [O] or null
  uint32_t majority, strict_gt, quorum_mode;
  const KeyEntry* keys;
  const FoldKey* fold;  // per-key fold matrices (k_rsa_pow)
  // scratch (context-owned)
  uint32_t* digest;    // [8][n_dist]  distinct results (prep_dev.h PrepArgs)
  int64_t* ts;         // [N]  (may be the caller's grant_ts output)
  uint64_t* hash_off;  // [n_dist]
  uint32_t* hash_len;  // [n_dist]
  uint32_t* lead;      // [N] distinct index per grant (with dedup; null: none)
  uint32_t n_dist;     // stride of the distinct arrays: >= N + C with dedup (0 = N)
  uint8_t* flags;      // [N]  (may be the caller's grant_flags output)
  uint32_t* count;     // [n_keys]
  uint32_t* cursor;    // [n_keys]
  uint32_t* total;     // [kTotalWords]: bucketed slot total, then per-call counters (zeroed by k_bucket_scan)
  uint8_t* rare;       // [N] grant prep: grants not covered by their certificate's first grants (null: no dedup)
  const uint32_t* grant_same;  // [N] or null: the wire decoder's byte-equal earlier grant of the certificate
  uint32_t* perm;      // [n_slots]
  uint32_t* xbuf;      // [kL][n_slots]
  // outputs
  uint32_t* grant_valid_bits;  // may be null
  uint32_t* cert_accept_bits;
  uint8_t* cert_reason;   // may be null
  uint8_t* cert_fail_op;  // may be null
  uint8_t* op_decision;   // [O] may be null
  uint32_t* op_g0;        // [O] may be null
  int64_t* op_ts;         // [O] may be null
  const uint32_t* op_out_off;  // [C+1] per-op output positions; null = cert_op_off
  // wire path: [C] message status (w2_decode.hip); k_tally applies k_w2_fixup's
  // overrides to the undecoded messages (else null)
  const uint8_t* msg_status;
  // mochi_rsa_public_op only: raw s^65537 mod n words [N][64] (else null)
  uint32_t* dbg_y;
  bool skip_prep_tally;
  uint32_t small_grants;  // small-batch launch sequence for N <= this (0: never)
  // grant prep runs on `aux` (forked from / joined back to the launch stream
  // with ev_fork / ev_join) beside k_rsa_pow; null = serial on the launch stream
  hipStream_t aux;
  hipEvent_t ev_fork, ev_join;
  // optional per-stage timing: a (start, end) event pair per stage, recorded on
  // the stream the stage runs on
  hipEvent_t* prof_events;
};

// LaunchArgs::total words
enum TotalWord { kTotSlots = 0, kTotPowGroup, kTotFinalGroup, kTotalWords = 4 };

// Stages timed when LaunchArgs::prof_events is set.
enum ProfStage { kStagePrep = 0, kStageBucket, kStagePow, kStageFinal, kStageTally, kProfStages };

// Slots of the signer-bucketed RSA grid: every bucket is padded to kBucketAlign
// (one k_rsa_pow block of one signer).
inline uint64_t slot_capacity(uint32_t n_grants, uint32_t n_keys) {
  return (uint64_t)n_grants + (uint64_t)kBucketAlign * (n_keys < n_grants ? n_keys : n_grants);
}

hipError_t launch_verify(const LaunchArgs& a, hipStream_t stream);

// Device signer (rsa_sign.hip).
size_t sign_key_bytes();
void sign_key_set(void* dst, const uint32_t* p, const uint32_t* q, const uint32_t* r3p, const uint32_t* r3q,
                  const uint32_t* qinv_r, const uint32_t* dp, const uint32_t* dq, const uint32_t* cpad, uint32_t p0inv,
                  uint32_t q0inv, uint32_t dp_bits, uint32_t dq_bits);
hipError_t launch_rsa_sign(const uint8_t* blob, const uint64_t* goff, const uint32_t* glen, uint32_t n,
                           const void* key, uint8_t* sig, uint32_t fault_idx, hipStream_t stream);
// Zero every signature whose flags lack MOCHI_GRANT_SIG_OK and count them.
hipError_t launch_withhold(const uint8_t* flags, uint32_t n, uint8_t* sig, uint32_t* rejected, hipStream_t stream);
hipError_t launch_pack_bits(const uint8_t* flags, uint32_t n, uint8_t mask, uint32_t* bits, hipStream_t stream);
// latency: the small-batch form (k_rsa_pow_lat: one signature chain spread over three SIMDs)
void launch_rsa_pow(const LaunchArgs& a, hipStream_t stream, bool latency = false);
// latency: a small batch -- k_rsa_final_lat, one 4-wave block per 64-slot chunk
void launch_rsa_final(const LaunchArgs& a, const uint32_t* lead, uint32_t n_dist, hipStream_t stream,
                      bool latency = false);
void launch_rsa_raw(const LaunchArgs& a, hipStream_t stream);  // dbg_y path (mochi_rsa_public_op)

}  // namespace mochi
