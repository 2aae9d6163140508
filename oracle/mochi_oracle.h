/*
 * mochi_oracle.h — CPU oracle for the Write2 certificate-verification path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing under oracle/ is part of the product:
 * only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load liboracle.so, and only as the checker / the timed CPU baseline.
 *
 * Parity pins:
 *   - SHA-256 + RSA-2048 PKCS#1 v1.5 verify: OpenSSL 3.0.2 libcrypto
 *     (EVP_DigestVerify, "SHA256withRSA"), checked against NIST SHA-256 vectors
 *     and OpenSSL-CLI-signed fixtures in tests/golden/.
 *   - Grant proto3 bytes: restated from MochiProtocol.java:7556-7574, checked
 *     against Python google.protobuf 7.35.1 with a hand-built descriptor
 *     (tests/golden/make_golden.py).
 *   - Certificate verdict logic: restated line by line from
 *     InMemoryDataStore.java:576-640 / ClusterConfiguration.java:264-267 /
 *     MochiDBClient.java:148-175,195-219,355-382.  The reference ships no
 *     executable or golden vector for these branches (it cannot run here: no
 *     JVM), so this part is "parity unpinned" against the reference and pinned
 *     only by the hand-constructed branch fixtures in tests/golden/.
 */
#ifndef MOCHI_ORACLE_H
#define MOCHI_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#include "../include/mochi_hip.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Grant.writeTo restated (MochiProtocol.java:7556-7574): proto3, fields in
 * number order, defaults skipped.  Returns the encoded length, or -1 if it
 * does not fit in `cap`. */
long oracle_grant_encode(const char* object_id, size_t object_id_len, int64_t timestamp, int64_t configstamp,
                         const char* txn_hash, size_t txn_hash_len, int32_t status, uint8_t* out, size_t cap);

/* The fields of a parsed Grant.  Offsets are into the parsed buffer. */
typedef struct oracle_grant_view {
  int64_t timestamp;
  int64_t configstamp;
  int32_t status;
  uint32_t object_id_off, object_id_len;
  uint32_t txn_hash_off, txn_hash_len;
} oracle_grant_view;

/* Grant(CodedInputStream) restated (MochiProtocol.java:7369-7425) with
 * protobuf-java 3.16.3 CodedInputStream semantics: last value wins, unknown
 * fields skipped by wire type, strings must be valid UTF-8
 * (readStringRequireUtf8), tag 0 / wire types 6,7 / stray END_GROUP /
 * truncated input are errors.  Unknown groups nest at most 100 deep
 * (CodedInputStream's default recursion limit).  Returns 1 ok, 0 malformed. */
int oracle_grant_parse(const uint8_t* buf, size_t len, oracle_grant_view* out);

/* SHA-256 (OpenSSL). */
void oracle_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);

/* SHA256withRSA verify of `msg` against a 2048-bit modulus (big-endian) with
 * e = 65537 (OpenSSL EVP_DigestVerify).  Returns 1 valid, 0 invalid. */
int oracle_rsa_verify(const uint8_t n_be[256], const uint8_t* msg, size_t len, const uint8_t sig[256]);

/* ClusterConfiguration.getServerMajority restated (ClusterConfiguration.java:264-267). */
uint32_t oracle_server_majority(uint32_t replication_factor);

/* Full batch verdict: per-grant signature + parse, then per-certificate
 * processMultiGrantsFromAllServers + write2apply verdict.  Host memory.
 * Signature checks are spread over `n_threads` pthreads (the CPU baseline);
 * the tally runs on the calling thread.  Same in/out contract as
 * mochi_verify_batch (include/mochi_hip.h).  Returns 0 or MOCHI_EINVAL. */
int oracle_verify_batch(const uint8_t* moduli_be, uint32_t n_keys, const mochi_batch* batch,
                        const mochi_params* params, mochi_verdicts* out, int n_threads);

/* Only the signature leg of oracle_verify_batch (what the CPU baseline times):
 * grant_flags[i] = MOCHI_GRANT_* for grants [begin, end). */
int oracle_verify_grants(const uint8_t* moduli_be, uint32_t n_keys, const mochi_batch* batch, uint32_t begin,
                         uint32_t end, uint8_t* grant_flags, int64_t* grant_ts, int n_threads);

/* Parse leg only: grant_flags[i] = MOCHI_GRANT_PARSED or 0, grant_ts[i] =
 * Grant.timestamp, for grants [begin, end); no signature checks. */
int oracle_parse_grants(const mochi_batch* batch, uint32_t begin, uint32_t end, uint8_t* grant_flags,
                        int64_t* grant_ts);

/* Only the tally leg, from precomputed grant_flags / grant_ts. */
int oracle_tally(const mochi_batch* batch, const mochi_params* params, const uint8_t* grant_flags,
                 const int64_t* grant_ts, mochi_verdicts* out);

/* Client-side response aggregation restated (MochiDBClient.java:148-175,
 * 355-382); same contract as mochi_tally_responses. */
int oracle_tally_responses(uint32_t n_requests, const uint32_t* resp_off, const uint32_t* n_ops,
                           const uint32_t* resp_n_ops, const uint64_t* status_off, const uint8_t* status,
                           const uint64_t* chosen_off, uint32_t replication_factor, int32_t* chosen,
                           uint8_t* reason, uint32_t* accept_bits);

/* Client isUniformTimeStampInMultiGrants restated (MochiDBClient.java:195-219)
 * for one Write1 round: grants listed MultiGrant by MultiGrant (wire order),
 * grant_key[i] = op key slot, ts[i] = timestamp.  Returns 1 uniform, 0 not. */
int oracle_write1_uniform(uint32_t n_grants, const uint8_t* grant_key, const int64_t* ts);

/* Client Write1 round classification restated (MochiDBClient.java:236-332,
 * with isUniformTimeStampInMultiGrants :195-219 and
 * removeWrongShardGrantFromMultiGrant :221-235); same contract as
 * mochi_write1_classify. */
int oracle_write1_classify(uint32_t n_requests, const uint32_t* resp_off, const uint8_t* resp_kind,
                           const uint32_t* resp_server, const uint32_t* resp_grant_off, const uint8_t* grant_key,
                           const int64_t* grant_ts, const uint8_t* grant_status, uint8_t* decision);

/* Write2ToServer wire decode restated (protobuf-java 3.16.3 semantics, see
 * mochi_oracle.c) into a mochi_batch whose grant_bytes is the wire blob.
 * Server ids: key k <-> ids[id_off[k], id_off[k+1]).  Free with oracle_w2_free. */
typedef struct oracle_w2_decoded {
  mochi_batch batch;
  uint8_t* msg_status; /* [M] enum mochi_msg_status */
  uint8_t* own_blob;   /* oracle_w2_decode_full: the blob batch.grant_bytes points into */
} oracle_w2_decoded;
int oracle_w2_decode(const mochi_write2_batch* w, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids,
                     oracle_w2_decoded* out);
void oracle_w2_free(oracle_w2_decoded* d);

/* Full protobuf-java decode of every message (no fast-path limits: merged
 * repeated fields, merged map values, non-canonical Grant bytes re-serialized
 * as Grant.toByteArray() incl. retained unknown fields, any number of
 * MultiGrants / grants).  grant_bytes is a new blob (own_blob) of the signed
 * bytes; op keys are slices of it.  msg_status: OK, MALFORMED, or FALLBACK for
 * more than MOCHI_MAX_OPS_PER_CERT operations. */
int oracle_w2_decode_full(const mochi_write2_batch* w, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids,
                          oracle_w2_decoded* out);

/* Decode + oracle_verify_batch + the per-message status fix-up; FALLBACK
 * messages are decided through oracle_w2_decode_full.  Same contract as
 * mochi_verify_write2. */
int oracle_verify_write2(const uint8_t* moduli_be, uint32_t n_keys, const uint8_t* ids, const uint32_t* id_off,
                         const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* out, uint8_t* msg_status,
                         int n_threads);

/* --- fixture generation helpers (tests only) --- */

/* Sign SHA-256(msg) with a PEM RSA private key (PKCS#1 v1.5).  Returns 1 ok. */
int oracle_rsa_sign(const char* pem_private_key, const uint8_t* msg, size_t len, uint8_t sig_out[256]);

/* Extract the big-endian modulus of a PEM private or public key.  Returns 1 ok. */
int oracle_pem_modulus(const char* pem_key, uint8_t n_be_out[256]);

#ifdef __cplusplus
}
#endif

#endif
