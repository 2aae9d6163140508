/*
 * mochi_hip.h — C ABI of libmochi_hip, the MI355X batch verifier for MochiDB's
 * Write2 certificate path.
 *
 * What this replaces in the reference (tomisetsu/mochi-db, Java):
 *
 *   InMemoryDataStore.processWrite2ToServer(Write2ToServer)           InMemoryDataStore.java:641-666
 *     ├ processMultiGrantsFromAllServers(wc.grantsMap, txn)           InMemoryDataStore.java:613-640
 *     └ write2apply(coalesced, msg)  (verdict part only)              InMemoryDataStore.java:576-611
 *   ClusterConfiguration.getServerMajority()                          ClusterConfiguration.java:264-267
 *   MochiDBClient Write2/Read response aggregation                    MochiDBClient.java:148-175, 355-382
 *
 * plus the per-grant signature check the reference leaves as a TODO
 * (MochiProtocol.proto:123 "// TODO: add signature"): SHA-256 over the
 * proto3-encoded Grant (MochiProtocol.java:7556-7574) and an RSA-2048
 * PKCS#1 v1.5 verify (JCA "SHA256withRSA", e = 65537).
 *
 * ABI rules: plain C, plain pointers and sizes, no torch / HIP types in the
 * signatures (a hipStream_t travels as void*).  Every entry point returns an
 * int status: 0 = ok, < 0 = argument / HIP error (text in mochi_last_error()).
 * A verdict is NEVER an error: rejects are bits and reason codes in the
 * output buffers (the reference throws, and RequestHandlerDispatcher.java:74-79
 * swallows, so a reject is observable only as a missing Write2Ans; the Java
 * shim in INTEGRATION.md maps reason codes back to those exception types).
 */
#ifndef MOCHI_HIP_H
#define MOCHI_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MOCHI_ABI_VERSION 3
#define MOCHI_RSA_BYTES 256     /* RSA-2048 modulus / signature size            */
#define MOCHI_RSA_E 65537u      /* the only public exponent supported          */
#define MOCHI_TXN_HASH_BYTES 128 /* lowercase-hex SHA-512 (Utils.java:135-153)  */
#define MOCHI_MAX_KEYS 4096     /* key-table entries per context               */
#define MOCHI_MAX_OPS_PER_CERT 64 /* transaction operations per certificate    */

/* Status codes. */
#define MOCHI_OK 0
#define MOCHI_EINVAL (-1)  /* bad argument / inconsistent batch          */
#define MOCHI_EHIP (-2)    /* HIP runtime error                          */
#define MOCHI_ENOMEM (-3)  /* device or pinned-host allocation failed    */
#define MOCHI_ENODEV (-4)  /* no usable gfx950 device                    */

/* Per-certificate verdict reason codes.  Each maps to the exception the
 * reference throws on that branch (see INTEGRATION.md for the Java mapping). */
enum mochi_reason {
  MOCHI_ACCEPT = 0,
  /* processMultiGrantsFromAllServers: a valid grant's timestamp differs from the
   * first valid grant seen for the same key -> UnsupportedOperationException
   * (InMemoryDataStore.java:626-628). */
  MOCHI_REJECT_TS_MISMATCH = 1,
  /* write2apply: no valid grant for a local op's key -> coalescedTxnGrantMap.get()
   * returns null -> NullPointerException (InMemoryDataStore.java:588). */
  MOCHI_REJECT_NO_GRANT = 2,
  /* write2apply: list.size() > getServerMajority() fails -> IllegalStateException
   * via Utils.assertTrue (InMemoryDataStore.java:590, Utils.java:43-47).  With
   * strict_gt = 0 the client predicate ">=" (MochiDBClient.java:172,379) is used. */
  MOCHI_REJECT_BELOW_QUORUM = 3,
  /* write2apply: g0.transactionHash != objectSHA512(txn) ->
   * UnsupportedOperationException (InMemoryDataStore.java:591,605-607). */
  MOCHI_REJECT_HASH_MISMATCH = 4,
  /* write2apply: no StoreValueObjectContainer for the key -> NullPointerException
   * (InMemoryDataStore.java:592-593).  Driven by MOCHI_OP_HAS_SVOC. */
  MOCHI_REJECT_NO_SVOC = 5,
  /* a grant's bytes are not a parseable proto3 Grant (the reference would fail
   * in the Netty protobuf decoder, MochiServerInitializer.java:30-34). */
  MOCHI_REJECT_MALFORMED = 6,
  /* Write2 wire path only: the message is legal protobuf but outside the
   * device decoder's fast path (enum mochi_msg_status MOCHI_MSG_FALLBACK /
   * MOCHI_MSG_OPS_MISMATCH) and the library's host decoder could not decide it
   * either (more than MOCHI_MAX_OPS_PER_CERT operations, or op_flags_off giving a
   * different operation count).  Never accepted. */
  MOCHI_UNDECIDED = 7,
  /* applyOperation: setCurrentC(wc) then getCurrentTimestampFromCurrentCertificate()
   * on the INCOMING certificate (InMemoryDataStore.java:533-534) throws
   * IllegalStateException: some MultiGrant of the certificate has no grant for the
   * op's key (StoreValueObjectContainer.java:186, Utils.assertNotNull) or two of
   * them carry different timestamps (:192-194).  Every MultiGrant counts here,
   * whatever its signatures (the Java loop runs over the stored certificate as
   * received).  Side effect in the reference: currentC is already replaced. */
  MOCHI_REJECT_APPLY_STATE = 8,
  /* write2apply :594: the key's STORED currentC throws in
   * getCurrentTimestampFromCurrentCertificate (op flag MOCHI_OP_CURRENT_C_BAD) ->
   * IllegalStateException. */
  MOCHI_REJECT_STORED_CERT = 9,
  /* readOperation / applyOperation on an op that is not a WRITE/DELETE, or whose
   * key holds no write lock (empty operand1 is never locked,
   * InMemoryDataStore.java:339-358): IllegalStateException (:525-526 / :560-561)
   * or UnsupportedOperationException (:551 / :572).  Op flag MOCHI_OP_NOT_WRITE. */
  MOCHI_REJECT_NOT_WRITE = 10,
};

/* Per-operation outcome of write2apply's loop (InMemoryDataStore.java:581-609),
 * mochi_verdicts.op_decision.  The reference is not atomic: the ops before a
 * failing op have already been applied when it throws. */
enum mochi_op_decision {
  MOCHI_OPD_SKIPPED = 0,     /* not reached (the certificate was rejected earlier)        */
  MOCHI_OPD_APPLY = 1,       /* applyOperation(op, wc) (:597): currentC := wc, ts = op_ts  */
  MOCHI_OPD_READ = 2,        /* readOperation(op) (:596): objectTS > g0.timestamp          */
  MOCHI_OPD_WRONG_SHARD = 3, /* WRONG_SHARD result (:582-587)                              */
  MOCHI_OPD_FAILED = 4,      /* this op's step threw: cert_reason / cert_fail_op          */
};

/* op_flags bits (one byte per transaction operation). */
#define MOCHI_OP_LOCAL 0x01    /* objectBelongsToCurrentShardServer(key)      InMemoryDataStore.java:63-72,582 */
#define MOCHI_OP_HAS_SVOC 0x02 /* getDataMap(key).get(key) != null           InMemoryDataStore.java:592 */
#define MOCHI_OP_HAS_CURRENT_C 0x04 /* the SVOC holds a certificate (currentC != null); its timestamp,
                                       getCurrentTimestampFromCurrentCertificate(), is op_object_ts[o]
                                       (StoreValueObjectContainer.java:175-198, InMemoryDataStore.java:594) */
#define MOCHI_OP_CURRENT_C_BAD 0x08 /* the SVOC's stored currentC makes that call throw (:594)    */
#define MOCHI_OP_NOT_WRITE 0x10     /* action is not WRITE/DELETE, or operand1 is empty (no write
                                       lock): the read/apply step throws.  The wire decoder sets it
                                       itself from Operation.action / operand1. */

/* grant_flags bits (one byte per grant, output). */
#define MOCHI_GRANT_SIG_OK 0x01   /* RSA/SHA-256 signature verified            */
#define MOCHI_GRANT_PARSED 0x02   /* bytes parsed as a Grant                   */

/*
 * A batch of Write2 certificates in struct-of-arrays form.
 *
 * Grants are listed certificate by certificate, in certificate WIRE order
 * (the MultiGrant map iteration order, which decides which grant is "g0",
 * InMemoryDataStore.java:588, MochiDBClient.java:333-338).  A grant's bytes
 * are the exact proto3 encoding that was signed (Grant.toByteArray(),
 * MochiProtocol.java:7556-7574) and may sit anywhere in `grant_bytes`
 * (e.g. as slices of the received Write2ToServer wire buffer: zero copy).
 *
 * All arrays are host pointers for mochi_verify_batch() and device pointers
 * for mochi_verify_batch_device().
 */
typedef struct mochi_batch {
  uint32_t n_grants;              /* N */
  uint32_t n_certs;               /* C */
  uint32_t n_ops;                 /* O = total transaction operations over all certificates */
  uint32_t n_mgs;                 /* total MultiGrants (size of mg_grant_off - 1); 0 with cert_mg_off NULL */
  uint64_t grant_bytes_len;       /* size of grant_bytes                                      */
  const uint8_t* grant_bytes;     /* blob holding every grant's proto3 bytes                  */
  const uint64_t* grant_off;      /* [N] byte offset of grant i in grant_bytes                */
  const uint32_t* grant_len;      /* [N] byte length of grant i (<= 65536)                    */
  const uint8_t* sig;             /* [N * 256] big-endian RSA signatures                      */
  const uint16_t* signer;         /* [N] key-table index of the signing server (MultiGrant.serverId) */
  const uint8_t* grant_key;       /* [N] key slot of the op key this grant is for (< ops in cert) */
  const uint32_t* cert_grant_off; /* [C+1] CSR: grants of cert c are [off[c], off[c+1])        */
  const uint32_t* cert_op_off;    /* [C+1] CSR: ops of cert c are [off[c], off[c+1])           */
  const uint8_t* op_key;          /* [O] key slot of each op (ops on the same key share a slot) */
  const uint8_t* op_flags;        /* [O] MOCHI_OP_* bits                                        */
  const uint8_t* expected_hash;   /* [C * 128] objectSHA512(txn) as lowercase hex (host-computed, §7.1.4) */
  /* --- ABI 2 --- */
  /* MultiGrant boundaries (the certificate map's values, wire order): the
   * MultiGrants of cert c are [cert_mg_off[c], cert_mg_off[c+1]) and the grants of
   * MultiGrant m are [mg_grant_off[m], mg_grant_off[m+1]) (empty MultiGrants
   * allowed); mg_grant_off[cert_mg_off[c]] == cert_grant_off[c].  NULL: every
   * maximal run of consecutive grants with one signer is one MultiGrant. */
  const uint32_t* cert_mg_off;    /* [C+1] or NULL                                              */
  const uint32_t* mg_grant_off;   /* [n_mgs+1] or NULL                                          */
  const int64_t* op_object_ts;    /* [O] stored currentC timestamp, read iff MOCHI_OP_HAS_CURRENT_C; NULL = none */
  /* The op key (Operation.operand1) bytes, as a slice of grant_bytes: needed only
   * by MOCHI_Q_BIND (Grant.objectId must equal it).  NULL otherwise. */
  const uint64_t* op_key_off;     /* [O] offset in grant_bytes                                  */
  const uint32_t* op_key_len;     /* [O]                                                        */
} mochi_batch;

/* mochi_params.quorum_mode bits.  0 = parity with the reference: every
 * signature-valid grant of the certificate counts once per op naming its key
 * (InMemoryDataStore.java:613-640, :590), whoever signed it.  The bits make the
 * new signature layer a Byzantine quorum; a grant they exclude is treated like
 * one with an invalid signature (absent, :622-624). */
#define MOCHI_Q_DISTINCT_SIGNERS 0x1 /* a signer counts at most once per key: only its first valid
                                        grant for the key (wire order) counts.  The honest client keys
                                        the certificate by MultiGrant.serverId (MochiDBClient.java:299,
                                        334), so honest certificates are unaffected. */
#define MOCHI_Q_BIND 0x2             /* a grant counts only if Grant.objectId equals the op key it is
                                        filed under and Grant.transactionHash equals expected_hash
                                        (no replay of a signer's grants for other objects or
                                        transactions).  Needs op_key_off / op_key_len. */

typedef struct mochi_params {
  uint32_t replication_factor; /* R = _CONFIG_BFT_REPLICATION; majority M = 2*(R/3)+1 */
  uint32_t strict_gt;          /* 1: server predicate count > M (InMemoryDataStore.java:590)
                                  0: client predicate count >= M (MochiDBClient.java:172,379) */
  uint32_t quorum_mode;        /* MOCHI_Q_* bits, 0 = reference parity */
  uint32_t _pad;
} mochi_params;

typedef struct mochi_verdicts {
  uint32_t* grant_valid_bits; /* [ceil(N/32)] bit i = grant i signature valid  (may be NULL) */
  uint8_t* grant_flags;       /* [N] MOCHI_GRANT_* bits                          (may be NULL) */
  int64_t* grant_ts;          /* [N] parsed Grant.timestamp                      (may be NULL) */
  uint32_t* cert_accept_bits; /* [ceil(C/32)] bit c = certificate accepted       (required)    */
  uint8_t* cert_reason;       /* [C] enum mochi_reason                           (may be NULL) */
  uint8_t* cert_fail_op;      /* [C] op index of the first failing op, 0xFF if none / n.a. (may be NULL) */
  /* --- ABI 2: per operation, in the batch's op order (may be NULL) --- */
  uint8_t* op_decision;       /* [O] enum mochi_op_decision                                     */
  uint32_t* op_g0;            /* [O] g0 of the op's key: certificate-relative index of the first
                                 counted grant for it (InMemoryDataStore.java:588), 0xFFFFFFFF none */
  int64_t* op_ts;             /* [O] g0's timestamp (the ts applyOperation records), 0 if none   */
} mochi_verdicts;

typedef struct mochi_ctx mochi_ctx;

/* ABI version of the loaded library (== MOCHI_ABI_VERSION). */
int mochi_abi_version(void);

/* Thread-local text of the last error returned on this thread. */
const char* mochi_last_error(void);

/* Number of visible HIP devices (0 when none). */
int mochi_device_count(void);

/*
 * Create a verifier on HIP device `device` with a key table of `n_keys`
 * RSA public keys.  `moduli_be` holds n_keys * key_bytes big-endian moduli
 * (key_bytes must be 256; every modulus exactly 2048 bits and odd);
 * `public_exponent` must be 65537.  Key index = MultiGrant.serverId's position
 * in the table.  Montgomery constants (n0', R^2 mod n) are derived here and
 * the table is uploaded once.  Returns NULL on error (see mochi_last_error()).
 */
mochi_ctx* mochi_ctx_create(int device, const uint8_t* moduli_be, uint32_t n_keys, uint32_t key_bytes,
                            uint32_t public_exponent);
/* Never blocks.  With no batcher holding the context it is freed now; while a
 * batcher built on it is alive (or a batcher destroyed from its own callback is
 * not yet freed by its last flusher) the context is freed by that batcher's
 * release instead.  Either way the handle must not be used after the call. */
void mochi_ctx_destroy(mochi_ctx* ctx);

/*
 * Verify a batch held in HOST memory.  The batch is cut into chunks of whole
 * certificates (~256k grants, env MOCHI_CHUNK_GRANTS); chunk j+1's upload
 * (hipMemcpyAsync on a copy stream; pageable arrays staged through pinned
 * buffers, pinned ones DMA'd in place) overlaps chunk j's kernels (grant prep
 * + RSA verify + certificate tally) and chunk j-1's verdict download.
 * Synchronous.  Thread-safe per context (calls on one context serialize).
 */
int mochi_verify_batch(mochi_ctx* ctx, const mochi_batch* batch, const mochi_params* params,
                       mochi_verdicts* out);

/*
 * Verify a batch already resident in DEVICE memory (every mochi_batch pointer
 * and every non-NULL mochi_verdicts pointer is a device pointer).  Enqueued on
 * `stream` (a hipStream_t; NULL = the null stream, as in every HIP API); asynchronous.  The
 * batch header itself is read on the host.  Scratch is owned by the context.
 */
int mochi_verify_batch_device(mochi_ctx* ctx, const mochi_batch* batch, const mochi_params* params,
                              mochi_verdicts* out, void* stream);

/*
 * The raw RSA public operation y = s^65537 mod n for n signatures (big-endian,
 * 256 bytes each) under key `signer[i]`, on the device, through the same
 * kernels as the verify path (k_rsa_pow + k_rsa_final).  out_be: n * 256
 * bytes.  out_z (optional, n * 74 words): the squaring-chain intermediate
 * z = s^(2^16) mod n in radix-2^28 limbs, not fully reduced (< 2^2064), for
 * tests.  Host memory, synchronous.
 */
int mochi_rsa_public_op(mochi_ctx* ctx, uint32_t n, const uint8_t* sig_be, const uint16_t* signer, uint8_t* out_be,
                        uint32_t* out_z);

/*
 * The k_rsa_pow fold matrix of one RSA-2048 modulus (inspection / tests; the
 * context builds one per key).  img: 102,400 int8 = the MFMA A fragments of
 * R_{j,b} = 2^(28(73+j)+8b) mod n in balanced mixed-radix digits (layout:
 * mochi-db_amd/csrc/fold.h); cadd: the int8 bias correction 128 * sum R_{j,b}
 * as 74 limbs of 28 bits.  Host memory.
 */
int mochi_fold_matrix(const uint8_t* modulus_be, int8_t* img, uint32_t* cadd);

/*
 * Per-stage device timing.  While profiling is on, every verify call records a
 * (start, end) hipEvent pair around each stage on the stream the stage runs
 * on; mochi_ctx_read_profile waits for them and returns the SUM over calls
 * since the last read, per stage: [0] grant prep (parse + SHA-256; it runs on
 * the context's aux stream, concurrently with [1] and [2]), [1] signer
 * bucketing, [2] k_rsa_pow, [3] k_rsa_final (+ bitmap pack), [4] k_tally.
 * n_stages <= 5.
 */
int mochi_ctx_set_profiling(mochi_ctx* ctx, int on);
int mochi_ctx_read_profile(mochi_ctx* ctx, float* stage_ms, uint32_t n_stages, uint32_t* n_calls);

/* Stream-event timings of the last mochi_verify_batch() call on this context
 * (milliseconds).  The host path is a chunked pipeline (uploads, kernels and
 * downloads of consecutive chunks overlap), so: h2d_ms = the first chunk's
 * upload (nothing else runs yet), kernels_ms = first kernel start -> last
 * kernel end, d2h_ms = the last chunk's download; mochi_ctx_last_total_ms
 * gives first upload start -> last download end. */
int mochi_ctx_last_timing(mochi_ctx* ctx, float* h2d_ms, float* kernels_ms, float* d2h_ms);
int mochi_ctx_last_total_ms(mochi_ctx* ctx, float* total_ms);

/* Host-path chunk size target in grants (0 = default: env MOCHI_CHUNK_GRANTS
 * or 262144).  Chunks always hold whole certificates, 32 at a time. */
int mochi_ctx_set_chunk_grants(mochi_ctx* ctx, uint32_t grants);

/* Small-batch launch sequence (a batcher flush of a few messages): a batch of
 * at most `grants` grants is bucketed by one kernel and prepped grant by grant
 * on the launch stream, instead of the large-batch sequence (three bucketing
 * kernels, the certificate-level grant dedup forked beside k_rsa_pow).  Same
 * outputs either way.  Default 4096; 0 = always the large-batch sequence. */
int mochi_ctx_set_small_batch(mochi_ctx* ctx, uint32_t grants);

/*
 * Pinned (page-locked) host memory for building batches in place: arrays of a
 * mochi_batch that live in such memory are DMA'd straight to the device by
 * mochi_verify_batch (no staging copy).  NULL on failure.
 */
void* mochi_host_alloc(uint64_t bytes);
void mochi_host_free(void* ptr);

/*
 * Producer side (the Write1 signing site the reference leaves as a TODO:
 * InMemoryDataStore.java:283-295, MochiProtocol.proto:123): sign SHA-256 of
 * each grant's bytes with an RSA-2048 private key (PEM, PKCS#1 v1.5,
 * "SHA256withRSA"), CPU / OpenSSL, `n_threads` threads.  sig_out: n * 256.
 */
int mochi_sign_grants(const char* pem_private_key, uint32_t n, const uint8_t* grant_bytes, const uint64_t* grant_off,
                      const uint32_t* grant_len, uint8_t* sig_out, int n_threads);

/* Big-endian modulus of a PEM RSA key (private or public) -> n_be_out[256]. */
int mochi_pem_modulus(const char* pem_key, uint8_t* n_be_out);

/*
 * Client-side response aggregation (MochiDBClient.java:148-175 reads,
 * 355-382 Write2): for each request r, responses [resp_off[r], resp_off[r+1])
 * each carry n_ops[r] op statuses (1 byte each, OperationResultStatus: 0 = OK,
 * 1 = WRONG_SHARD) at status + status_off[resp]; resp_n_ops[resp] is the op
 * count that response actually returned.  Request r is accepted iff every
 * response returned n_ops[r] results and, for every op, the number of
 * non-WRONG_SHARD results is >= M = 2*(R/3)+1.  chosen[status_off-aligned]
 * receives, per (request, op), the index of the LAST non-WRONG_SHARD response
 * (MochiDBClient.java:166,373) or -1.  reason[r]: 0 accept, 1 op-count
 * mismatch (InconsistentRead/WriteException at :159-161 / :366-368), 2 below
 * majority (:171-175 / :378-381).  Host memory; pure CPU.
 */
int mochi_tally_responses(uint32_t n_requests, const uint32_t* resp_off, const uint32_t* n_ops,
                          const uint32_t* resp_n_ops, const uint64_t* status_off, const uint8_t* status,
                          const uint64_t* chosen_off, uint32_t replication_factor, int32_t* chosen,
                          uint8_t* reason, uint32_t* accept_bits);

/* The same aggregation on the device, batched across in-flight transactions
 * (every pointer a device pointer; asynchronous on `stream`, a hipStream_t).
 * Lane = request.  accept_bits must hold ceil(n_requests/32) words. */
int mochi_tally_responses_device(uint32_t n_requests, const uint32_t* resp_off, const uint32_t* n_ops,
                                 const uint32_t* resp_n_ops, const uint64_t* status_off, const uint8_t* status,
                                 const uint64_t* chosen_off, uint32_t replication_factor, int32_t* chosen,
                                 uint8_t* reason, uint32_t* accept_bits, void* stream);

/* Write1 response kinds: the ProtocolMessage payload case a Write1ToServer got
 * back (MochiDBClient.java:274-289). */
#define MOCHI_W1_OK 0             /* WRITE1OKFROMSERVER                        */
#define MOCHI_W1_REFUSED 1        /* WRITE1REFUSEDFROMSERVER                   */
#define MOCHI_W1_REQUEST_FAILED 2 /* REQUESTFAILEDFROMSERVER                   */
#define MOCHI_W1_OTHER 3          /* any other payload                         */

/* Write1 round outcomes (MochiDBClient.executeWriteTransactionBL). */
enum mochi_write1_decision {
  MOCHI_W1_PROCEED = 0,           /* every response OK, timestamps uniform -> Write2 (:320-324)      */
  MOCHI_W1_RETRY = 1,             /* OK multigrants disagree on a key's timestamp -> sleep 1 ms and
                                     resend Write1 (isUniformTimeStampInMultiGrants, :195-219, :310-318) */
  MOCHI_W1_THROW_REFUSED = 2,     /* RequestRefusedException (:325-328)                              */
  MOCHI_W1_THROW_FAILED = 3,      /* RequestFailedException (:281-283)                               */
  MOCHI_W1_THROW_UNSUPPORTED = 4, /* a WRONG_SHARD grant in an OK/REFUSED multigrant:
                                     removeWrongShardGrantFromMultiGrant removes from protobuf's
                                     read-only map view -> UnsupportedOperationException (:221-228) */
};

/*
 * Client Write1 round classification (a8 + a9), batched over requests.
 * Request r owns responses [resp_off[r], resp_off[r+1]) in arrival order;
 * response q has payload kind resp_kind[q] (MOCHI_W1_*), the replying
 * MultiGrant.serverId as a small integer resp_server[q], and grants
 * [resp_grant_off[q], resp_grant_off[q+1]) (CSR over all responses).  Grant g:
 * grant_key[g] = slot of its objectId among the transaction's op keys (0xFF if
 * it is no op's key), grant_ts[g] = Grant.timestamp, grant_status[g] =
 * OperationResultStatus (0 OK, 1 WRONG_SHARD).  decision[r] receives an enum
 * mochi_write1_decision.  Host memory; pure CPU.
 */
int mochi_write1_classify(uint32_t n_requests, const uint32_t* resp_off, const uint8_t* resp_kind,
                          const uint32_t* resp_server, const uint32_t* resp_grant_off, const uint8_t* grant_key,
                          const int64_t* grant_ts, const uint8_t* grant_status, uint8_t* decision);
/* The Write1 classification on the device (device pointers, async on `stream`). */
int mochi_write1_classify_device(uint32_t n_requests, const uint32_t* resp_off, const uint8_t* resp_kind,
                                 const uint32_t* resp_server, const uint32_t* resp_grant_off, const uint8_t* grant_key,
                                 const int64_t* grant_ts, const uint8_t* grant_status, uint8_t* decision,
                                 void* stream);

/* ------------------------------------------------------------------------
 * Write2ToServer wire path: the device decodes the received protobuf bytes.
 *
 * Replaces the SoA assembly a caller of mochi_verify_batch has to do: it takes
 * the Write2ToServer message bodies exactly as they arrived
 * (MochiProtocol.proto:144-147, field 110 of a
 * ProtocolMessage), decodes them on the device with protobuf-java 3.16.3
 * semantics (map fields keep first-insertion order with last-value-wins,
 * unknown fields skipped, proto3 strings UTF-8 checked, any malformation fails
 * the whole message) and verifies them.  Grant bytes are verified in place
 * (zero copy); each grant's signature is MultiGrant.grantSignatures[objectId]
 * (the field INTEGRATION.md adds as MochiProtocol.proto:123's TODO) and its
 * signer is the key whose server id (mochi_ctx_set_server_ids) equals
 * MultiGrant.serverId.
 * ------------------------------------------------------------------------ */

/* Per-message decode status. */
enum mochi_msg_status {
  MOCHI_MSG_OK = 0,
  /* not a parseable Write2ToServer: protobuf-java's parser would throw
   * InvalidProtocolBufferException in the Netty decoder
   * (MochiServerInitializer.java:30-34) -> reason MOCHI_REJECT_MALFORMED */
  MOCHI_MSG_MALFORMED = 1,
  /* legal, but outside the device decoder's fast path -> reason
   * MOCHI_UNDECIDED: writeCertificate or transaction given more than once; a
   * map entry whose MultiGrant or Grant value is given more than once; a Grant
   * whose bytes are not the canonical encoding Grant.toByteArray() would give
   * (MochiProtocol.java:7556-7574); more than 32 certificate entries, or 64
   * grants or 64 grantSignatures entries in a decoded MultiGrant (counted on the
   * wire, repeated keys included), or more than 64 operations */
  MOCHI_MSG_FALLBACK = 2,
  /* op_flags_off gives a different operation count than the message holds */
  MOCHI_MSG_OPS_MISMATCH = 3,
};

typedef struct mochi_write2_batch {
  uint32_t n_msgs; /* M */
  uint32_t _pad0;
  uint64_t wire_len;              /* size of wire                                             */
  const uint8_t* wire;            /* blob holding every Write2ToServer body                    */
  const uint64_t* msg_off;        /* [M] byte offset of message m in wire                      */
  const uint32_t* msg_len;        /* [M] byte length of message m                              */
  const uint32_t* op_flags_off;   /* [M+1] CSR into op_flags; NULL = every op LOCAL|HAS_SVOC    */
  const uint8_t* op_flags;        /* MOCHI_OP_* per operation, transaction order               */
  const uint8_t* expected_hash;   /* [M * 128] objectSHA512(transaction), lowercase hex         */
  /* --- ABI 2 --- */
  const int64_t* op_object_ts;    /* aligned with op_flags (CSR op_flags_off): stored currentC
                                     timestamp, read iff MOCHI_OP_HAS_CURRENT_C; NULL = none      */
} mochi_write2_batch;

/* Server-id table of the context: key i of the key table belongs to the server
 * whose MultiGrant.serverId is ids[id_off[i], id_off[i+1]).  n_ids must equal
 * the context's key count; ids <= 256 bytes each. */
int mochi_ctx_set_server_ids(mochi_ctx* ctx, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids);

/* Decode + verify M Write2ToServer messages held in HOST memory.  Only the
 * certificate-level and per-op verdict arrays of `out` are written (grant-level
 * pointers must be NULL); per-op arrays need op_flags_off and follow its layout
 * (ops of messages that were not decoded read MOCHI_OPD_SKIPPED).
 * msg_status[M] receives enum mochi_msg_status.  Messages the device decoder
 * leaves to the host (MOCHI_MSG_FALLBACK: repeated / merged fields, non-canonical
 * Grant bytes, more than 32 MultiGrants or 64 grants per MultiGrant) are decoded
 * by the library's host decoder with full protobuf-java semantics and verified
 * on the device like any other certificate -- signatures are always checked;
 * msg_status still reports MOCHI_MSG_FALLBACK for them.  Synchronous; batches
 * larger than the chunk target are pipelined (upload / decode+verify / download
 * of consecutive chunks overlap). */
int mochi_verify_write2(mochi_ctx* ctx, const mochi_write2_batch* batch, const mochi_params* params,
                        mochi_verdicts* out, uint8_t* msg_status);

/* Same with every pointer of `batch`, `out` and msg_status in DEVICE memory,
 * enqueued on `stream` (hipStream_t; NULL = null stream).  The decoded batch
 * is sized on the device; the call waits for its grant / op totals. */
int mochi_verify_write2_device(mochi_ctx* ctx, const mochi_write2_batch* batch, const mochi_params* params,
                               mochi_verdicts* out, uint8_t* msg_status, void* stream);

/* The device decoder's output for M messages in HOST memory (inspection and
 * tests; mochi_verify_write2 never copies it back).  Arrays are allocated by
 * the library; release them with mochi_write2_decoded_free.  grant_off is
 * relative to the start of `wire`. */
typedef struct mochi_write2_decoded {
  uint32_t n_msgs, n_grants, n_ops, n_mgs;
  uint64_t* grant_off;      /* [N] */
  uint32_t* grant_len;      /* [N] */
  uint8_t* sig;             /* [N * 256] */
  uint16_t* signer;         /* [N] key index, 0xFFFF = unknown serverId */
  uint8_t* grant_key;       /* [N] op key slot, 0xFF = no op names it */
  uint32_t* cert_grant_off; /* [M+1] */
  uint32_t* cert_op_off;    /* [M+1] */
  uint8_t* op_key;          /* [O] */
  uint8_t* op_flags;        /* [O] */
  uint8_t* msg_status;      /* [M] enum mochi_msg_status */
  /* ABI 2 */
  uint32_t* cert_mg_off;    /* [M+1] MultiGrants per message (CSR) */
  uint32_t* mg_grant_off;   /* [n_mgs+1] grants per MultiGrant (CSR) */
  uint64_t* op_key_off;     /* [O] Operation.operand1, offset relative to `wire` */
  uint32_t* op_key_len;     /* [O] */
} mochi_write2_decoded;
int mochi_write2_decode(mochi_ctx* ctx, const mochi_write2_batch* batch, mochi_write2_decoded* out);
void mochi_write2_decoded_free(mochi_write2_decoded* d);

/* ------------------------------------------------------------------------
 * Producer side on the device: SHA256withRSA over each grant's bytes with ONE
 * server's private key (RSA-2048, CRT), the Write1 signing site
 * (InMemoryDataStore.java:283-295, MochiProtocol.proto:123 TODO).  Output is
 * bit-identical to mochi_sign_grants / OpenSSL (PKCS#1 v1.5 is deterministic).
 * ------------------------------------------------------------------------ */
typedef struct mochi_signer mochi_signer;
mochi_signer* mochi_signer_create(int device, const char* pem_private_key);
void mochi_signer_destroy(mochi_signer* s);
/* Host memory, synchronous; sig_out: n * 256 bytes. */
int mochi_sign_batch(mochi_signer* s, const uint8_t* grant_bytes, uint64_t grant_bytes_len, const uint64_t* grant_off,
                     const uint32_t* grant_len, uint32_t n, uint8_t* sig_out);
/* Device memory, asynchronous on `stream`. */
int mochi_sign_batch_device(mochi_signer* s, const uint8_t* grant_bytes, const uint64_t* grant_off,
                            const uint32_t* grant_len, uint32_t n, uint8_t* sig_out, void* stream);
/* Every signature is verified with the signer's public key before it is
 * released (same stream, ~2 % of the signing cost): a transient fault in one
 * RSA-CRT half would otherwise publish s with gcd(s^e - EM, n) = a prime factor.
 * A failing signature is written as 256 zero bytes (it verifies nowhere).
 * mochi_signer_rejected waits for the device and returns (and clears) the
 * number withheld since the last call. */
int mochi_signer_rejected(mochi_signer* s, uint64_t* rejected);
/* Test hook: corrupt the CRT half m_p of grant `grant_index` of every later call
 * (0xFFFFFFFF = off), to show the fault check withholding it. */
int mochi_signer_set_fault(mochi_signer* s, uint32_t grant_index);

/* ------------------------------------------------------------------------
 * Micro-batcher: the blocking per-request call the Java handler keeps
 * (Write2ToServerRequestHandler.handle -> processWrite2ToServer on a 2..20
 * thread pool, MochiServer.java:36-40), coalesced across threads into one
 * mochi_verify_write2 call by a flusher thread: a batch goes out when
 * max_msgs requests are pending or the oldest has waited max_wait_us.
 * ------------------------------------------------------------------------ */
typedef struct mochi_batcher mochi_batcher;

typedef struct mochi_verdict1 {
  uint8_t accepted;   /* certificate accepted                 */
  uint8_t reason;     /* enum mochi_reason                    */
  uint8_t fail_op;    /* first failing op, 0xFF if none       */
  uint8_t msg_status; /* enum mochi_msg_status                */
} mochi_verdict1;

/* with_op_flags: 1 = every call passes op_flags[n_ops] (MOCHI_OP_* per op, in
 * transaction order); 0 = calls pass NULL / 0 and every op counts as
 * LOCAL|HAS_SVOC.  The batcher borrows `ctx` (one batcher per context). */
mochi_batcher* mochi_batcher_create(mochi_ctx* ctx, const mochi_params* params, uint32_t max_msgs,
                                    uint32_t max_wait_us, int with_op_flags);
/* The same over n_ctx contexts (e.g. two on one GPU): one flusher thread per
 * context takes the next batch while the others are on the GPU, so n batches
 * are in flight.  The batcher borrows the contexts. */
mochi_batcher* mochi_batcher_create_multi(mochi_ctx* const* ctxs, uint32_t n_ctx, const mochi_params* params,
                                          uint32_t max_msgs, uint32_t max_wait_us, int with_op_flags);
typedef void (*mochi_verdict_cb)(void* user, int rc, const mochi_verdict1* verdict);

/* One Write2ToServer request (ABI 3): the message body plus the receiving
 * server's per-op state and optional per-op outputs.  Everything stays owned by
 * the caller and must stay valid until the verdict is delivered. */
typedef struct mochi_write2_request {
  const uint8_t* msg;            /* Write2ToServer body (ProtocolMessage field 110)            */
  uint32_t msg_len;
  uint32_t n_ops;                /* operations in the message's transaction                   */
  const uint8_t* op_flags;       /* [n_ops] MOCHI_OP_* (batcher created with with_op_flags)     */
  const int64_t* op_object_ts;   /* [n_ops] stored currentC timestamp, read iff HAS_CURRENT_C;
                                    NULL = none                                                */
  const uint8_t* expected_hash;  /* [128] objectSHA512(transaction), lowercase hex              */
  uint8_t* op_decision;          /* [n_ops] out: enum mochi_op_decision (NULL = not wanted)     */
  uint32_t* op_g0;               /* [n_ops] out: certificate-relative index of g0               */
  int64_t* op_ts;                /* [n_ops] out: g0's timestamp (what applyOperation records)   */
} mochi_write2_request;

/* Blocks until this request's verdict is in `out` (and its per-op outputs are
 * written).  Thread-safe.  Returns the status of the batch call that carried
 * it.  This is the call a server's Write2 handler makes in place of
 * InMemoryDataStore.processWrite2ToServer (InMemoryDataStore.java:641-666): the
 * per-op decision says which operations applyOperation / readOperation runs.
 * MOCHI_EINVAL (and mochi_last_error) from a completion callback running on
 * this batcher: a callback submits instead. */
int mochi_batcher_verify_request(mochi_batcher* b, const mochi_write2_request* req, mochi_verdict1* out);
/* Non-blocking form: cb(user, rc, &verdict) runs on a flusher thread once the
 * batch is verified, after the per-op outputs are written.  A callback may
 * submit to the batcher running it (e.g. the next stage of a future chain);
 * _verify* from a callback returns MOCHI_EINVAL. */
int mochi_batcher_submit_request(mochi_batcher* b, const mochi_write2_request* req, mochi_verdict_cb cb, void* user);
/* Blocks until this message's verdict is in `out`.  Thread-safe.  Returns the
 * status of the batch call that carried it. */
int mochi_batcher_verify(mochi_batcher* b, const uint8_t* msg, uint32_t msg_len, const uint8_t* op_flags,
                         uint32_t n_ops, const uint8_t* expected_hash, mochi_verdict1* out);
/* Non-blocking form for an event-loop caller (e.g. a Netty handler completing a
 * future): enqueue one message and return; cb(user, rc, &verdict) runs on a
 * flusher thread once its batch is verified (rc = the batch call's status).
 * msg / op_flags / expected_hash must stay valid until the callback.  With
 * thousands of requests in flight the batches grow to max_msgs, so throughput
 * follows the bulk wire path instead of 1 / latency per blocked thread. */
int mochi_batcher_submit(mochi_batcher* b, const uint8_t* msg, uint32_t msg_len, const uint8_t* op_flags,
                         uint32_t n_ops, const uint8_t* expected_hash, mochi_verdict_cb cb, void* user);
int mochi_batcher_stats(mochi_batcher* b, uint64_t* batches, uint64_t* msgs);
/* Drains pending requests, then stops the flushers and frees the batcher once
 * every blocked caller has returned.  From one of the batcher's own callbacks
 * the teardown is deferred instead: later submissions are refused with
 * MOCHI_EINVAL, requests already queued still complete, and the last flusher
 * frees the batcher; the handle must not be used after the call either way.
 * The batcher holds its contexts until it is freed: mochi_ctx_destroy on one of
 * them while a batcher still holds it returns at once and the context is freed
 * by the batcher's release (never while a flusher still uses it), so a caller
 * that tears down right after its last callback -- or closes the context before
 * the batcher -- neither blocks nor frees a context in use.  A process that
 * exits without destroying the contexts must not exit from a callback. */
void mochi_batcher_destroy(mochi_batcher* b);

/* ------------------------------------------------------------------------
 * Cluster configuration (ABI 3): the reference's properties file
 * (ClusterConfiguration.loadInitialConfigurationFromProperties,
 * ClusterConfiguration.java:138-187; config/sample_config): _CONFIG_SERVERS,
 * _CONFIG_BFT_REPLICATION, _CONFIG_SERVER_<id>_URL, _CONFIG_SERVER_<id>_TOKENS.
 * Host only.  Errors (MOCHI_EINVAL + mochi_last_error()) where the reference
 * throws: a server without URL, a token >= 1024 or mapped twice, a token left
 * unassigned, no replication factor, R < 4 or R > the token owners (:182-184).
 * ------------------------------------------------------------------------ */
typedef struct mochi_config mochi_config;
mochi_config* mochi_config_load(const char* path);
/* The same from the properties text itself. */
mochi_config* mochi_config_parse(const char* text, uint64_t len);
void mochi_config_free(mochi_config* c);
/* R (_CONFIG_BFT_REPLICATION) and M = getServerMajority() = 2*(R/3)+1. */
uint32_t mochi_config_replication(const mochi_config* c);
uint32_t mochi_config_majority(const mochi_config* c);
/* Servers in _CONFIG_SERVERS order: id and URL (NUL-terminated, owned by c). */
uint32_t mochi_config_n_servers(const mochi_config* c);
const char* mochi_config_server_id(const mochi_config* c, uint32_t i);
const char* mochi_config_server_url(const mochi_config* c, uint32_t i);
/* getServersForObject(key) (ClusterConfiguration.java:194-226): R indices into
 * the server table, in replica order.  Faithful to the reference, whose loop
 * reads token i instead of ithTokenValue (:215), so every key maps to the
 * owners of tokens 0..R-1; key = UTF-8 bytes (hashed as Java String.hashCode). */
int mochi_config_servers_for_key(const mochi_config* c, const uint8_t* key, uint32_t key_len, uint32_t* idx_out);
/* Server-id table of the replica set of `key` (or of tokens 0..R-1 for key =
 * NULL), laid out for mochi_ctx_set_server_ids: ids_out = the ids back to back,
 * id_off[R+1].  ids_cap = capacity of ids_out; returns the bytes needed (or
 * < 0 on error), writing nothing beyond ids_cap. */
int64_t mochi_config_replica_ids(const mochi_config* c, const uint8_t* key, uint32_t key_len, uint8_t* ids_out,
                                 uint64_t ids_cap, uint32_t* id_off);

/* ------------------------------------------------------------------------
 * Multi-GPU: certificates are independent, so a batch is cut
 * into contiguous certificate ranges, one per GPU, every boundary a multiple of
 * 32 certificates (the per-GPU accept bitmaps then concatenate word by word).
 * The only collective is one RCCL all-gather of those bitmaps over xGMI, after
 * which every GPU holds the whole batch's verdict bitmap.
 * ------------------------------------------------------------------------ */

/* Shard plan: cert_lo[n_shards+1], shard s = [cert_lo[s], cert_lo[s+1]), every
 * inner boundary a multiple of 32, the shards' work as even as that allows
 * (work = grants via cert_grant_off[C+1]; NULL = certificates).  Host only. */
int mochi_shard_plan(uint32_t n_certs, const uint32_t* cert_grant_off, uint32_t n_shards, uint32_t* cert_lo);
/* Words per shard slot of the all-gather (max over shards of ceil(size/32)). */
uint32_t mochi_shard_words(uint32_t n_shards, const uint32_t* cert_lo);
/* The batch's accept bitmap from an all-gathered buffer of n_shards slots of
 * words_per_shard words (slot s = shard s's bitmap, zero-padded). */
int mochi_bits_assemble(uint32_t n_shards, const uint32_t* cert_lo, uint32_t words_per_shard, const uint32_t* gathered,
                        uint32_t* bits_out);

/* One process owning several GPUs (e.g. one JVM server on an 8-GPU node):
 * bit i of device_mask = HIP device i; one context per device, each driven by
 * its own host thread, and an RCCL communicator over them (ncclCommInitAll). */
typedef struct mochi_mctx mochi_mctx;
mochi_mctx* mochi_mctx_create(uint64_t device_mask, const uint8_t* moduli_be, uint32_t n_keys, uint32_t key_bytes,
                              uint32_t public_exponent);
void mochi_mctx_destroy(mochi_mctx* m);
/* Device ids of the context (returns their count). */
int mochi_mctx_devices(mochi_mctx* m, int* devices, int max);
/* The per-device context i (profiling, chunk size, ...); owned by m. */
mochi_ctx* mochi_mctx_context(mochi_mctx* m, int i);
int mochi_mctx_set_server_ids(mochi_mctx* m, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids);
/* Host batch across the devices: each device runs mochi_verify_batch on its
 * shard (outputs land in their slices of `out`; grant_valid_bits is not
 * supported here, use grant_flags), then each device's accept bitmap is
 * all-gathered from where the verify left it in device memory (no host
 * round trip) and out->cert_accept_bits is assembled from one copy of device
 * 0's gathered buffer.  The per-device contexts must not be used by other
 * threads during the call. */
int mochi_mverify_batch(mochi_mctx* m, const mochi_batch* batch, const mochi_params* params, mochi_verdicts* out);
/* Write2ToServer messages across the devices (shards by wire bytes); as
 * mochi_verify_write2, the grant-level outputs must be NULL (MOCHI_EINVAL). */
int mochi_mverify_write2(mochi_mctx* m, const mochi_write2_batch* batch, const mochi_params* params,
                         mochi_verdicts* out, uint8_t* msg_status);
/* After a call: device i's all-gathered buffer (n_devices slots of
 * words_per_device words, device memory of device i). */
int mochi_mctx_gathered_bits(mochi_mctx* m, int i, const uint32_t** d_bits, uint32_t* words_per_device);

/* One process per GPU (torchrun / MPI style).  Rank 0 makes the 128-byte id,
 * the caller moves it to every rank by any transport, each rank joins. */
#define MOCHI_COMM_ID_BYTES 128
typedef struct mochi_comm mochi_comm;
int mochi_comm_unique_id(uint8_t* id_out /* [128] */);
mochi_comm* mochi_comm_init(const uint8_t* id /* [128] */, int n_ranks, int rank, int device);
/* ncclAllGather of words_per_rank uint32 per rank: d_recv[n_ranks * words_per_rank]
 * (d_send may be d_recv + rank * words_per_rank), async on `stream`. */
int mochi_comm_allgather_bits(mochi_comm* c, const uint32_t* d_send, uint32_t words_per_rank, uint32_t* d_recv,
                              void* stream);
void mochi_comm_destroy(mochi_comm* c);

/* Test hook (host only, no GPU): the per-device protocol mochi_mverify_* use
 * around the all-gather (multi.cpp run_gather), with n simulated devices whose
 * device selection / slot fill / collective enqueue fail per bit of the masks
 * and whose collective is a host rendezvous of all n.  Returns the protocol's
 * status; *entered_collective = devices that enqueued, *timed_out = devices that
 * waited `timeout_ms` for a peer that never came (the hang the protocol must
 * rule out: always 0). */
int mochi_test_gather_protocol(uint32_t n, uint32_t fail_select, uint32_t fail_fill, uint32_t fail_enqueue,
                               uint32_t timeout_ms, uint32_t* entered_collective, uint32_t* timed_out);

#ifdef __cplusplus
}
#endif

#endif /* MOCHI_HIP_H */
