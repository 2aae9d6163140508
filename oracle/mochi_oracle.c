/*
 * mochi_oracle.c — CPU restatement of MochiDB's Write2 certificate path plus
 * the OpenSSL-pinned per-grant signature check.  TEST INFRASTRUCTURE ONLY
 * (see mochi_oracle.h): never linked into libmochi_hip.
 *
 * Every function cites the reference lines it restates; paths are relative to
 * /root/reference/src/main/java/edu/stanford/cs244b/mochi/.
 */
#define _GNU_SOURCE
#include "mochi_oracle.h"

#include <openssl/bn.h>
#include <openssl/evp.h>
#include <openssl/pem.h>
#include <openssl/rsa.h>
#include <openssl/core_names.h>
#include <openssl/param_build.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* a1: Grant encoding — server/messages/MochiProtocol.java:7556-7574          */
/* ------------------------------------------------------------------------ */

static size_t put_varint(uint8_t* p, uint64_t v) {
  size_t n = 0;
  while (v >= 0x80) {
    p[n++] = (uint8_t)(v | 0x80);
    v >>= 7;
  }
  p[n++] = (uint8_t)v;
  return n;
}

long oracle_grant_encode(const char* object_id, size_t object_id_len, int64_t timestamp, int64_t configstamp,
                         const char* txn_hash, size_t txn_hash_len, int32_t status, uint8_t* out, size_t cap) {
  uint8_t tmp[16];
  size_t need = 0;
  /* worst-case size first */
  need = (object_id_len ? 1 + 5 + object_id_len : 0) + (timestamp ? 11 : 0) + (configstamp ? 11 : 0) +
         (txn_hash_len ? 1 + 5 + txn_hash_len : 0) + (status ? 11 : 0);
  uint8_t* buf = (uint8_t*)malloc(need + 1);
  size_t n = 0;
  /* if (!getObjectIdBytes().isEmpty()) writeString(output, 1, objectId_)  :7558-7560 */
  if (object_id_len) {
    buf[n++] = 0x0A;
    n += put_varint(buf + n, object_id_len);
    memcpy(buf + n, object_id, object_id_len);
    n += object_id_len;
  }
  /* if (timestamp_ != 0L) output.writeInt64(2, timestamp_)  :7561-7563 (int64 -> varint of the u64 bits) */
  if (timestamp) {
    buf[n++] = 0x10;
    n += put_varint(buf + n, (uint64_t)timestamp);
  }
  /* if (configstamp_ != 0L) output.writeInt64(3, configstamp_)  :7564-7566 */
  if (configstamp) {
    buf[n++] = 0x18;
    n += put_varint(buf + n, (uint64_t)configstamp);
  }
  /* if (!getTransactionHashBytes().isEmpty()) writeString(output, 4, transactionHash_)  :7567-7569 */
  if (txn_hash_len) {
    buf[n++] = 0x22;
    n += put_varint(buf + n, txn_hash_len);
    memcpy(buf + n, txn_hash, txn_hash_len);
    n += txn_hash_len;
  }
  /* if (status_ != OK) output.writeEnum(5, status_)  :7570-7572 (enum = int32 varint, sign-extended) */
  if (status) {
    buf[n++] = 0x28;
    n += put_varint(buf + n, (uint64_t)(int64_t)status);
  }
  (void)tmp;
  long ret = -1;
  if (n <= cap) {
    memcpy(out, buf, n);
    ret = (long)n;
  }
  free(buf);
  return ret;
}

/* ------------------------------------------------------------------------ */
/* Grant parse — MochiProtocol.java:7369-7425 (protobuf-java 3.16.3           */
/* CodedInputStream: readTag / readRawVarint64 / readStringRequireUtf8 /      */
/* parseUnknownFieldProto3 -> skipField).                                      */
/* ------------------------------------------------------------------------ */

typedef struct {
  const uint8_t* b;
  size_t len, pos;
} rd_t;

/* readRawVarint64: at most 10 bytes, else malformedVarint. */
static int rd_varint(rd_t* r, uint64_t* v) {
  uint64_t x = 0;
  for (int i = 0; i < 10; i++) {
    if (r->pos >= r->len) return 0; /* truncatedMessage */
    uint8_t c = r->b[r->pos++];
    x |= (uint64_t)(c & 0x7F) << (7 * i);
    if (!(c & 0x80)) {
      *v = x;
      return 1;
    }
  }
  return 0; /* malformedVarint */
}

/* Utf8.isValidUtf8 (strict: no overlong forms, no surrogates, <= U+10FFFF). */
static int valid_utf8(const uint8_t* s, size_t n) {
  size_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) {
      i++;
      continue;
    }
    if (c < 0xC2) return 0;
    if (c < 0xE0) {
      if (i + 1 >= n || (s[i + 1] & 0xC0) != 0x80) return 0;
      i += 2;
      continue;
    }
    if (c < 0xF0) {
      if (i + 2 >= n) return 0;
      uint8_t c1 = s[i + 1], c2 = s[i + 2];
      if ((c1 & 0xC0) != 0x80 || (c2 & 0xC0) != 0x80) return 0;
      if (c == 0xE0 && c1 < 0xA0) return 0; /* overlong */
      if (c == 0xED && c1 >= 0xA0) return 0; /* surrogate */
      i += 3;
      continue;
    }
    if (c < 0xF5) {
      if (i + 3 >= n) return 0;
      uint8_t c1 = s[i + 1], c2 = s[i + 2], c3 = s[i + 3];
      if ((c1 & 0xC0) != 0x80 || (c2 & 0xC0) != 0x80 || (c3 & 0xC0) != 0x80) return 0;
      if (c == 0xF0 && c1 < 0x90) return 0; /* overlong */
      if (c == 0xF4 && c1 >= 0x90) return 0; /* > U+10FFFF */
      i += 4;
      continue;
    }
    return 0;
  }
  return 1;
}

/* readStringRequireUtf8: varint32 length (negative -> error), bytes, UTF-8 check. */
static int rd_string(rd_t* r, uint32_t* off, uint32_t* len) {
  uint64_t l;
  if (!rd_varint(r, &l)) return 0;
  int32_t l32 = (int32_t)(uint32_t)l; /* readRawVarint32 keeps the low 32 bits */
  if (l32 < 0) return 0;                /* negativeSize */
  if ((uint64_t)l32 > r->len - r->pos) return 0; /* truncatedMessage */
  if (!valid_utf8(r->b + r->pos, (size_t)l32)) return 0; /* invalidUtf8 */
  *off = (uint32_t)r->pos;
  *len = (uint32_t)l32;
  r->pos += (size_t)l32;
  return 1;
}

#define ORACLE_MAX_GROUP_DEPTH 100 /* CodedInputStream default recursion limit */

int oracle_grant_parse(const uint8_t* buf, size_t len, oracle_grant_view* out) {
  rd_t r = {buf, len, 0};
  oracle_grant_view g;
  memset(&g, 0, sizeof g);
  uint32_t group_stack[ORACLE_MAX_GROUP_DEPTH];
  int depth = 0;
  while (r.pos < r.len) {
    uint64_t tag64;
    if (!rd_varint(&r, &tag64)) return 0;
    uint32_t tag = (uint32_t)tag64; /* readTag -> readRawVarint32 */
    uint32_t field = tag >> 3, wt = tag & 7;
    if (field == 0) return 0; /* invalidTag */
    if (depth > 0) {
      /* inside an unknown group being skipped (skipMessage) */
      if (wt == 4) {
        if (group_stack[depth - 1] != field) return 0; /* invalidEndTag */
        depth--;
        continue;
      }
    } else {
      switch (tag) {
        case 10: /* objectId  :7389-7393 */
          if (!rd_string(&r, &g.object_id_off, &g.object_id_len)) return 0;
          continue;
        case 16: { /* timestamp :7394-7398 */
          uint64_t v;
          if (!rd_varint(&r, &v)) return 0;
          g.timestamp = (int64_t)v;
          continue;
        }
        case 24: { /* configstamp :7399-7403 */
          uint64_t v;
          if (!rd_varint(&r, &v)) return 0;
          g.configstamp = (int64_t)v;
          continue;
        }
        case 34: /* transactionHash :7404-7408 */
          if (!rd_string(&r, &g.txn_hash_off, &g.txn_hash_len)) return 0;
          continue;
        case 40: { /* status (readEnum = readRawVarint32) :7409-7413 */
          uint64_t v;
          if (!rd_varint(&r, &v)) return 0;
          g.status = (int32_t)(uint32_t)v;
          continue;
        }
        default:
          break;
      }
    }
    /* parseUnknownFieldProto3 -> skipField by wire type */
    switch (wt) {
      case 0: {
        uint64_t v;
        if (!rd_varint(&r, &v)) return 0;
        break;
      }
      case 1:
        if (r.len - r.pos < 8) return 0;
        r.pos += 8;
        break;
      case 2: {
        uint64_t l;
        if (!rd_varint(&r, &l)) return 0;
        int32_t l32 = (int32_t)(uint32_t)l;
        if (l32 < 0 || (uint64_t)l32 > r.len - r.pos) return 0;
        r.pos += (size_t)l32;
        break;
      }
      case 3:
        if (depth >= ORACLE_MAX_GROUP_DEPTH) return 0;
        group_stack[depth++] = field;
        break;
      case 4:
        return 0; /* END_GROUP at top level: parse stops, checkLastTagWas(0) fails */
      case 5:
        if (r.len - r.pos < 4) return 0;
        r.pos += 4;
        break;
      default:
        return 0; /* invalidWireType */
    }
  }
  if (depth != 0) return 0; /* truncated inside a group */
  *out = g;
  return 1;
}

/* ------------------------------------------------------------------------ */
/* a2 (NEW, no reference): SHA-256 + RSA-2048 PKCS#1 v1.5 ("SHA256withRSA")    */
/* Signing site: InMemoryDataStore.java:283-295 / MochiProtocol.proto:123.    */
/* ------------------------------------------------------------------------ */

void oracle_sha256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  unsigned int olen = 32;
  EVP_Digest(msg, len, out, &olen, EVP_sha256(), NULL);
}

static EVP_PKEY* make_pubkey(const uint8_t n_be[256]) {
  BIGNUM* n = BN_bin2bn(n_be, 256, NULL);
  BIGNUM* e = BN_new();
  BN_set_word(e, MOCHI_RSA_E);
  OSSL_PARAM_BLD* bld = OSSL_PARAM_BLD_new();
  OSSL_PARAM_BLD_push_BN(bld, OSSL_PKEY_PARAM_RSA_N, n);
  OSSL_PARAM_BLD_push_BN(bld, OSSL_PKEY_PARAM_RSA_E, e);
  OSSL_PARAM* params = OSSL_PARAM_BLD_to_param(bld);
  EVP_PKEY_CTX* pctx = EVP_PKEY_CTX_new_from_name(NULL, "RSA", NULL);
  EVP_PKEY* pkey = NULL;
  if (pctx && EVP_PKEY_fromdata_init(pctx) > 0) EVP_PKEY_fromdata(pctx, &pkey, EVP_PKEY_PUBLIC_KEY, params);
  EVP_PKEY_CTX_free(pctx);
  OSSL_PARAM_free(params);
  OSSL_PARAM_BLD_free(bld);
  BN_free(n);
  BN_free(e);
  return pkey;
}

static int verify_with_pkey(EVP_PKEY* pkey, const uint8_t* msg, size_t len, const uint8_t sig[256]) {
  EVP_MD_CTX* md = EVP_MD_CTX_new();
  int ok = 0;
  if (EVP_DigestVerifyInit(md, NULL, EVP_sha256(), NULL, pkey) > 0)
    ok = EVP_DigestVerify(md, sig, 256, msg, len) == 1;
  EVP_MD_CTX_free(md);
  return ok;
}

int oracle_rsa_verify(const uint8_t n_be[256], const uint8_t* msg, size_t len, const uint8_t sig[256]) {
  EVP_PKEY* pkey = make_pubkey(n_be);
  if (!pkey) return 0;
  int ok = verify_with_pkey(pkey, msg, len, sig);
  EVP_PKEY_free(pkey);
  return ok;
}

int oracle_rsa_sign(const char* pem_private_key, const uint8_t* msg, size_t len, uint8_t sig_out[256]) {
  BIO* bio = BIO_new_mem_buf(pem_private_key, -1);
  EVP_PKEY* pkey = PEM_read_bio_PrivateKey(bio, NULL, NULL, NULL);
  BIO_free(bio);
  if (!pkey) return 0;
  EVP_MD_CTX* md = EVP_MD_CTX_new();
  size_t slen = 256;
  int ok = EVP_DigestSignInit(md, NULL, EVP_sha256(), NULL, pkey) > 0 &&
           EVP_DigestSign(md, sig_out, &slen, msg, len) == 1 && slen == 256;
  EVP_MD_CTX_free(md);
  EVP_PKEY_free(pkey);
  return ok;
}

int oracle_pem_modulus(const char* pem_key, uint8_t n_be_out[256]) {
  BIO* bio = BIO_new_mem_buf(pem_key, -1);
  EVP_PKEY* pkey = PEM_read_bio_PrivateKey(bio, NULL, NULL, NULL);
  if (!pkey) {
    BIO_free(bio);
    bio = BIO_new_mem_buf(pem_key, -1);
    pkey = PEM_read_bio_PUBKEY(bio, NULL, NULL, NULL);
  }
  BIO_free(bio);
  if (!pkey) return 0;
  BIGNUM* n = NULL;
  int ok = EVP_PKEY_get_bn_param(pkey, OSSL_PKEY_PARAM_RSA_N, &n) == 1 && BN_num_bytes(n) == 256 &&
           BN_bn2binpad(n, n_be_out, 256) == 256;
  BN_free(n);
  EVP_PKEY_free(pkey);
  return ok;
}

/* ------------------------------------------------------------------------ */
/* a5: ClusterConfiguration.getServerMajority — ClusterConfiguration.java:264-267 */
/* ------------------------------------------------------------------------ */
uint32_t oracle_server_majority(uint32_t replication_factor) {
  const uint32_t f = replication_factor / 3; /* final int f = getReplicationFactor() / 3; */
  return 2 * f + 1;                          /* return 2 * f + 1; */
}

/* ------------------------------------------------------------------------ */
/* Signature leg (CPU baseline): pthreads over grant ranges.                  */
/* ------------------------------------------------------------------------ */

typedef struct {
  const mochi_batch* batch;
  EVP_PKEY** keys;
  uint32_t n_keys;
  uint32_t begin, end;
  uint8_t* flags;
  int64_t* ts;
} sig_job;

/* One EVP_PKEY_CTX per (thread, key), initialised once for RSASSA-PKCS1-v1_5
 * with SHA-256; per grant: one SHA-256 and one EVP_PKEY_verify.  This is the
 * cheapest OpenSSL 3 path (EVP_DigestVerifyInit per grant re-fetches the
 * provider algorithms and costs ~4x more), so the CPU baseline is not a straw man. */
static EVP_PKEY_CTX* verify_ctx(EVP_PKEY* key) {
  EVP_PKEY_CTX* c = EVP_PKEY_CTX_new(key, NULL);
  if (!c) return NULL;
  if (EVP_PKEY_verify_init(c) <= 0 || EVP_PKEY_CTX_set_rsa_padding(c, RSA_PKCS1_PADDING) <= 0 ||
      EVP_PKEY_CTX_set_signature_md(c, EVP_sha256()) <= 0) {
    EVP_PKEY_CTX_free(c);
    return NULL;
  }
  return c;
}

static void* sig_worker(void* arg) {
  sig_job* j = (sig_job*)arg;
  const mochi_batch* b = j->batch;
  /* per-thread key objects, digest and contexts: OpenSSL 3 serialises threads
   * that share EVP_PKEY / implicitly fetched EVP_MD objects */
  EVP_PKEY_CTX** ctxs = (EVP_PKEY_CTX**)calloc(j->n_keys ? j->n_keys : 1, sizeof(EVP_PKEY_CTX*));
  EVP_PKEY** mykeys = (EVP_PKEY**)calloc(j->n_keys ? j->n_keys : 1, sizeof(EVP_PKEY*));
  EVP_MD* sha = EVP_MD_fetch(NULL, "SHA256", NULL);
  EVP_MD_CTX* mdc = EVP_MD_CTX_new();
  for (uint32_t i = j->begin; i < j->end; i++) {
    const uint8_t* g = b->grant_bytes + b->grant_off[i];
    const uint32_t gl = b->grant_len[i];
    oracle_grant_view v;
    uint8_t f = 0;
    int64_t ts = 0;
    if (oracle_grant_parse(g, gl, &v)) {
      f |= MOCHI_GRANT_PARSED;
      ts = v.timestamp;
    }
    const uint16_t s = b->signer[i];
    if (s < j->n_keys) {
      if (!ctxs[s]) {
        unsigned char nbe[256];
        BIGNUM* nbn = NULL;
        if (EVP_PKEY_get_bn_param(j->keys[s], OSSL_PKEY_PARAM_RSA_N, &nbn) == 1 && BN_bn2binpad(nbn, nbe, 256) == 256)
          mykeys[s] = make_pubkey(nbe);
        BN_free(nbn);
        if (mykeys[s]) ctxs[s] = verify_ctx(mykeys[s]);
      }
      uint8_t md[32];
      unsigned int mdlen = 32;
      if (ctxs[s] && EVP_DigestInit_ex(mdc, sha, NULL) == 1 && EVP_DigestUpdate(mdc, g, gl) == 1 &&
          EVP_DigestFinal_ex(mdc, md, &mdlen) == 1 && EVP_PKEY_verify(ctxs[s], b->sig + (size_t)i * 256, 256, md, 32) == 1)
        f |= MOCHI_GRANT_SIG_OK;
    }
    j->flags[i] = f;
    if (j->ts) j->ts[i] = ts;
  }
  for (uint32_t k = 0; k < j->n_keys; k++) {
    EVP_PKEY_CTX_free(ctxs[k]);
    EVP_PKEY_free(mykeys[k]);
  }
  free(ctxs);
  free(mykeys);
  EVP_MD_CTX_free(mdc);
  EVP_MD_free(sha);
  return NULL;
}

int oracle_verify_grants(const uint8_t* moduli_be, uint32_t n_keys, const mochi_batch* batch, uint32_t begin,
                         uint32_t end, uint8_t* grant_flags, int64_t* grant_ts, int n_threads) {
  if (!batch || begin > end || end > batch->n_grants || !grant_flags) return MOCHI_EINVAL;
  EVP_PKEY** keys = (EVP_PKEY**)calloc(n_keys ? n_keys : 1, sizeof(EVP_PKEY*));
  for (uint32_t k = 0; k < n_keys; k++) {
    keys[k] = make_pubkey(moduli_be + (size_t)k * 256);
    if (!keys[k]) {
      for (uint32_t q = 0; q < k; q++) EVP_PKEY_free(keys[q]);
      free(keys);
      return MOCHI_EINVAL;
    }
  }
  if (n_threads < 1) n_threads = 1;
  pthread_t* th = (pthread_t*)calloc((size_t)n_threads, sizeof(pthread_t));
  sig_job* jobs = (sig_job*)calloc((size_t)n_threads, sizeof(sig_job));
  const uint32_t n = end - begin;
  for (int t = 0; t < n_threads; t++) {
    jobs[t].batch = batch;
    jobs[t].keys = keys;
    jobs[t].n_keys = n_keys;
    jobs[t].begin = begin + (uint32_t)((uint64_t)n * t / n_threads);
    jobs[t].end = begin + (uint32_t)((uint64_t)n * (t + 1) / n_threads);
    jobs[t].flags = grant_flags;
    jobs[t].ts = grant_ts;
  }
  if (n_threads == 1) {
    sig_worker(&jobs[0]);
  } else {
    for (int t = 0; t < n_threads; t++) pthread_create(&th[t], NULL, sig_worker, &jobs[t]);
    for (int t = 0; t < n_threads; t++) pthread_join(th[t], NULL);
  }
  for (uint32_t k = 0; k < n_keys; k++) EVP_PKEY_free(keys[k]);
  free(keys);
  free(th);
  free(jobs);
  return MOCHI_OK;
}

/* Parse leg only (no signatures): MOCHI_GRANT_PARSED and Grant.timestamp of
 * grants [begin, end) by oracle_grant_parse, so a large batch's tally can be
 * checked against the oracle's own parse without re-verifying every signature. */
int oracle_parse_grants(const mochi_batch* b, uint32_t begin, uint32_t end, uint8_t* grant_flags, int64_t* grant_ts) {
  if (!b || begin > end || end > b->n_grants || !grant_flags || !grant_ts) return MOCHI_EINVAL;
  for (uint32_t i = begin; i < end; i++) {
    oracle_grant_view v;
    const int ok = oracle_grant_parse(b->grant_bytes + b->grant_off[i], b->grant_len[i], &v);
    grant_flags[i] = ok ? MOCHI_GRANT_PARSED : 0;
    grant_ts[i] = ok ? v.timestamp : 0;
  }
  return MOCHI_OK;
}

/* ------------------------------------------------------------------------ */
/* a3 + a4: the certificate verdict                                           */
/* ------------------------------------------------------------------------ */

static int hash_equals(const uint8_t* g, uint32_t glen, const uint8_t expected[MOCHI_TXN_HASH_BYTES]) {
  oracle_grant_view v;
  if (!oracle_grant_parse(g, glen, &v)) return 0;
  /* grantForObject.getTransactionHash().equals(txnHash): String equality; both
   * valid UTF-8, so byte equality of the encodings. */
  return v.txn_hash_len == MOCHI_TXN_HASH_BYTES && memcmp(g + v.txn_hash_off, expected, MOCHI_TXN_HASH_BYTES) == 0;
}

/* MOCHI_Q_BIND: Grant.objectId == the op key it is filed under, and
 * Grant.transactionHash == objectSHA512(txn). */
static int grant_bound(const mochi_batch* b, uint32_t g, uint32_t op, const uint8_t* expected) {
  oracle_grant_view v;
  const uint8_t* gb = b->grant_bytes + b->grant_off[g];
  if (!oracle_grant_parse(gb, b->grant_len[g], &v)) return 0;
  if (!b->op_key_off || !b->op_key_len) return 0;
  const uint32_t kl = b->op_key_len[op];
  if (v.object_id_len != kl || memcmp(gb + v.object_id_off, b->grant_bytes + b->op_key_off[op], kl) != 0) return 0;
  return hash_equals(gb, b->grant_len[g], expected);
}

/* MultiGrant index (certificate-relative) of every grant of certificate c:
 * explicit CSR (cert_mg_off / mg_grant_off) or, without it, one MultiGrant per
 * maximal run of equal signers.  Returns the MultiGrant count. */
static uint32_t cert_multigrants(const mochi_batch* b, uint32_t c, uint32_t* mg_of /* [g_hi - g_lo] */) {
  const uint32_t g_lo = b->cert_grant_off[c], g_hi = b->cert_grant_off[c + 1];
  if (b->cert_mg_off && b->mg_grant_off) {
    const uint32_t m_lo = b->cert_mg_off[c], m_hi = b->cert_mg_off[c + 1];
    for (uint32_t m = m_lo; m < m_hi; m++)
      for (uint32_t g = b->mg_grant_off[m]; g < b->mg_grant_off[m + 1]; g++) mg_of[g - g_lo] = m - m_lo;
    return m_hi - m_lo;
  }
  uint32_t n = 0;
  for (uint32_t g = g_lo; g < g_hi; g++) {
    if (g == g_lo || b->signer[g] != b->signer[g - 1]) n++;
    mg_of[g - g_lo] = n - 1;
  }
  return n;
}

/* StoreValueObjectContainer.getCurrentTimestampFromCurrentCertificate (:175-198)
 * on the INCOMING certificate, as applyOperation calls it after setCurrentC(wc)
 * (InMemoryDataStore.java:533-534):
 *   for (multiGrant : currentC.grants.values())                 -- every MultiGrant
 *     grant = multiGrant.grants.get(key)
 *     Utils.assertNotNull(grant, ...)                          -- :186 -> IllegalStateException
 *     if (timestamp == null) timestamp = grant.ts
 *     else if (timestamp != grant.ts) throw IllegalStateException  -- :192-194
 * Signatures play no part: the Java loop sees the certificate as received.
 * Returns 1 and the timestamp, or 0 (throws). */
static int incoming_cert_ts(const mochi_batch* b, uint32_t c, uint32_t slot, const int64_t* grant_ts,
                            const uint32_t* mg_of, uint32_t n_mg, int64_t* ts_out) {
  const uint32_t g_lo = b->cert_grant_off[c], g_hi = b->cert_grant_off[c + 1];
  int have = 0;
  int64_t ts = 0;
  for (uint32_t m = 0; m < n_mg; m++) {
    int found = 0;
    for (uint32_t g = g_lo; g < g_hi; g++) {
      if (mg_of[g - g_lo] != m || b->grant_key[g] != slot) continue;
      found = 1;
      if (!have) {
        have = 1;
        ts = grant_ts[g];
      } else if (grant_ts[g] != ts) {
        return 0;
      }
    }
    if (!found) return 0;
  }
  if (!have) return 0; /* no MultiGrant at all: the Long is null and `long timestamp = ...` unboxes it (NPE) */
  *ts_out = ts;
  return 1;
}

int oracle_tally(const mochi_batch* b, const mochi_params* p, const uint8_t* grant_flags, const int64_t* grant_ts,
                 mochi_verdicts* out) {
  if (!b || !p || !grant_flags || !grant_ts || !out || !out->cert_accept_bits) return MOCHI_EINVAL;
  const uint32_t M = oracle_server_majority(p->replication_factor);
  memset(out->cert_accept_bits, 0, ((size_t)b->n_certs + 31) / 32 * 4);
  uint32_t* mg_of = NULL;
  size_t mg_cap = 0;
  uint8_t* counted = NULL;
  size_t cnt_cap = 0;
  for (uint32_t c = 0; c < b->n_certs; c++) {
    const uint32_t g_lo = b->cert_grant_off[c], g_hi = b->cert_grant_off[c + 1];
    const uint32_t o_lo = b->cert_op_off[c], o_hi = b->cert_op_off[c + 1];
    const uint32_t n_ops = o_hi - o_lo, n_g = g_hi - g_lo;
    const uint8_t* expected = b->expected_hash + (size_t)c * MOCHI_TXN_HASH_BYTES;
    uint8_t reason = MOCHI_ACCEPT, fail_op = 0xFF;
    if (n_g > mg_cap) {
      mg_cap = n_g * 2;
      mg_of = (uint32_t*)realloc(mg_of, mg_cap * sizeof *mg_of);
    }
    if (n_g > cnt_cap) {
      cnt_cap = n_g * 2;
      counted = (uint8_t*)realloc(counted, cnt_cap);
    }
    const uint32_t n_mg = cert_multigrants(b, c, mg_of);

    /* Malformed grant bytes: the reference fails in the protobuf decoder
     * before any of the protocol code runs (MochiServerInitializer.java:30-34). */
    for (uint32_t g = g_lo; g < g_hi && reason == MOCHI_ACCEPT; g++)
      if (!(grant_flags[g] & MOCHI_GRANT_PARSED)) reason = MOCHI_REJECT_MALFORMED;

    /* multiplicity of each key slot = number of txn ops naming that key;
     * first_op[s] = the first op naming slot s (its operand1 is the key) */
    uint32_t mult[MOCHI_MAX_OPS_PER_CERT], first_op[MOCHI_MAX_OPS_PER_CERT];
    memset(mult, 0, sizeof mult);
    for (uint32_t o = o_hi; o-- > o_lo;) {
      mult[b->op_key[o]]++;
      first_op[b->op_key[o]] = o;
    }

    /* Which grants count.  Reference parity (quorum_mode 0): a grant counts iff
     * its signature verified ("invalid signature => absent", the null skip at
     * InMemoryDataStore.java:622-624) and an op names its key.  MOCHI_Q_BIND /
     * MOCHI_Q_DISTINCT_SIGNERS exclude more grants the same way. */
    for (uint32_t g = g_lo; g < g_hi; g++) {
      const uint32_t s = b->grant_key[g];
      int ok = (grant_flags[g] & MOCHI_GRANT_SIG_OK) && s < MOCHI_MAX_OPS_PER_CERT && mult[s] != 0;
      if (ok && (p->quorum_mode & MOCHI_Q_BIND)) ok = grant_bound(b, g, first_op[s], expected);
      if (ok && (p->quorum_mode & MOCHI_Q_DISTINCT_SIGNERS))
        for (uint32_t q = g_lo; q < g && ok; q++)
          if (counted[q - g_lo] && b->grant_key[q] == s && b->signer[q] == b->signer[g]) ok = 0;
      counted[g - g_lo] = (uint8_t)ok;
    }

    /* processMultiGrantsFromAllServers  InMemoryDataStore.java:613-640
     *   for (multiGrant : wc.grants.values())            -- wire order
     *     for (op : transaction.operations)              -- txn order
     *       grant = multiGrant.grants.get(op.operand1)   -- (not counted => absent)
     *       if (grant == null) continue;                 -- :622-624
     *       if (coalesced.containsKey(key)) {
     *         if (coalesced[key].ts != grant.ts) throw UnsupportedOperationException  -- :626-628
     *         coalesced[key].list.add(grant)             -- :629
     *       } else coalesced.put(key, (grant.ts, [grant])) -- :631-634
     * A grant for key slot s is appended once per op naming s (mult[s] times);
     * its own comparisons against ts0 all agree, so only the first sighting
     * per slot matters for ts0 and g0. */
    int seen[MOCHI_MAX_OPS_PER_CERT];
    int64_t ts0[MOCHI_MAX_OPS_PER_CERT];
    uint32_t cnt[MOCHI_MAX_OPS_PER_CERT], first[MOCHI_MAX_OPS_PER_CERT];
    memset(seen, 0, sizeof seen);
    memset(cnt, 0, sizeof cnt);
    int ts_bad = 0;
    for (uint32_t g = g_lo; g < g_hi; g++) {
      if (!counted[g - g_lo]) continue;
      const uint32_t s = b->grant_key[g];
      if (!seen[s]) {
        seen[s] = 1;
        ts0[s] = grant_ts[g];
        first[s] = g;
        cnt[s] = mult[s];
      } else {
        if (ts0[s] != grant_ts[g]) ts_bad = 1;
        cnt[s] += mult[s];
      }
    }
    if (reason == MOCHI_ACCEPT && ts_bad) reason = MOCHI_REJECT_TS_MISMATCH;

    /* write2apply  InMemoryDataStore.java:576-611, ops in txn order */
    uint8_t decision[MOCHI_MAX_OPS_PER_CERT];
    memset(decision, MOCHI_OPD_SKIPPED, sizeof decision);
    int applied[MOCHI_MAX_OPS_PER_CERT]; /* slot s applied earlier in this txn: SVOC.currentC == wc */
    memset(applied, 0, sizeof applied);
    for (uint32_t j = 0; j < n_ops && reason == MOCHI_ACCEPT; j++) {
      const uint32_t o = o_lo + j;
      const uint8_t fl = b->op_flags[o];
      if (!(fl & MOCHI_OP_LOCAL)) { /* WRONG_SHARD result  :582-587 */
        decision[j] = MOCHI_OPD_WRONG_SHARD;
        continue;
      }
      const uint32_t s = b->op_key[o];
      uint8_t why = MOCHI_ACCEPT;
      if (!seen[s]) why = MOCHI_REJECT_NO_GRANT; /* coalescedTxnGrantMap.get(key) == null -> NPE  :588 */
      /* Utils.assertTrue(list.size() > getServerMajority())  :590 (client: >=) */
      else if (!(p->strict_gt ? (cnt[s] > M) : (cnt[s] >= M))) why = MOCHI_REJECT_BELOW_QUORUM;
      /* if (grantForObject.getTransactionHash().equals(txnHash)) ... else throw  :591,605-607 */
      else if (!hash_equals(b->grant_bytes + b->grant_off[first[s]], b->grant_len[first[s]], expected))
        why = MOCHI_REJECT_HASH_MISMATCH;
      /* storeValueContainer = getDataMap(key).get(key); op.getOperand1().equals(svoc.getKey()) -> NPE if null  :592-593 */
      else if (!(fl & MOCHI_OP_HAS_SVOC)) why = MOCHI_REJECT_NO_SVOC;
      if (why == MOCHI_ACCEPT) {
        /* Long objectTS = svoc.getCurrentTimestampFromCurrentCertificate()  :594 -- on the
         * stored certificate: wc itself once an earlier op of this txn applied to this key */
        const int has_cc = applied[s] || (fl & MOCHI_OP_HAS_CURRENT_C);
        const int cc_bad = !applied[s] && (fl & MOCHI_OP_CURRENT_C_BAD);
        const int64_t g0_ts = grant_ts[first[s]];
        const int64_t obj_ts = applied[s] ? g0_ts : (b->op_object_ts ? b->op_object_ts[o] : 0);
        if (cc_bad) {
          why = MOCHI_REJECT_STORED_CERT;
        } else {
          /* if (objectTS != null && objectTS > g0.getTimestamp()) readOperation else applyOperation  :595-599;
           * both first check the write lock and the action (:525-529 / :560-562, :551 / :572) */
          const int read = has_cc && obj_ts > g0_ts;
          int64_t t_in;
          if (fl & MOCHI_OP_NOT_WRITE) why = MOCHI_REJECT_NOT_WRITE;
          else if (read) decision[j] = MOCHI_OPD_READ;
          /* applyOperation: setCurrentC(wc); getCurrentTimestampFromCurrentCertificate()  :533-534 */
          else if (!incoming_cert_ts(b, c, s, grant_ts, mg_of, n_mg, &t_in)) why = MOCHI_REJECT_APPLY_STATE;
          else {
            decision[j] = MOCHI_OPD_APPLY;
            applied[s] = 1; /* t_in == g0_ts: g0 is one of the grants the check compared */
          }
        }
      }
      if (why != MOCHI_ACCEPT) {
        reason = why;
        fail_op = (uint8_t)j;
        decision[j] = MOCHI_OPD_FAILED;
      }
    }

    if (reason == MOCHI_ACCEPT) out->cert_accept_bits[c >> 5] |= 1u << (c & 31);
    if (out->cert_reason) out->cert_reason[c] = reason;
    if (out->cert_fail_op) out->cert_fail_op[c] = fail_op;
    for (uint32_t j = 0; j < n_ops; j++) {
      const uint32_t o = o_lo + j, s = b->op_key[o];
      if (out->op_decision) out->op_decision[o] = decision[j];
      if (out->op_g0) out->op_g0[o] = seen[s] ? first[s] - g_lo : 0xFFFFFFFFu;
      if (out->op_ts) out->op_ts[o] = seen[s] ? grant_ts[first[s]] : 0;
    }
  }
  free(mg_of);
  free(counted);
  return MOCHI_OK;
}

int oracle_verify_batch(const uint8_t* moduli_be, uint32_t n_keys, const mochi_batch* batch,
                        const mochi_params* params, mochi_verdicts* out, int n_threads) {
  if (!batch || !params || !out) return MOCHI_EINVAL;
  const uint32_t N = batch->n_grants;
  uint8_t* flags = out->grant_flags ? out->grant_flags : (uint8_t*)malloc(N ? N : 1);
  int64_t* ts = out->grant_ts ? out->grant_ts : (int64_t*)malloc(sizeof(int64_t) * (N ? N : 1));
  int rc = oracle_verify_grants(moduli_be, n_keys, batch, 0, N, flags, ts, n_threads);
  if (rc == MOCHI_OK) {
    if (out->grant_valid_bits) {
      memset(out->grant_valid_bits, 0, ((size_t)N + 31) / 32 * 4);
      for (uint32_t i = 0; i < N; i++)
        if (flags[i] & MOCHI_GRANT_SIG_OK) out->grant_valid_bits[i >> 5] |= 1u << (i & 31);
    }
    rc = oracle_tally(batch, params, flags, ts, out);
  }
  if (!out->grant_flags) free(flags);
  if (!out->grant_ts) free(ts);
  return rc;
}

/* ------------------------------------------------------------------------ */
/* a8: MochiDBClient.isUniformTimeStampInMultiGrants — MochiDBClient.java:195-219 */
/* ------------------------------------------------------------------------ */
int oracle_write1_uniform(uint32_t n_grants, const uint8_t* grant_key, const int64_t* ts) {
  int seen[256] = {0};
  int64_t ts0[256];
  for (uint32_t g = 0; g < n_grants; g++) {
    const uint8_t s = grant_key[g];
    if (!seen[s]) { /* coalescedTxnGrantMap.put(key, (ts, grant))  :212-214 */
      seen[s] = 1;
      ts0[s] = ts[g];
    } else if (ts0[s] != ts[g]) { /* != timestampFromGrant -> return false  :208-210 */
      return 0;
    }
  }
  return 1;
}

/* ------------------------------------------------------------------------ */
/* a8 + a9: client Write1 round — MochiDBClient.java:236-332                   */
/* ------------------------------------------------------------------------ */
int oracle_write1_classify(uint32_t n_requests, const uint32_t* resp_off, const uint8_t* resp_kind,
                           const uint32_t* resp_server, const uint32_t* resp_grant_off, const uint8_t* grant_key,
                           const int64_t* grant_ts, const uint8_t* grant_status, uint8_t* decision) {
  if (!resp_off || !resp_kind || !resp_server || !resp_grant_off || !decision) return MOCHI_EINVAL;
  for (uint32_t r = 0; r < n_requests; r++) {
    const uint32_t q0 = resp_off[r], q1 = resp_off[r + 1];
    int all_ok = 1, d = -1;
    /* :274-290 response loop: REQUESTFAILED throws on the spot */
    for (uint32_t q = q0; q < q1; q++) {
      if (resp_kind[q] != MOCHI_W1_OK) all_ok = 0;
      if (resp_kind[q] == MOCHI_W1_REQUEST_FAILED) {
        d = MOCHI_W1_THROW_FAILED; /* :281-283 */
        break;
      }
    }
    /* :295-307 multigrant maps; removeWrongShardGrantFromMultiGrant removes from
     * the read-only protobuf map view -> UnsupportedOperationException (:221-228) */
    for (uint32_t q = q0; q < q1 && d < 0; q++) {
      if (resp_kind[q] != MOCHI_W1_OK && resp_kind[q] != MOCHI_W1_REFUSED) continue;
      for (uint32_t g = resp_grant_off[q]; g < resp_grant_off[q + 1]; g++)
        if (grant_status[g] == 1 /* WRONG_SHARD */) {
          d = MOCHI_W1_THROW_UNSUPPORTED;
          break;
        }
    }
    if (d < 0) {
      /* :310 isUniformTimeStampInMultiGrants over write1mutiGrants: one entry per
       * serverId, the last OK response with that id wins (HashMap.put, :299) */
      int seen[256] = {0};
      int64_t ts0[256];
      int uniform = 1;
      for (uint32_t q = q0; q < q1 && uniform; q++) {
        if (resp_kind[q] != MOCHI_W1_OK) continue;
        int superseded = 0;
        for (uint32_t p = q + 1; p < q1; p++)
          if (resp_kind[p] == MOCHI_W1_OK && resp_server[p] == resp_server[q]) superseded = 1;
        if (superseded) continue;
        for (uint32_t g = resp_grant_off[q]; g < resp_grant_off[q + 1] && uniform; g++) {
          const uint8_t k = grant_key[g];
          if (k == 0xFF) continue; /* allGrants.get(op.getOperand1()) never reaches it :202-205 */
          if (!seen[k]) {
            seen[k] = 1;
            ts0[k] = grant_ts[g]; /* :212-214 */
          } else if (ts0[k] != grant_ts[g]) {
            uniform = 0; /* :208-210 */
          }
        }
      }
      if (!uniform) d = MOCHI_W1_RETRY;                          /* :310-318 */
      else d = all_ok ? MOCHI_W1_PROCEED : MOCHI_W1_THROW_REFUSED; /* :320-328 */
    }
    decision[r] = (uint8_t)d;
  }
  return MOCHI_OK;
}

/* ------------------------------------------------------------------------ */
/* a10: client Read / Write2 aggregation — MochiDBClient.java:148-175, 355-382 */
/* ------------------------------------------------------------------------ */
int oracle_tally_responses(uint32_t n_requests, const uint32_t* resp_off, const uint32_t* n_ops,
                           const uint32_t* resp_n_ops, const uint64_t* status_off, const uint8_t* status,
                           const uint64_t* chosen_off, uint32_t replication_factor, int32_t* chosen,
                           uint8_t* reason, uint32_t* accept_bits) {
  if (!resp_off || !n_ops || !resp_n_ops || !status_off || !status || !chosen_off || !accept_bits)
    return MOCHI_EINVAL;
  const uint32_t M = oracle_server_majority(replication_factor);
  memset(accept_bits, 0, ((size_t)n_requests + 31) / 32 * 4);
  for (uint32_t r = 0; r < n_requests; r++) {
    const uint32_t k = n_ops[r];
    int32_t* ch = chosen ? chosen + chosen_off[r] : NULL;
    uint32_t cnt[MOCHI_MAX_OPS_PER_CERT];
    if (k > MOCHI_MAX_OPS_PER_CERT) return MOCHI_EINVAL;
    for (uint32_t j = 0; j < k; j++) { /* consistentTRCount[index] = 0; coalescedResult.add(null)  :150-155 / :357-362 */
      cnt[j] = 0;
      if (ch) ch[j] = -1;
    }
    uint8_t why = 0;
    for (uint32_t q = resp_off[r]; q < resp_off[r + 1] && !why; q++) {
      if (resp_n_ops[q] != k) { /* operations.size() != transactionOps.size() -> Inconsistent*Exception  :159-161 / :366-368 */
        why = 1;
        break;
      }
      const uint8_t* st = status + status_off[q];
      for (uint32_t j = 0; j < k; j++) {
        if (st[j] != 1 /* WRONG_SHARD */) { /* :164-167 / :371-374 */
          cnt[j]++;
          if (ch) ch[j] = (int32_t)(q - resp_off[r]);
        }
      }
    }
    for (uint32_t j = 0; j < k && !why; j++)
      if (cnt[j] < M) why = 2; /* consistentTRCount[index] < getServerMajority() -> throw  :171-175 / :378-381 */
    if (reason) reason[r] = why;
    if (!why) accept_bits[r >> 5] |= 1u << (r & 31);
  }
  return MOCHI_OK;
}

/* ------------------------------------------------------------------------ */
/* Write2ToServer wire decode (MochiProtocol.proto:107-147 + the proposed    */
/* MultiGrant.grantSignatures = 5), protobuf-java 3.16.3 semantics:           */
/*   - generated parsers (MochiProtocol.java Write2ToServer / WriteCertificate */
/*     / MultiGrant / Transaction / Operation constructors) take the LAST      */
/*     value of a singular scalar/string field, MERGE repeated occurrences of  */
/*     a singular message field, and skip unknown fields (parseUnknownField);  */
/*   - map fields: each entry is parsed by MapEntryLite.parseEntry (key and    */
/*     value last-wins, message values merged, unknown fields skipped) and     */
/*     put into MapField's LinkedHashMap: a repeated key keeps its FIRST       */
/*     position and takes the LAST value;                                      */
/*   - proto3 string fields and string map keys require valid UTF-8;          */
/*   - any malformation fails the whole message (InvalidProtocolBufferException).*/
/* The device decoder's fast path (include/mochi_hip.h, MOCHI_MSG_FALLBACK)   */
/* is restated here too, so the two agree message by message.                 */
/* ------------------------------------------------------------------------ */

typedef struct {
  uint32_t field, wt;
  uint64_t v;
  size_t off, len; /* wt 2 payload */
} fld_t;

static int skip_group(rd_t* r, uint32_t field, int depth) {
  if (depth > ORACLE_MAX_GROUP_DEPTH) return 0;
  for (;;) {
    uint64_t t64, v;
    if (!rd_varint(r, &t64)) return 0; /* truncated inside the group */
    const uint32_t t = (uint32_t)t64, f = t >> 3, wt = t & 7;
    if (f == 0) return 0;
    switch (wt) {
      case 0: if (!rd_varint(r, &v)) return 0; break;
      case 1: if (r->len - r->pos < 8) return 0; r->pos += 8; break;
      case 2: {
        if (!rd_varint(r, &v)) return 0;
        const int32_t l = (int32_t)(uint32_t)v;
        if (l < 0 || (uint64_t)l > r->len - r->pos) return 0;
        r->pos += (size_t)l;
        break;
      }
      case 3: if (!skip_group(r, f, depth + 1)) return 0; break;
      case 4: return f == field; /* checkLastTagWas(END_GROUP of this field) */
      case 5: if (r->len - r->pos < 4) return 0; r->pos += 4; break;
      default: return 0;
    }
  }
}

/* Next field of the message being read: 1 field, 0 end, -1 malformed. */
static int next_fld(rd_t* r, fld_t* f) {
  if (r->pos >= r->len) return 0;
  uint64_t t64;
  if (!rd_varint(r, &t64)) return -1;
  const uint32_t t = (uint32_t)t64;
  f->field = t >> 3;
  f->wt = t & 7;
  f->off = f->len = 0;
  f->v = 0;
  if (f->field == 0) return -1;
  switch (f->wt) {
    case 0: return rd_varint(r, &f->v) ? 1 : -1;
    case 1: if (r->len - r->pos < 8) return -1; r->pos += 8; return 1;
    case 2: {
      uint64_t l;
      if (!rd_varint(r, &l)) return -1;
      const int32_t l32 = (int32_t)(uint32_t)l;
      if (l32 < 0 || (uint64_t)l32 > r->len - r->pos) return -1;
      f->off = r->pos;
      f->len = (size_t)l32;
      r->pos += (size_t)l32;
      return 1;
    }
    case 3: return skip_group(r, f->field, 1) ? 1 : -1;
    case 5: if (r->len - r->pos < 4) return -1; r->pos += 4; return 1;
    default: return -1; /* END_GROUP at message level, wire types 6, 7 */
  }
}

#define FOR_FIELDS(buf, o, l, f, rc)                                   \
  for (rd_t r_ = {(buf) + (o), (l), 0}; (rc = next_fld(&r_, &f)) > 0;)

/* --- full validity (what protobuf-java's parser checks) --- */
static int valid_str(const uint8_t* m, const fld_t* f) { return valid_utf8(m + f->off, f->len); }

static int valid_grant_msg(const uint8_t* m, size_t off, size_t len) {
  oracle_grant_view v;
  return oracle_grant_parse(m + off, len, &v);
}

/* map entry with a string key; value validated by `val` (NULL: bytes) */
static int valid_entry(const uint8_t* m, size_t off, size_t len, int (*val)(const uint8_t*, size_t, size_t)) {
  fld_t f;
  int rc;
  FOR_FIELDS(m, off, len, f, rc) {
    if (f.field == 1 && f.wt == 2 && !valid_str(m + off, &f)) return 0;
    if (f.field == 2 && f.wt == 2 && val && !val(m + off, f.off, f.len)) return 0;
  }
  return rc == 0;
}

static int valid_multigrant(const uint8_t* m, size_t off, size_t len) {
  fld_t f;
  int rc;
  FOR_FIELDS(m, off, len, f, rc) {
    if (f.wt != 2) continue;
    if (f.field == 1 && !valid_entry(m + off, f.off, f.len, valid_grant_msg)) return 0;
    if ((f.field == 2 || f.field == 3 || f.field == 4) && !valid_str(m + off, &f)) return 0;
    if (f.field == 5 && !valid_entry(m + off, f.off, f.len, NULL)) return 0;
  }
  return rc == 0;
}

static int valid_wc(const uint8_t* m, size_t off, size_t len) {
  fld_t f;
  int rc;
  FOR_FIELDS(m, off, len, f, rc)
    if (f.field == 1 && f.wt == 2 && !valid_entry(m + off, f.off, f.len, valid_multigrant)) return 0;
  return rc == 0;
}

static int valid_operation(const uint8_t* m, size_t off, size_t len) {
  fld_t f;
  int rc;
  FOR_FIELDS(m, off, len, f, rc)
    if (f.field >= 2 && f.field <= 4 && f.wt == 2 && !valid_str(m + off, &f)) return 0;
  return rc == 0;
}

static int valid_txn(const uint8_t* m, size_t off, size_t len) {
  fld_t f;
  int rc;
  FOR_FIELDS(m, off, len, f, rc)
    if (f.field == 1 && f.wt == 2 && !valid_operation(m + off, f.off, f.len)) return 0;
  return rc == 0;
}

static int valid_write2(const uint8_t* m, size_t len) {
  fld_t f;
  int rc;
  FOR_FIELDS(m, 0, len, f, rc) {
    if (f.field == 1 && f.wt == 2 && !valid_wc(m, f.off, f.len)) return 0;
    if (f.field == 2 && f.wt == 2 && !valid_txn(m, f.off, f.len)) return 0;
  }
  return rc == 0;
}

/* --- extraction on a valid message --- */
typedef struct {
  size_t koff, klen; /* key (default "") */
  size_t voff, vlen; /* last value occurrence (default empty) */
  int nval;          /* value occurrences */
} entry_t;

static void read_entry(const uint8_t* m, size_t off, size_t len, entry_t* e) {
  fld_t f;
  int rc;
  memset(e, 0, sizeof *e);
  FOR_FIELDS(m, off, len, f, rc) {
    if (f.wt != 2) continue;
    if (f.field == 1) {
      e->koff = off + f.off;
      e->klen = f.len;
    } else if (f.field == 2) {
      e->voff = off + f.off;
      e->vlen = f.len;
      e->nval++;
    }
  }
}

static int same(const uint8_t* m, size_t a, size_t al, size_t b, size_t bl) {
  return al == bl && memcmp(m + a, m + b, al) == 0;
}

/* entries of map field `field` in [off, off+len): LinkedHashMap put order.
 * Returns the number of entries (all of them, before de-duplication). */
static size_t list_entries(const uint8_t* m, size_t off, size_t len, uint32_t field, entry_t** out) {
  size_t n = 0, cap = 8;
  entry_t* v = (entry_t*)malloc(cap * sizeof *v);
  fld_t f;
  int rc;
  FOR_FIELDS(m, off, len, f, rc) {
    if (f.field != field || f.wt != 2) continue;
    if (n == cap) v = (entry_t*)realloc(v, (cap *= 2) * sizeof *v);
    read_entry(m, off + f.off, f.len, &v[n++]);
  }
  *out = v;
  return n;
}

/* index of the entry holding key i's final value, or -1 if i is not the first occurrence */
static long map_slot(const uint8_t* m, const entry_t* e, size_t n, size_t i) {
  for (size_t j = 0; j < i; j++)
    if (same(m, e[j].koff, e[j].klen, e[i].koff, e[i].klen)) return -1;
  size_t last = i;
  for (size_t j = i + 1; j < n; j++)
    if (same(m, e[j].koff, e[j].klen, e[i].koff, e[i].klen)) last = j;
  return (long)last;
}

static void last_string(const uint8_t* m, size_t off, size_t len, uint32_t field, size_t* so, size_t* sl) {
  fld_t f;
  int rc;
  *so = 0;
  *sl = 0;
  FOR_FIELDS(m, off, len, f, rc)
    if (f.field == field && f.wt == 2) {
      *so = off + f.off;
      *sl = f.len;
    }
}

/* Grant bytes equal to what Grant.toByteArray() gives for the parsed Grant. */
static int grant_canonical(const uint8_t* g, size_t len) {
  oracle_grant_view v;
  if (!oracle_grant_parse(g, len, &v)) return 0;
  uint8_t buf[1024];
  if (len > sizeof buf) return 0;
  const long n = oracle_grant_encode((const char*)g + v.object_id_off, v.object_id_len, v.timestamp, v.configstamp,
                                     (const char*)g + v.txn_hash_off, v.txn_hash_len, v.status, buf, sizeof buf);
  return n == (long)len && memcmp(buf, g, len) == 0;
}

#define W2_MAX_MULTIGRANTS 32
#define W2_MAX_GRANTS_PER_MG 64

typedef struct {
  uint32_t n; /* grants emitted so far */
  uint32_t cap;
  uint64_t* off;
  uint32_t* len;
  uint8_t* sig;
  uint16_t* signer;
  uint8_t* key;
} gout_t;

static void gout_push(gout_t* o, uint64_t off, uint32_t len, const uint8_t* sig, uint16_t signer, uint8_t key) {
  if (o->n == o->cap) {
    o->cap = o->cap ? o->cap * 2 : 1024;
    o->off = (uint64_t*)realloc(o->off, o->cap * sizeof(uint64_t));
    o->len = (uint32_t*)realloc(o->len, o->cap * sizeof(uint32_t));
    o->sig = (uint8_t*)realloc(o->sig, (size_t)o->cap * MOCHI_RSA_BYTES);
    o->signer = (uint16_t*)realloc(o->signer, o->cap * sizeof(uint16_t));
    o->key = (uint8_t*)realloc(o->key, o->cap);
  }
  o->off[o->n] = off;
  o->len[o->n] = len;
  if (sig) memcpy(o->sig + (size_t)o->n * MOCHI_RSA_BYTES, sig, MOCHI_RSA_BYTES);
  else memset(o->sig + (size_t)o->n * MOCHI_RSA_BYTES, 0, MOCHI_RSA_BYTES);
  o->signer[o->n] = signer;
  o->key[o->n] = key;
  o->n++;
}

/* Last value of varint field `field` (wire type 0) of [off, off+len); 0 when absent. */
static uint64_t last_varint(const uint8_t* m, size_t off, size_t len, uint32_t field) {
  fld_t f;
  int rc;
  uint64_t v = 0;
  FOR_FIELDS(m, off, len, f, rc)
    if (f.field == field && f.wt == 0) v = f.v;
  return v;
}

typedef struct {
  uint8_t key;     /* key slot: index of the first op with the same operand1 */
  uint8_t notw;    /* MOCHI_OP_NOT_WRITE derived from the message            */
  uint64_t k_off;  /* operand1 (absolute wire offset) and length            */
  uint32_t k_len;
} op_info_t;

typedef struct {
  uint32_t n, cap;
  uint32_t* cnt; /* grants per MultiGrant */
} mgout_t;

static void mg_push(mgout_t* o, uint32_t n) {
  if (o->n == o->cap) {
    o->cap = o->cap ? o->cap * 2 : 1024;
    o->cnt = (uint32_t*)realloc(o->cnt, o->cap * sizeof(uint32_t));
  }
  o->cnt[o->n++] = n;
}

/* Decode message m (valid) into grants / MultiGrants / ops; returns MOCHI_MSG_OK
 * or MOCHI_MSG_FALLBACK. */
static int decode_one(const uint8_t* m, size_t mlen, uint64_t base, const uint8_t* ids, const uint32_t* id_off,
                      uint32_t n_ids, gout_t* go, mgout_t* mo_out, op_info_t* ops, uint32_t* n_ops) {
  fld_t f;
  int rc;
  size_t wc_off = 0, wc_len = 0, tx_off = 0, tx_len = 0;
  int n_wc = 0, n_tx = 0;
  FOR_FIELDS(m, 0, mlen, f, rc) {
    if (f.field == 1 && f.wt == 2) { wc_off = f.off; wc_len = f.len; n_wc++; }
    if (f.field == 2 && f.wt == 2) { tx_off = f.off; tx_len = f.len; n_tx++; }
  }
  if (n_wc > 1 || n_tx > 1) return MOCHI_MSG_FALLBACK; /* merged singular message fields */
  /* operations, transaction order; key slot = first op with the same operand1 */
  size_t op_o[MOCHI_MAX_OPS_PER_CERT], op_l[MOCHI_MAX_OPS_PER_CERT];
  uint32_t no = 0;
  FOR_FIELDS(m, tx_off, tx_len, f, rc) {
    if (f.field != 1 || f.wt != 2) continue;
    if (no == MOCHI_MAX_OPS_PER_CERT) return MOCHI_MSG_FALLBACK;
    last_string(m, tx_off + f.off, f.len, 2, &op_o[no], &op_l[no]);
    uint32_t slot = no;
    for (uint32_t j = 0; j < no; j++)
      if (same(m, op_o[j], op_l[j], op_o[no], op_l[no])) { slot = ops[j].key; break; }
    /* Operation.action (field 1, enum; proto3 open: any value but WRITE = 2 /
     * DELETE = 1 fails applyOperation / readOperation, :529 / :562), and an empty
     * operand1 is never write-locked (getObjectsToWriteLock, :339-358) */
    const int32_t action = (int32_t)(uint32_t)last_varint(m, tx_off + f.off, f.len, 1);
    ops[no].key = (uint8_t)slot;
    ops[no].notw = (action != 1 && action != 2) || op_l[no] == 0 ? MOCHI_OP_NOT_WRITE : 0;
    ops[no].k_off = base + op_o[no];
    ops[no].k_len = (uint32_t)op_l[no];
    no++;
  }
  *n_ops = no;
  /* certificate entries: WriteCertificate.grants (serverId -> MultiGrant) */
  entry_t* ce;
  const size_t nce = list_entries(m, wc_off, wc_len, 1, &ce);
  int status = MOCHI_MSG_OK;
  const uint32_t g_start = go->n, mg_start = mo_out->n;
  /* fast path: at most 32 certificate entries on the wire (duplicates included) */
  if (nce > W2_MAX_MULTIGRANTS) status = MOCHI_MSG_FALLBACK;
  for (size_t i = 0; i < nce && status == MOCHI_MSG_OK; i++)
    if (ce[i].nval > 1) status = MOCHI_MSG_FALLBACK;
  for (size_t i = 0; i < nce && status == MOCHI_MSG_OK; i++) {
    const long s = map_slot(m, ce, nce, i);
    if (s < 0) continue;
    const size_t mo = ce[s].voff, ml = ce[s].vlen;
    size_t sid_o, sid_l;
    last_string(m, mo, ml, 4, &sid_o, &sid_l); /* MultiGrant.serverId */
    uint16_t signer = 0xFFFF;
    for (uint32_t k = 0; k < n_ids; k++)
      if (id_off[k + 1] - id_off[k] == sid_l && memcmp(ids + id_off[k], m + sid_o, sid_l) == 0) { signer = (uint16_t)k; break; }
    entry_t *ge, *se;
    const size_t nge = list_entries(m, mo, ml, 1, &ge);
    const size_t nse = list_entries(m, mo, ml, 5, &se);
    uint32_t n_g = 0;
    /* fast path: at most 64 grants and 64 grantSignatures entries on the wire
     * per decoded MultiGrant (duplicates included) */
    if (nge > W2_MAX_GRANTS_PER_MG || nse > W2_MAX_GRANTS_PER_MG) status = MOCHI_MSG_FALLBACK;
    for (size_t a = 0; a < nge && status == MOCHI_MSG_OK; a++)
      if (ge[a].nval > 1) status = MOCHI_MSG_FALLBACK;
    for (size_t a = 0; a < nge && status == MOCHI_MSG_OK; a++) {
      const long t = map_slot(m, ge, nge, a);
      if (t < 0) continue;
      if (++n_g > W2_MAX_GRANTS_PER_MG) { status = MOCHI_MSG_FALLBACK; break; }
      if (!grant_canonical(m + ge[t].voff, ge[t].vlen)) { status = MOCHI_MSG_FALLBACK; break; }
      /* grantSignatures[key]: the last entry with this key, its (last) value */
      const uint8_t* sig = NULL;
      for (size_t q = 0; q < nse; q++)
        if (same(m, se[q].koff, se[q].klen, ge[a].koff, ge[a].klen))
          sig = se[q].vlen == MOCHI_RSA_BYTES ? m + se[q].voff : NULL;
      uint8_t key = 0xFF;
      for (uint32_t j = 0; j < no; j++)
        if (same(m, op_o[j], op_l[j], ge[a].koff, ge[a].klen)) { key = ops[j].key; break; }
      gout_push(go, base + ge[t].voff, (uint32_t)ge[t].vlen, sig, signer, key);
    }
    if (status == MOCHI_MSG_OK) mg_push(mo_out, n_g);
    free(ge);
    free(se);
  }
  free(ce);
  if (status != MOCHI_MSG_OK) { /* drop partial output */
    go->n = g_start;
    mo_out->n = mg_start;
  }
  return status;
}

int oracle_w2_decode(const mochi_write2_batch* w, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids,
                     oracle_w2_decoded* out) {
  if (!w || !out) return MOCHI_EINVAL;
  memset(out, 0, sizeof *out);
  const uint32_t M = w->n_msgs;
  gout_t go;
  memset(&go, 0, sizeof go);
  mgout_t mg;
  memset(&mg, 0, sizeof mg);
  uint32_t* cg = (uint32_t*)calloc(M + 1, sizeof(uint32_t));
  uint32_t* co = (uint32_t*)calloc(M + 1, sizeof(uint32_t));
  uint32_t* cm = (uint32_t*)calloc(M + 1, sizeof(uint32_t));
  uint8_t* st = (uint8_t*)calloc(M ? M : 1, 1);
  size_t ocap = 1024, on = 0;
  uint8_t* opk = (uint8_t*)malloc(ocap);
  uint8_t* opf = (uint8_t*)malloc(ocap);
  int64_t* opt = (int64_t*)malloc(ocap * sizeof(int64_t));
  uint64_t* oko = (uint64_t*)malloc(ocap * sizeof(uint64_t));
  uint32_t* okl = (uint32_t*)malloc(ocap * sizeof(uint32_t));
  for (uint32_t i = 0; i < M; i++) {
    const uint8_t* m = w->wire + w->msg_off[i];
    const size_t ml = w->msg_len[i];
    op_info_t ops[MOCHI_MAX_OPS_PER_CERT];
    uint32_t no = 0;
    const uint32_t mg0 = mg.n;
    int s = valid_write2(m, ml) ? decode_one(m, ml, w->msg_off[i], ids, id_off, n_ids, &go, &mg, ops, &no)
                                : MOCHI_MSG_MALFORMED;
    if (s == MOCHI_MSG_OK && w->op_flags_off && w->op_flags_off[i + 1] - w->op_flags_off[i] != no)
      s = MOCHI_MSG_OPS_MISMATCH;
    if (s != MOCHI_MSG_OK) {
      no = 0;
      go.n = cg[i];
      mg.n = mg0;
    }
    st[i] = (uint8_t)s;
    if (on + no > ocap) {
      while (on + no > ocap) ocap *= 2;
      opk = (uint8_t*)realloc(opk, ocap);
      opf = (uint8_t*)realloc(opf, ocap);
      opt = (int64_t*)realloc(opt, ocap * sizeof(int64_t));
      oko = (uint64_t*)realloc(oko, ocap * sizeof(uint64_t));
      okl = (uint32_t*)realloc(okl, ocap * sizeof(uint32_t));
    }
    for (uint32_t j = 0; j < no; j++) {
      const size_t src = w->op_flags_off ? w->op_flags_off[i] + j : 0;
      opk[on + j] = ops[j].key;
      opf[on + j] = (uint8_t)((w->op_flags_off ? w->op_flags[src] : (MOCHI_OP_LOCAL | MOCHI_OP_HAS_SVOC)) | ops[j].notw);
      opt[on + j] = w->op_flags_off && w->op_object_ts ? w->op_object_ts[src] : 0;
      oko[on + j] = ops[j].k_off;
      okl[on + j] = ops[j].k_len;
    }
    on += no;
    cg[i + 1] = go.n;
    co[i + 1] = (uint32_t)on;
    cm[i + 1] = mg.n;
  }
  uint32_t* mgo = (uint32_t*)malloc(((size_t)mg.n + 1) * sizeof(uint32_t));
  mgo[0] = 0;
  for (uint32_t j = 0; j < mg.n; j++) mgo[j + 1] = mgo[j] + mg.cnt[j];
  free(mg.cnt);
  mochi_batch* b = &out->batch;
  b->n_grants = go.n;
  b->n_certs = M;
  b->n_ops = (uint32_t)on;
  b->n_mgs = mg.n;
  b->grant_bytes_len = w->wire_len;
  b->grant_bytes = w->wire;
  b->grant_off = go.off;
  b->grant_len = go.len;
  b->sig = go.sig;
  b->signer = go.signer;
  b->grant_key = go.key;
  b->cert_grant_off = cg;
  b->cert_op_off = co;
  b->op_key = opk;
  b->op_flags = opf;
  b->expected_hash = w->expected_hash;
  b->cert_mg_off = cm;
  b->mg_grant_off = mgo;
  b->op_object_ts = opt;
  b->op_key_off = oko;
  b->op_key_len = okl;
  out->msg_status = st;
  return MOCHI_OK;
}

void oracle_w2_free(oracle_w2_decoded* d) {
  if (!d) return;
  free((void*)d->batch.grant_off);
  free((void*)d->batch.grant_len);
  free((void*)d->batch.sig);
  free((void*)d->batch.signer);
  free((void*)d->batch.grant_key);
  free((void*)d->batch.cert_grant_off);
  free((void*)d->batch.cert_op_off);
  free((void*)d->batch.op_key);
  free((void*)d->batch.op_flags);
  free((void*)d->batch.cert_mg_off);
  free((void*)d->batch.mg_grant_off);
  free((void*)d->batch.op_object_ts);
  free((void*)d->batch.op_key_off);
  free((void*)d->batch.op_key_len);
  free(d->msg_status);
  free(d->own_blob);
  memset(d, 0, sizeof *d);
}

/* ------------------------------------------------------------------------ */
/* Full Write2ToServer decode (the messages the device fast path declines),   */
/* restated literally: a singular message field given several times is        */
/* parsed as the CONCATENATION of its occurrences (protobuf merge semantics); */
/* map entries: LinkedHashMap put (first position, last entry's value, whose  */
/* message value is again the concatenation of its occurrences; a bytes value */
/* takes the last occurrence).  The signed grant bytes are Grant.toByteArray()*/
/* of the parsed Grant (MochiProtocol.java:7556-7574): known fields, then the */
/* retained unknown fields (parseUnknownFieldProto3) as UnknownFieldSet       */
/* writes them -- ascending field number; per number varint, fixed32,        */
/* fixed64, length-delimited, group values in arrival order; group bodies     */
/* normalised the same way.                                                    */
/* ------------------------------------------------------------------------ */

typedef struct {
  uint8_t* b;
  size_t n, cap;
} buf_t;

static void buf_put(buf_t* o, const void* p, size_t n) {
  if (o->n + n > o->cap) {
    o->cap = (o->n + n) * 2 + 64;
    o->b = (uint8_t*)realloc(o->b, o->cap);
  }
  memcpy(o->b + o->n, p, n);
  o->n += n;
}
static void buf_varint(buf_t* o, uint64_t v) {
  uint8_t t[10];
  buf_put(o, t, put_varint(t, v));
}

/* concatenation of every wt-2 payload of field `field` in [off, off+len) */
static void concat_field(const uint8_t* m, size_t off, size_t len, uint32_t field, buf_t* out) {
  fld_t f;
  int rc;
  FOR_FIELDS(m, off, len, f, rc)
    if (f.field == field && f.wt == 2) buf_put(out, m + off + f.off, f.len);
}

typedef struct {
  uint32_t field;
  int cls; /* 0 varint, 1 fixed32, 2 fixed64, 3 length-delimited, 4 group */
  uint64_t v;
  const uint8_t* p;
  size_t n;
} unk_t;

/* Grant parse retaining unknown fields; returns 0 on malformed input. */
typedef struct {
  const uint8_t *oid, *hash;
  size_t oid_n, hash_n;
  int64_t ts, cfg;
  int32_t status;
  unk_t* unk;
  size_t n_unk;
} full_grant_t;

static int collect_unknown(rd_t* r, uint32_t field, uint32_t wt, unk_t** list, size_t* n, int depth);

/* body of a group that started before r->pos: returns its end offset (before the END tag) */
static int group_body(rd_t* r, uint32_t field, size_t* body_end, int depth) {
  if (depth > 100) return 0;
  for (;;) {
    const size_t at = r->pos;
    uint64_t t64, v;
    if (!rd_varint(r, &t64)) return 0;
    const uint32_t t = (uint32_t)t64, f = t >> 3, wt = t & 7;
    if (f == 0) return 0;
    switch (wt) {
      case 0: if (!rd_varint(r, &v)) return 0; break;
      case 1: if (r->len - r->pos < 8) return 0; r->pos += 8; break;
      case 2: {
        if (!rd_varint(r, &v)) return 0;
        const int32_t l = (int32_t)(uint32_t)v;
        if (l < 0 || (uint64_t)l > r->len - r->pos) return 0;
        r->pos += (size_t)l;
        break;
      }
      case 3: { size_t e; if (!group_body(r, f, &e, depth + 1)) return 0; break; }
      case 4: if (f != field) return 0; *body_end = at; return 1;
      case 5: if (r->len - r->pos < 4) return 0; r->pos += 4; break;
      default: return 0;
    }
  }
}

static int collect_unknown(rd_t* r, uint32_t field, uint32_t wt, unk_t** list, size_t* n, int depth) {
  unk_t u;
  memset(&u, 0, sizeof u);
  u.field = field;
  uint64_t v;
  switch (wt) {
    case 0: if (!rd_varint(r, &v)) return 0; u.cls = 0; u.v = v; break;
    case 5: if (r->len - r->pos < 4) return 0; u.cls = 1; u.p = r->b + r->pos; u.n = 4; r->pos += 4; break;
    case 1: if (r->len - r->pos < 8) return 0; u.cls = 2; u.p = r->b + r->pos; u.n = 8; r->pos += 8; break;
    case 2: {
      if (!rd_varint(r, &v)) return 0;
      const int32_t l = (int32_t)(uint32_t)v;
      if (l < 0 || (uint64_t)l > r->len - r->pos) return 0;
      u.cls = 3; u.p = r->b + r->pos; u.n = (size_t)l; r->pos += (size_t)l;
      break;
    }
    case 3: {
      const size_t start = r->pos;
      size_t end;
      if (!group_body(r, field, &end, depth + 1)) return 0;
      u.cls = 4; u.p = r->b + start; u.n = end - start;
      break;
    }
    default: return 0;
  }
  *list = (unk_t*)realloc(*list, (*n + 1) * sizeof(unk_t));
  (*list)[(*n)++] = u;
  return 1;
}

/* UnknownFieldSet.writeTo of a list (arrival order): by field number, then class */
static void write_unknowns(buf_t* o, const unk_t* u, size_t n);

static void write_group_body(buf_t* o, const uint8_t* p, size_t n) {
  rd_t r = {p, n, 0};
  unk_t* list = NULL;
  size_t k = 0;
  while (r.pos < r.len) {
    uint64_t t64;
    if (!rd_varint(&r, &t64)) break;
    const uint32_t t = (uint32_t)t64;
    if (!collect_unknown(&r, t >> 3, t & 7, &list, &k, 1)) break;
  }
  write_unknowns(o, list, k);
  free(list);
}

static void write_unknowns(buf_t* o, const unk_t* u, size_t n) {
  /* selection over (field, class) pairs in ascending order, arrival order within */
  uint64_t last = 0;
  int first = 1;
  for (;;) {
    uint64_t best = UINT64_MAX;
    for (size_t i = 0; i < n; i++) {
      const uint64_t key = (uint64_t)u[i].field << 3 | (uint64_t)u[i].cls;
      if ((first || key > last) && key < best) best = key;
    }
    if (best == UINT64_MAX) return;
    for (size_t i = 0; i < n; i++) {
      const uint64_t key = (uint64_t)u[i].field << 3 | (uint64_t)u[i].cls;
      if (key != best) continue;
      static const int wt_of[5] = {0, 5, 1, 2, 3};
      buf_varint(o, (uint64_t)u[i].field << 3 | (uint64_t)wt_of[u[i].cls]);
      switch (u[i].cls) {
        case 0: buf_varint(o, u[i].v); break;
        case 1: case 2: buf_put(o, u[i].p, u[i].n); break;
        case 3: buf_varint(o, u[i].n); buf_put(o, u[i].p, u[i].n); break;
        default:
          write_group_body(o, u[i].p, u[i].n);
          buf_varint(o, (uint64_t)u[i].field << 3 | 4);
      }
    }
    last = best;
    first = 0;
  }
}

static int parse_grant_full(const uint8_t* b, size_t n, full_grant_t* g) {
  memset(g, 0, sizeof *g);
  rd_t r = {b, n, 0};
  while (r.pos < r.len) {
    uint64_t t64, v;
    if (!rd_varint(&r, &t64)) return 0;
    const uint32_t tag = (uint32_t)t64, field = tag >> 3, wt = tag & 7;
    if (field == 0) return 0;
    uint32_t so, sl;
    switch (tag) {
      case 10: if (!rd_string(&r, &so, &sl)) return 0; g->oid = b + so; g->oid_n = sl; continue;
      case 16: if (!rd_varint(&r, &v)) return 0; g->ts = (int64_t)v; continue;
      case 24: if (!rd_varint(&r, &v)) return 0; g->cfg = (int64_t)v; continue;
      case 34: if (!rd_string(&r, &so, &sl)) return 0; g->hash = b + so; g->hash_n = sl; continue;
      case 40: if (!rd_varint(&r, &v)) return 0; g->status = (int32_t)(uint32_t)v; continue;
      default:
        if (wt == 4) return 0;
        if (!collect_unknown(&r, field, wt, &g->unk, &g->n_unk, 0)) return 0;
    }
  }
  return 1;
}

static void grant_to_bytes(const full_grant_t* g, buf_t* o) {
  uint8_t tmp[1];
  (void)tmp;
  if (g->oid_n) { buf_varint(o, 10); buf_varint(o, g->oid_n); buf_put(o, g->oid, g->oid_n); }
  if (g->ts) { buf_varint(o, 16); buf_varint(o, (uint64_t)g->ts); }
  if (g->cfg) { buf_varint(o, 24); buf_varint(o, (uint64_t)g->cfg); }
  if (g->hash_n) { buf_varint(o, 34); buf_varint(o, g->hash_n); buf_put(o, g->hash, g->hash_n); }
  if (g->status) { buf_varint(o, 40); buf_varint(o, (uint64_t)(int64_t)g->status); }
  write_unknowns(o, g->unk, g->n_unk);
}

/* map entries of field `field` in [off, off+len): key (last) and the concatenation
 * of the value occurrences (last occurrence only when last_only) */
typedef struct {
  const uint8_t* k;
  size_t kn;
  buf_t val;
} fentry_t;

static size_t full_entries(const uint8_t* m, size_t off, size_t len, uint32_t field, int last_only, fentry_t** out) {
  fentry_t* v = NULL;
  size_t n = 0;
  fld_t f;
  int rc;
  FOR_FIELDS(m, off, len, f, rc) {
    if (f.field != field || f.wt != 2) continue;
    v = (fentry_t*)realloc(v, (n + 1) * sizeof *v);
    fentry_t* e = &v[n++];
    memset(e, 0, sizeof *e);
    fld_t g;
    int rc2;
    const size_t eo = off + f.off;
    FOR_FIELDS(m, eo, f.len, g, rc2) {
      if (g.wt != 2) continue;
      if (g.field == 1) { e->k = m + eo + g.off; e->kn = g.len; }
      if (g.field == 2) {
        if (last_only) e->val.n = 0;
        buf_put(&e->val, m + eo + g.off, g.len);
      }
    }
  }
  *out = v;
  return n;
}

static void free_entries(fentry_t* e, size_t n) {
  for (size_t i = 0; i < n; i++) free(e[i].val.b);
  free(e);
}

/* index of the entry holding the final value of e[i]'s key, or -1 if e[i] is not the key's first entry */
static long fmap_slot(const fentry_t* e, size_t n, size_t i) {
  for (size_t j = 0; j < i; j++)
    if (e[j].kn == e[i].kn && (e[i].kn == 0 || memcmp(e[j].k, e[i].k, e[i].kn) == 0)) return -1;
  size_t last = i;
  for (size_t j = i + 1; j < n; j++)
    if (e[j].kn == e[i].kn && (e[i].kn == 0 || memcmp(e[j].k, e[i].k, e[i].kn) == 0)) last = j;
  return (long)last;
}

/* index of the last entry whose key equals k, -1 if none (map value of key k) */
static long fmap_slot_key(const fentry_t* e, size_t n, const uint8_t* k, size_t kn) {
  long last = -1;
  for (size_t j = 0; j < n; j++)
    if (e[j].kn == kn && (kn == 0 || memcmp(e[j].k, k, kn) == 0)) last = (long)j;
  return last;
}

/* Decode message m fully into `b` (appending one certificate): grants,
 * MultiGrants, ops; grant and op-key bytes go to `blob`.  Returns
 * MOCHI_MSG_OK, or MOCHI_MSG_FALLBACK when it has more than
 * MOCHI_MAX_OPS_PER_CERT operations (one-byte op slots). */
typedef struct {
  buf_t blob;
  gout_t go;
  mgout_t mg;
  uint8_t* opk;
  uint8_t* opn; /* MOCHI_OP_NOT_WRITE per op */
  uint64_t* oko;
  uint32_t* okl;
  size_t on;
} full_out_t;

static int decode_full_one(const uint8_t* m, size_t mlen, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids,
                           full_out_t* o) {
  buf_t wc = {0}, tx = {0};
  concat_field(m, 0, mlen, 1, &wc);
  concat_field(m, 0, mlen, 2, &tx);
  int status = MOCHI_MSG_OK;
  /* operations: every field-1 occurrence of the transaction is one Operation */
  size_t op_o[1024], op_l[1024];
  size_t no = 0;
  uint8_t slots[1024];
  fld_t f;
  int rc;
  const size_t on0 = o->on;
  if (wc.n == 0 && wc.b == NULL) wc.b = (uint8_t*)malloc(1);
  if (tx.b == NULL) tx.b = (uint8_t*)malloc(1);
  FOR_FIELDS(tx.b, 0, tx.n, f, rc) {
    if (f.field != 1 || f.wt != 2) continue;
    if (no == 1024) { status = MOCHI_MSG_FALLBACK; break; }
    last_string(tx.b, f.off, f.len, 2, &op_o[no], &op_l[no]);
    const int32_t action = (int32_t)(uint32_t)last_varint(tx.b, f.off, f.len, 1);
    uint32_t slot = (uint32_t)no;
    for (size_t j = 0; j < no; j++)
      if (same(tx.b, op_o[j], op_l[j], op_o[no], op_l[no])) { slot = slots[j]; break; }
    slots[no] = (uint8_t)(slot < 255 ? slot : 255);
    o->opk = (uint8_t*)realloc(o->opk, o->on + 1);
    o->opn = (uint8_t*)realloc(o->opn, o->on + 1);
    o->oko = (uint64_t*)realloc(o->oko, (o->on + 1) * sizeof(uint64_t));
    o->okl = (uint32_t*)realloc(o->okl, (o->on + 1) * sizeof(uint32_t));
    o->opk[o->on] = slots[no];
    o->opn[o->on] = (action != 1 && action != 2) || op_l[no] == 0 ? MOCHI_OP_NOT_WRITE : 0;
    o->oko[o->on] = o->blob.n;
    o->okl[o->on] = (uint32_t)op_l[no];
    buf_put(&o->blob, tx.b + op_o[no], op_l[no]);
    o->on++;
    no++;
  }
  if (no > MOCHI_MAX_OPS_PER_CERT) status = MOCHI_MSG_FALLBACK;
  const uint32_t g0 = o->go.n, m0 = o->mg.n;
  if (status == MOCHI_MSG_OK) {
    fentry_t* ce;
    const size_t nce = full_entries(wc.b, 0, wc.n, 1, 0, &ce);
    for (size_t i = 0; i < nce; i++) {
      const long s = fmap_slot(ce, nce, i);
      if (s < 0) continue;
      const fentry_t* mgv = &ce[s];
      const uint8_t* mb = mgv->val.b ? mgv->val.b : (const uint8_t*)"";
      size_t sid_o, sid_l;
      last_string(mb, 0, mgv->val.n, 4, &sid_o, &sid_l);
      uint16_t signer = 0xFFFF;
      for (uint32_t k = 0; k < n_ids; k++)
        if (id_off[k + 1] - id_off[k] == sid_l && memcmp(ids + id_off[k], mb + sid_o, sid_l) == 0) { signer = (uint16_t)k; break; }
      fentry_t *ge, *se;
      const size_t nge = full_entries(mb, 0, mgv->val.n, 1, 0, &ge);
      const size_t nse = full_entries(mb, 0, mgv->val.n, 5, 1, &se);
      uint32_t n_g = 0;
      for (size_t a = 0; a < nge; a++) {
        const long t = fmap_slot(ge, nge, a);
        if (t < 0) continue;
        full_grant_t g;
        if (!parse_grant_full(ge[t].val.b ? ge[t].val.b : (const uint8_t*)"", ge[t].val.n, &g)) { status = MOCHI_MSG_MALFORMED; free(g.unk); break; }
        const uint64_t goff = o->blob.n;
        grant_to_bytes(&g, &o->blob);
        free(g.unk);
        const uint8_t* sig = NULL;
        const long st = fmap_slot_key(se, nse, ge[a].k, ge[a].kn);
        if (st >= 0 && se[st].val.n == MOCHI_RSA_BYTES) sig = se[st].val.b;
        uint8_t key = 0xFF;
        for (size_t j = 0; j < no; j++)
          if (op_l[j] == ge[a].kn && (ge[a].kn == 0 || memcmp(tx.b + op_o[j], ge[a].k, ge[a].kn) == 0)) { key = slots[j]; break; }
        gout_push(&o->go, goff, (uint32_t)(o->blob.n - goff), sig, signer, key);
        n_g++;
      }
      mg_push(&o->mg, n_g);
      free_entries(ge, nge);
      free_entries(se, nse);
      if (status != MOCHI_MSG_OK) break;
    }
    free_entries(ce, nce);
  }
  if (status != MOCHI_MSG_OK) {
    o->go.n = g0;
    o->mg.n = m0;
    o->on = on0;
  }
  free(wc.b);
  free(tx.b);
  return status;
}

int oracle_w2_decode_full(const mochi_write2_batch* w, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids,
                          oracle_w2_decoded* out) {
  if (!w || !out) return MOCHI_EINVAL;
  memset(out, 0, sizeof *out);
  const uint32_t M = w->n_msgs;
  full_out_t o;
  memset(&o, 0, sizeof o);
  uint32_t* cg = (uint32_t*)calloc(M + 1, sizeof(uint32_t));
  uint32_t* co = (uint32_t*)calloc(M + 1, sizeof(uint32_t));
  uint32_t* cm = (uint32_t*)calloc(M + 1, sizeof(uint32_t));
  uint8_t* st = (uint8_t*)calloc(M ? M : 1, 1);
  for (uint32_t i = 0; i < M; i++) {
    const uint8_t* m = w->wire + w->msg_off[i];
    const size_t ml = w->msg_len[i];
    st[i] = (uint8_t)(valid_write2(m, ml) ? decode_full_one(m, ml, ids, id_off, n_ids, &o) : MOCHI_MSG_MALFORMED);
    cg[i + 1] = o.go.n;
    co[i + 1] = (uint32_t)o.on;
    cm[i + 1] = o.mg.n;
  }
  uint32_t* mgo = (uint32_t*)malloc(((size_t)o.mg.n + 1) * sizeof(uint32_t));
  mgo[0] = 0;
  for (uint32_t j = 0; j < o.mg.n; j++) mgo[j + 1] = mgo[j] + o.mg.cnt[j];
  free(o.mg.cnt);
  if (!o.blob.b) o.blob.b = (uint8_t*)malloc(1);
  uint8_t* opf = (uint8_t*)malloc(o.on + 1);
  int64_t* opt = (int64_t*)calloc(o.on + 1, sizeof(int64_t));
  for (uint32_t i = 0; i < M; i++)
    for (uint32_t j = co[i]; j < co[i + 1]; j++) {
      const int flagged = w->op_flags_off && w->op_flags_off[i + 1] - w->op_flags_off[i] == co[i + 1] - co[i];
      opf[j] = (uint8_t)((flagged ? w->op_flags[w->op_flags_off[i] + j - co[i]] : (MOCHI_OP_LOCAL | MOCHI_OP_HAS_SVOC)) |
                         o.opn[j]);
      opt[j] = flagged && w->op_object_ts ? w->op_object_ts[w->op_flags_off[i] + j - co[i]] : 0;
    }
  free(o.opn);
  mochi_batch* b = &out->batch;
  b->n_grants = o.go.n;
  b->n_certs = M;
  b->n_ops = (uint32_t)o.on;
  b->n_mgs = cm[M];
  b->grant_bytes_len = o.blob.n;
  b->grant_bytes = o.blob.b;
  b->grant_off = o.go.off;
  b->grant_len = o.go.len;
  b->sig = o.go.sig;
  b->signer = o.go.signer;
  b->grant_key = o.go.key;
  b->cert_grant_off = cg;
  b->cert_op_off = co;
  b->op_key = o.opk ? o.opk : (uint8_t*)malloc(1);
  b->op_flags = opf;
  b->expected_hash = w->expected_hash;
  b->cert_mg_off = cm;
  b->mg_grant_off = mgo;
  b->op_object_ts = opt;
  b->op_key_off = o.oko;
  b->op_key_len = o.okl;
  out->msg_status = st;
  out->own_blob = o.blob.b;
  return MOCHI_OK;
}

int oracle_verify_write2(const uint8_t* moduli_be, uint32_t n_keys, const uint8_t* ids, const uint32_t* id_off,
                         const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* out, uint8_t* msg_status,
                         int n_threads) {
  oracle_w2_decoded d;
  int rc = oracle_w2_decode(w, ids, id_off, n_keys, &d);
  if (rc) return rc;
  const uint32_t O = d.batch.n_ops;
  const int per_op = out->op_decision || out->op_g0 || out->op_ts;
  if (per_op && !w->op_flags_off) {
    oracle_w2_free(&d);
    return MOCHI_EINVAL;
  }
  mochi_verdicts v = *out;
  v.grant_valid_bits = NULL;
  v.grant_flags = NULL;
  v.grant_ts = NULL;
  /* per-op results in decoded order, scattered to the op_flags_off layout below */
  v.op_decision = (uint8_t*)malloc(O ? O : 1);
  v.op_g0 = (uint32_t*)malloc(sizeof(uint32_t) * (O ? O : 1));
  v.op_ts = (int64_t*)malloc(sizeof(int64_t) * (O ? O : 1));
  rc = oracle_verify_batch(moduli_be, n_keys, &d.batch, p, &v, n_threads);
  for (uint32_t i = 0; rc == MOCHI_OK && i < w->n_msgs; i++) {
    const uint8_t s = d.msg_status[i];
    if (msg_status) msg_status[i] = s;
    if (per_op) {
      const uint32_t lo = w->op_flags_off[i], hi = w->op_flags_off[i + 1], dlo = d.batch.cert_op_off[i];
      for (uint32_t o = lo; o < hi; o++) {
        const int ok = s == MOCHI_MSG_OK;
        if (out->op_decision) out->op_decision[o] = ok ? v.op_decision[dlo + o - lo] : MOCHI_OPD_SKIPPED;
        if (out->op_g0) out->op_g0[o] = ok ? v.op_g0[dlo + o - lo] : 0xFFFFFFFFu;
        if (out->op_ts) out->op_ts[o] = ok ? v.op_ts[dlo + o - lo] : 0;
      }
    }
    if (s == MOCHI_MSG_OK) continue;
    out->cert_accept_bits[i >> 5] &= ~(1u << (i & 31));
    if (out->cert_reason) out->cert_reason[i] = s == MOCHI_MSG_MALFORMED ? MOCHI_REJECT_MALFORMED : MOCHI_UNDECIDED;
    if (out->cert_fail_op) out->cert_fail_op[i] = 0xFF;
  }
  free(v.op_decision);
  free(v.op_g0);
  free(v.op_ts);
  /* FALLBACK messages: the full decode, verified like any other certificate.
   * Left UNDECIDED: more than MOCHI_MAX_OPS_PER_CERT operations, op_flags_off
   * disagreeing with the operation count, or a grant over 64 KiB. */
  uint32_t n_fb = 0;
  for (uint32_t i = 0; rc == MOCHI_OK && i < w->n_msgs; i++) n_fb += d.msg_status[i] == MOCHI_MSG_FALLBACK;
  if (rc == MOCHI_OK && n_fb) {
    oracle_w2_decoded f;
    rc = oracle_w2_decode_full(w, ids, id_off, n_keys, &f);
    if (rc == MOCHI_OK) {
      const uint32_t C = w->n_msgs, O = f.batch.n_ops, N = f.batch.n_grants;
      mochi_verdicts fv;
      memset(&fv, 0, sizeof fv);
      fv.cert_accept_bits = (uint32_t*)calloc((C + 31) / 32 + 1, 4);
      fv.cert_reason = (uint8_t*)malloc(C + 1);
      fv.cert_fail_op = (uint8_t*)malloc(C + 1);
      fv.op_decision = (uint8_t*)malloc(O + 1);
      fv.op_g0 = (uint32_t*)malloc(4 * ((size_t)O + 1));
      fv.op_ts = (int64_t*)malloc(8 * ((size_t)O + 1));
      rc = oracle_verify_batch(moduli_be, n_keys, &f.batch, p, &fv, n_threads);
      for (uint32_t i = 0; rc == MOCHI_OK && i < C; i++) {
        if (d.msg_status[i] != MOCHI_MSG_FALLBACK || f.msg_status[i] != MOCHI_MSG_OK) continue;
        const uint32_t lo = f.batch.cert_op_off[i], no = f.batch.cert_op_off[i + 1] - lo;
        if (w->op_flags_off && w->op_flags_off[i + 1] - w->op_flags_off[i] != no) continue;
        int big = 0;
        for (uint32_t g = f.batch.cert_grant_off[i]; g < f.batch.cert_grant_off[i + 1]; g++) big |= f.batch.grant_len[g] > 65536;
        if (big) continue;
        const int a = (fv.cert_accept_bits[i >> 5] >> (i & 31)) & 1;
        if (a) out->cert_accept_bits[i >> 5] |= 1u << (i & 31);
        else out->cert_accept_bits[i >> 5] &= ~(1u << (i & 31));
        if (out->cert_reason) out->cert_reason[i] = fv.cert_reason[i];
        if (out->cert_fail_op) out->cert_fail_op[i] = fv.cert_fail_op[i];
        if (per_op)
          for (uint32_t j = 0; j < no; j++) {
            const size_t dst = w->op_flags_off[i] + j;
            if (out->op_decision) out->op_decision[dst] = fv.op_decision[lo + j];
            if (out->op_g0) out->op_g0[dst] = fv.op_g0[lo + j];
            if (out->op_ts) out->op_ts[dst] = fv.op_ts[lo + j];
          }
      }
      (void)N;
      free(fv.cert_accept_bits);
      free(fv.cert_reason);
      free(fv.cert_fail_op);
      free(fv.op_decision);
      free(fv.op_g0);
      free(fv.op_ts);
      oracle_w2_free(&f);
    }
  }
  oracle_w2_free(&d);
  return rc;
}
