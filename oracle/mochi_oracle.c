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

#define ORACLE_MAX_GROUP_DEPTH 16

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

int oracle_tally(const mochi_batch* b, const mochi_params* p, const uint8_t* grant_flags, const int64_t* grant_ts,
                 mochi_verdicts* out) {
  if (!b || !p || !grant_flags || !grant_ts || !out || !out->cert_accept_bits) return MOCHI_EINVAL;
  const uint32_t M = oracle_server_majority(p->replication_factor);
  memset(out->cert_accept_bits, 0, ((size_t)b->n_certs + 31) / 32 * 4);
  for (uint32_t c = 0; c < b->n_certs; c++) {
    const uint32_t g_lo = b->cert_grant_off[c], g_hi = b->cert_grant_off[c + 1];
    const uint32_t o_lo = b->cert_op_off[c], o_hi = b->cert_op_off[c + 1];
    const uint32_t n_ops = o_hi - o_lo;
    uint8_t reason = MOCHI_ACCEPT, fail_op = 0xFF;

    /* Malformed grant bytes: the reference fails in the protobuf decoder
     * before any of the protocol code runs (MochiServerInitializer.java:30-34). */
    for (uint32_t g = g_lo; g < g_hi && reason == MOCHI_ACCEPT; g++)
      if (!(grant_flags[g] & MOCHI_GRANT_PARSED)) reason = MOCHI_REJECT_MALFORMED;

    /* multiplicity of each key slot = number of txn ops naming that key */
    uint32_t mult[MOCHI_MAX_OPS_PER_CERT];
    int seen[MOCHI_MAX_OPS_PER_CERT];
    int64_t ts0[MOCHI_MAX_OPS_PER_CERT];
    uint32_t cnt[MOCHI_MAX_OPS_PER_CERT];
    uint32_t first[MOCHI_MAX_OPS_PER_CERT];
    memset(mult, 0, sizeof mult);
    memset(seen, 0, sizeof seen);
    memset(cnt, 0, sizeof cnt);
    for (uint32_t o = o_lo; o < o_hi; o++) mult[b->op_key[o]]++;

    /* processMultiGrantsFromAllServers  InMemoryDataStore.java:613-640
     *   for (multiGrant : wc.grants.values())            -- wire order
     *     for (op : transaction.operations)              -- txn order
     *       grant = multiGrant.grants.get(op.operand1)   -- (invalid signature => absent)
     *       if (grant == null) continue;                 -- :622-624
     *       if (coalesced.containsKey(key)) {
     *         if (coalesced[key].ts != grant.ts) throw UnsupportedOperationException  -- :626-628
     *         coalesced[key].list.add(grant)             -- :629
     *       } else coalesced.put(key, (grant.ts, [grant])) -- :631-634
     * A grant for key slot s is appended once per op naming s (mult[s] times);
     * its own comparisons against ts0 all agree, so only the first sighting
     * per slot matters for ts0 and g0. */
    for (uint32_t g = g_lo; g < g_hi && reason == MOCHI_ACCEPT; g++) {
      if (!(grant_flags[g] & MOCHI_GRANT_SIG_OK)) continue;
      const uint32_t s = b->grant_key[g];
      if (s >= MOCHI_MAX_OPS_PER_CERT || mult[s] == 0) continue; /* never looked up */
      if (!seen[s]) {
        seen[s] = 1;
        ts0[s] = grant_ts[g];
        first[s] = g;
        cnt[s] = mult[s];
      } else {
        if (ts0[s] != grant_ts[g]) {
          reason = MOCHI_REJECT_TS_MISMATCH;
          break;
        }
        cnt[s] += mult[s];
      }
    }

    /* write2apply verdict part  InMemoryDataStore.java:576-611, ops in txn order */
    for (uint32_t j = 0; j < n_ops && reason == MOCHI_ACCEPT; j++) {
      const uint32_t o = o_lo + j;
      const uint8_t fl = b->op_flags[o];
      if (!(fl & MOCHI_OP_LOCAL)) continue; /* WRONG_SHARD result  :582-587 */
      const uint32_t s = b->op_key[o];
      if (!seen[s]) { /* coalescedTxnGrantMap.get(key) == null -> NPE  :588 */
        reason = MOCHI_REJECT_NO_GRANT;
        fail_op = (uint8_t)j;
        break;
      }
      /* Utils.assertTrue(list.size() > getServerMajority())  :590 (client: >=) */
      const int quorum_ok = p->strict_gt ? (cnt[s] > M) : (cnt[s] >= M);
      if (!quorum_ok) {
        reason = MOCHI_REJECT_BELOW_QUORUM;
        fail_op = (uint8_t)j;
        break;
      }
      /* if (grantForObject.getTransactionHash().equals(txnHash)) ... else throw  :591,605-607 */
      const uint32_t g0 = first[s];
      if (!hash_equals(b->grant_bytes + b->grant_off[g0], b->grant_len[g0],
                       b->expected_hash + (size_t)c * MOCHI_TXN_HASH_BYTES)) {
        reason = MOCHI_REJECT_HASH_MISMATCH;
        fail_op = (uint8_t)j;
        break;
      }
      /* storeValueContainer = getDataMap(key).get(key); op.getOperand1().equals(svoc.getKey()) -> NPE if null  :592-593 */
      if (!(fl & MOCHI_OP_HAS_SVOC)) {
        reason = MOCHI_REJECT_NO_SVOC;
        fail_op = (uint8_t)j;
        break;
      }
    }

    if (reason == MOCHI_ACCEPT) out->cert_accept_bits[c >> 5] |= 1u << (c & 31);
    if (out->cert_reason) out->cert_reason[c] = reason;
    if (out->cert_fail_op) out->cert_fail_op[c] = fail_op;
  }
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
