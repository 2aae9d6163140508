// signer.cpp — producer-side grant signing (CPU, OpenSSL).
//
// The reference builds each MultiGrant at InMemoryDataStore.java:283-295 and
// leaves "// TODO: add signature" at MochiProtocol.proto:123.  This is that
// signature: RSA-2048 PKCS#1 v1.5 over SHA-256(Grant.toByteArray()).  Used by
// the synthetic workload generator and by a signing server; the verify hot
// path never calls it.
#include <openssl/bn.h>
#include <openssl/core_names.h>
#include <openssl/evp.h>
#include <openssl/pem.h>

#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mochi_hip.h"

namespace {
EVP_PKEY* load_key(const char* pem) {
  BIO* bio = BIO_new_mem_buf(pem, -1);
  EVP_PKEY* k = PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  return k;
}
}  // namespace

extern "C" int mochi_sign_grants(const char* pem_private_key, uint32_t n, const uint8_t* grant_bytes,
                                 const uint64_t* grant_off, const uint32_t* grant_len, uint8_t* sig_out,
                                 int n_threads) {
  if (!pem_private_key || (n && (!grant_bytes || !grant_off || !grant_len || !sig_out))) return MOCHI_EINVAL;
  EVP_PKEY* probe = load_key(pem_private_key);
  if (!probe) return MOCHI_EINVAL;
  const bool rsa2048 = EVP_PKEY_get_bits(probe) == 2048;
  EVP_PKEY_free(probe);
  if (!rsa2048) return MOCHI_EINVAL;
  if (n_threads < 1) n_threads = 1;
  std::vector<int> status(n_threads, MOCHI_OK);
  auto work = [&](int t) {
    EVP_PKEY* key = load_key(pem_private_key);  // one key object per thread
    EVP_MD_CTX* md = EVP_MD_CTX_new();
    const uint32_t lo = (uint32_t)((uint64_t)n * t / n_threads), hi = (uint32_t)((uint64_t)n * (t + 1) / n_threads);
    for (uint32_t i = lo; i < hi; i++) {
      size_t slen = MOCHI_RSA_BYTES;
      if (EVP_DigestSignInit(md, nullptr, EVP_sha256(), nullptr, key) <= 0 ||
          EVP_DigestSign(md, sig_out + (size_t)i * MOCHI_RSA_BYTES, &slen, grant_bytes + grant_off[i], grant_len[i]) != 1 ||
          slen != MOCHI_RSA_BYTES) {
        status[t] = MOCHI_EINVAL;
        break;
      }
    }
    EVP_MD_CTX_free(md);
    EVP_PKEY_free(key);
  };
  if (n_threads == 1) {
    work(0);
  } else {
    std::vector<std::thread> th;
    for (int t = 0; t < n_threads; t++) th.emplace_back(work, t);
    for (auto& x : th) x.join();
  }
  for (int s : status)
    if (s) return s;
  return MOCHI_OK;
}

extern "C" int mochi_pem_modulus(const char* pem_key, uint8_t* n_be_out) {
  if (!pem_key || !n_be_out) return MOCHI_EINVAL;
  BIO* bio = BIO_new_mem_buf(pem_key, -1);
  EVP_PKEY* k = PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr);
  BIO_free(bio);
  if (!k) {
    bio = BIO_new_mem_buf(pem_key, -1);
    k = PEM_read_bio_PUBKEY(bio, nullptr, nullptr, nullptr);
    BIO_free(bio);
  }
  if (!k) return MOCHI_EINVAL;
  BIGNUM* nn = nullptr;
  const bool ok = EVP_PKEY_get_bn_param(k, OSSL_PKEY_PARAM_RSA_N, &nn) == 1 && BN_num_bytes(nn) == MOCHI_RSA_BYTES &&
                  BN_bn2binpad(nn, n_be_out, MOCHI_RSA_BYTES) == MOCHI_RSA_BYTES;
  BN_free(nn);
  EVP_PKEY_free(k);
  return ok ? MOCHI_OK : MOCHI_EINVAL;
}
