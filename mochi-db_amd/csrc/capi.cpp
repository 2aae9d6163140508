// capi.cpp — libmochi_hip C ABI (include/mochi_hip.h): contexts, key tables,
// device scratch, host<->device staging, and the client-side tally.
//
// The verify path it drives replaces, in the reference,
//   InMemoryDataStore.processWrite2ToServer  (InMemoryDataStore.java:641-666)
// with one batched call over many certificates.
#include <hip/hip_runtime.h>
#include <openssl/bn.h>
#include <openssl/core_names.h>
#include <openssl/evp.h>
#include <openssl/pem.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <condition_variable>
#include <mutex>
#include <thread>
#include <string>
#include <vector>

#include "../../include/mochi_hip.h"
#include "kernels.h"
#include "mont.h"
#include "w2.h"
#include "w2_host.h"

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

bool prep_serial() {
  static const bool v = [] {
    const char* e = getenv("MOCHI_PREP_SERIAL");
    return e && atoi(e) != 0;
  }();
  return v;
}

bool fixup_kernel() {
  static const bool v = [] {
    const char* e = getenv("MOCHI_W2_FIXUP_KERNEL");
    return e && atoi(e) != 0;
  }();
  return v;
}

bool copy_streams() {
  static const bool v = [] {
    const char* e = getenv("MOCHI_COPY_STREAMS");
    return e && atoi(e) != 0;
  }();
  return v;
}

uint32_t default_chunk_grants() {
  const char* e = getenv("MOCHI_CHUNK_GRANTS");
  const long x = e ? atol(e) : 0;
  return (uint32_t)(x > 0 ? x : 262144);
}

#define HIP_TRY(expr)                                                                        \
  do {                                                                                       \
    hipError_t e_ = (expr);                                                                  \
    if (e_ != hipSuccess) return fail(MOCHI_EHIP, "%s: %s", #expr, hipGetErrorString(e_));   \
  } while (0)

// Growable device allocation.
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return MOCHI_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 256 ? 256 : bytes;
    if (hipMalloc(&p, want) != hipSuccess) return fail(MOCHI_ENOMEM, "hipMalloc(%zu) failed", want);
    cap = want;
    return MOCHI_OK;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  template <typename T>
  T* as() const {
    return static_cast<T*>(p);
  }
};

struct PinnedBuf {
  void* p = nullptr;
  size_t cap = 0;
  int ensure(size_t bytes) {
    if (bytes <= cap) return MOCHI_OK;
    if (p) (void)hipHostFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes < 4096 ? 4096 : bytes + bytes / 4;
    if (hipHostMalloc(&p, want, hipHostMallocDefault) != hipSuccess)
      return fail(MOCHI_ENOMEM, "hipHostMalloc(%zu) failed", want);
    cap = want;
    return MOCHI_OK;
  }
  ~PinnedBuf() {
    if (p) (void)hipHostFree(p);
  }
};

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- host-side key precompute (OpenSSL BN, setup only) --------------------

// Cpad = EMSA-PKCS1-v1_5 encoding (RFC 8017 §9.2) of SHA-256 with an all-zero
// digest: 00 01 FF..FF 00 || DigestInfo(SHA-256) || 32 zero bytes.
void pkcs1_cpad(uint8_t cpad[256]) {
  static const uint8_t kDigestInfo[19] = {0x30, 0x31, 0x30, 0x0d, 0x06, 0x09, 0x60, 0x86, 0x48, 0x01,
                                          0x65, 0x03, 0x04, 0x02, 0x01, 0x05, 0x00, 0x04, 0x20};
  memset(cpad, 0xFF, 256);
  cpad[0] = 0x00;
  cpad[1] = 0x01;
  cpad[256 - 32 - 19 - 1] = 0x00;
  memcpy(cpad + 256 - 32 - 19, kDigestInfo, 19);
  memset(cpad + 256 - 32, 0, 32);
}

int make_key_entry(const uint8_t* n_be, mochi::KeyEntry* e) {
  using namespace mochi;
  memset(e, 0, sizeof *e);
  if (!(n_be[0] & 0x80)) return fail(MOCHI_EINVAL, "modulus is not 2048 bits (top bit clear)");
  if (!(n_be[255] & 1)) return fail(MOCHI_EINVAL, "modulus is even");
  // 32-bit words, little-endian word order
  for (int i = 0; i < 64; i++) {
    const uint8_t* b = n_be + 256 - 4 * (i + 1);
    e->n32[i] = (uint32_t)b[0] << 24 | (uint32_t)b[1] << 16 | (uint32_t)b[2] << 8 | b[3];
  }
  auto to_limbs = [](const uint32_t* w, uint32_t* x) {
    for (int j = 0; j < kL; j++) {
      const int bit = j * kLimbBits, wi = bit >> 5, sh = bit & 31;
      const uint64_t lo = wi < 64 ? w[wi] : 0, hi = wi + 1 < 64 ? w[wi + 1] : 0;
      x[j] = (uint32_t)(((hi << 32) | lo) >> sh) & kLimbMask;
    }
  };
  to_limbs(e->n32, e->n);
  // n0inv = -n^{-1} mod 2^28 (Newton iteration on 32 bits)
  uint32_t inv = 1;
  for (int i = 0; i < 6; i++) inv *= 2u - e->n32[0] * inv;
  e->n0inv = (0u - inv) & kLimbMask;
  // Per-key constants (R = 2^(28*74)); k_rsa_pow leaves z = s^(2^16) mod n:
  //   kfix = R^2 mod n                           (k_rsa_raw: MontMul(MontMul(z, K), s) = s^65537)
  //   q    = R^-1 mod n                          (k_rsa_final: MontMul(z, s) = s^65537 * q)
  //   a2   = (Cpad * q mod n) + 2n               (k_rsa_final: target EM*q = Cpad*q + H*q)
  uint8_t cpad[256];
  pkcs1_cpad(cpad);
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *n = BN_bin2bn(n_be, 256, nullptr), *r = BN_new(), *k = BN_new(), *ex = BN_new(), *t = BN_new(),
         *q = BN_new(), *a2 = BN_new(), *cp = BN_bin2bn(cpad, 256, nullptr), *n2 = BN_new();
  int ok = ctx && n && r && k && ex && t && q && a2 && cp && n2;
  ok = ok && BN_set_bit(r, kL * kLimbBits) && BN_mod(r, r, n, ctx);
  ok = ok && BN_mod_mul(k, r, r, n, ctx);
  ok = ok && BN_copy(t, r) && BN_mod_inverse(q, t, n, ctx) != nullptr;
  ok = ok && BN_mod_mul(a2, cp, q, n, ctx) && BN_lshift1(n2, n) && BN_add(a2, a2, n2);
  auto to_limbs_bn = [](const BIGNUM* v, uint32_t* x) {
    uint8_t le[264];
    if (BN_bn2lebinpad(v, le, sizeof le) != (int)sizeof le) return 0;
    for (int j = 0; j < kL; j++) {
      const int bit = j * kLimbBits, by = bit >> 3, sh = bit & 7;
      uint64_t w = 0;
      for (int b = 0; b < 5; b++) w |= (uint64_t)le[by + b] << (8 * b);
      x[j] = (uint32_t)(w >> sh) & kLimbMask;
    }
    return 1;
  };
  ok = ok && to_limbs_bn(k, e->kfix) && to_limbs_bn(q, e->q) && to_limbs_bn(a2, e->a2);
  for (BIGNUM* b : {n, r, k, ex, t, q, a2, cp, n2}) BN_free(b);
  BN_CTX_free(ctx);
  if (!ok) return fail(MOCHI_EINVAL, "key precompute failed");
  return MOCHI_OK;
}

// Fold matrix of k_rsa_pow (fold.h): R_{j,b} = 2^(28(73+j)+8b) mod n as balanced
// mixed-radix digits (8, 8, 8, 4 bits per 28-bit limb), laid out as MFMA A fragments.
int make_fold_key(const uint8_t* n_be, mochi::FoldKey* f) {
  using namespace mochi;
  memset(f, 0, sizeof *f);
  static thread_local std::vector<int8_t> W;  // [296 rows][300 k]
  constexpr int kRows = kFoldLimbs * 4, kK = kFoldNH * 4;
  W.assign((size_t)kRows * kK, 0);
  BN_CTX* ctx = BN_CTX_new();
  BIGNUM *n = BN_bin2bn(n_be, 256, nullptr), *r = BN_new(), *sum = BN_new();
  int ok = ctx && n && r && sum;
  if (ok) BN_zero(sum);
  ok = ok && BN_set_bit(r, kLimbBits * kFoldF) && BN_mod(r, r, n, ctx);
  uint8_t le[264];
  for (int k = 0; k < kK && ok; k++) {
    if (k) ok = BN_lshift(r, r, (k & 3) ? 8 : 4) && BN_mod(r, r, n, ctx);  // limb = 8 + 8 + 8 + 4 bits
    if ((k & 3) != 3) ok = ok && BN_add(sum, sum, r);  // bytes 0..2 are biased, byte 3 is a signed digit
    ok = ok && BN_bn2lebinpad(r, le, sizeof le) == (int)sizeof le;
    int carry = 0;
    for (int row = 0; row < kRows && ok; row++) {
      const int bit = 28 * (row >> 2) + 8 * (row & 3), w = (row & 3) == 3 ? 4 : 8;
      const int field = (int)((((uint32_t)le[bit >> 3] | (uint32_t)le[(bit >> 3) + 1] << 8) >> (bit & 7)) & ((1u << w) - 1));
      int d = field + carry;
      carry = d >= (1 << (w - 1));
      if (carry) d -= 1 << w;
      W[(size_t)row * kK + k] = (int8_t)d;
    }
    ok = ok && carry == 0;
  }
  // cadd = 128 * sum_{j, b<3} R_{j,b} + kFoldOffN * n (fold.h) and cnc = cadd + n - Cpad
  // (k_rsa_final) as 74 limbs of 28 bits
  auto limbs = [&](const BIGNUM* v, uint32_t* out) {
    if (BN_num_bits(v) > kLimbBits * kFoldLimbs || BN_bn2lebinpad(v, le, sizeof le) != (int)sizeof le) return 0;
    for (int q = 0; q < kFoldLimbs; q++) {
      const int bit = q * kLimbBits, by = bit >> 3;
      uint64_t w = 0;
      for (int b = 0; b < 5 && by + b < (int)sizeof le; b++) w |= (uint64_t)le[by + b] << (8 * b);
      out[q] = (uint32_t)(w >> (bit & 7)) & kLimbMask;
    }
    return 1;
  };
  uint8_t cpad[256];
  pkcs1_cpad(cpad);
  BIGNUM* cp = BN_bin2bn(cpad, 256, nullptr);
  BIGNUM* off = BN_new();
  ok = ok && cp && off && BN_lshift(sum, sum, 7) && BN_set_word(off, kFoldOffN) && BN_mul(off, off, n, ctx) &&
       BN_add(sum, sum, off) && limbs(sum, f->cadd);
  BN_free(off);
  ok = ok && BN_add(sum, sum, n) && BN_sub(sum, sum, cp) && !BN_is_negative(sum) && limbs(sum, f->cnc);
  BN_free(cp);
  BN_free(n);
  BN_free(r);
  BN_free(sum);
  BN_CTX_free(ctx);
  if (!ok) return fail(MOCHI_EINVAL, "fold matrix precompute failed");
  for (int mt = 0; mt < kFoldMT; mt++)
    for (int ks = 0; ks < kFoldKS; ks++)
      for (int lane = 0; lane < 64; lane++)
        for (int jj = 0; jj < 16; jj++) {
          const int row = 32 * mt + (lane & 31), limb = 8 * ks + 4 * (lane >> 5) + jj / 4;
          if (row < kRows && limb < kFoldNH)
            f->img[((mt * kFoldKS + ks) * 64 + lane) * 16 + jj] = W[(size_t)row * kK + 4 * limb + jj % 4];
        }
  return MOCHI_OK;
}

}  // namespace

namespace mochi {
// multi.cpp: the device accept bitmap of the context's last host-path call
const uint32_t* ctx_last_accept_dev(mochi_ctx* c, uint32_t* words, int* device, hipStream_t* stream);
int set_error(int code, const std::string& msg) {
  g_err = msg;
  return code;
}
}  // namespace mochi

struct mochi_ctx {
  // batchers built on this context (mochi_batcher_create*) hold it until they
  // are freed -- a batcher destroyed from its own callback is freed later by
  // its last flusher thread, which still uses the context's streams and pinned
  // buffers until then.  mochi_ctx_destroy with a holder left never blocks: it
  // marks the context and the last holder's release frees it.
  std::mutex ref_mu;
  int batcher_refs = 0;
  bool destroy_pending = false;
  int device = 0;
  hipStream_t stream = nullptr;
  uint32_t n_keys = 0;
  mochi::KeyEntry* d_keys = nullptr;
  mochi::FoldKey* d_fold = nullptr;  // per-key k_rsa_pow fold matrices (~101 KB each)
  std::mutex mu;
  // verify scratch
  DevBuf digest, ts, hash_off, hash_len, flags, count, cursor, total, perm, xbuf, dedup, lead;
  // host-path device copies
  DevBuf dev_in, dev_out;
  PinnedBuf pin_in, pin_out;
  hipStream_t s_in = nullptr, s_out = nullptr;  // host-path copy streams
  hipStream_t aux = nullptr;                     // grant prep (high priority), beside k_rsa_pow
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // Scratch ordering: every launch that uses the context's scratch waits for
  // the previous one to be done with it (the device entry points are async on a
  // caller-chosen stream, so two calls on different streams would otherwise
  // race on digest / perm / xbuf / decode buffers).
  hipEvent_t ev_scratch = nullptr;
  bool scratch_used = false;
  hipStream_t scratch_st = nullptr;  // the stream ev_scratch was last recorded on
  std::vector<hipEvent_t> chunk_ev;              // host-path chunk hand-offs
  std::vector<hipEvent_t> tot_ev;                // wire host path: per-chunk decode totals on the host
  // two sets of the host-path call's span events: a call records into one while
  // the other keeps the last completed call's, read only when asked
  hipEvent_t evs[2][4] = {{nullptr, nullptr, nullptr, nullptr}, {nullptr, nullptr, nullptr, nullptr}};
  hipEvent_t* ev = evs[0];   // the set of the call in progress
  int ev_set = 0, ev_done = 0;  // ev's set; the last completed call's
  float last_ms[3] = {0, 0, 0};  // first upload, compute span, last download of the last host-path call
  float last_total_ms = 0;       // whole pipelined host-path call (first H2D start -> last D2H end)
  bool timing_pending = false;   // ev[0..3] recorded, last_ms not yet read from them (resolve_timing)
  uint32_t chunk_grants = 0;     // host-path chunk target (grants), mochi_ctx_set_chunk_grants
  uint32_t small_grants = 4096;  // small-batch launch sequence up to this many grants (mochi_ctx_set_small_batch)
  // Write2 wire path: server-id table + decode scratch
  DevBuf ids, id_off;
  uint32_t n_ids = 0;
  std::vector<std::string> server_ids;  // host copy for the fallback decoder (w2_host.cpp)
  DevBuf w2_cnt, w2_status, w2_scan, w2_goff, w2_glen, w2_sig, w2_signer, w2_gkey, w2_okey, w2_oflags, w2_sigsrc,
      w2_mgo, w2_ots, w2_okoff, w2_oklen, w2_same;
  PinnedBuf w2_tot;
  hipEvent_t ev_tot = nullptr;
  // the last host-path call's certificate accept bitmap on the device (a slice
  // of dev_out, valid until the next call on this context; nullptr when the
  // device copy is not the final verdict, e.g. after host fallback decisions):
  // multi.cpp all-gathers it in place of re-uploading the host bits
  const uint32_t* acc_dev = nullptr;
  uint32_t acc_words = 0;
  uint64_t gen = 0;  // bumped (under mu) by every call that may rewrite dev_out / scratch
  // per-stage profiling (mochi_ctx_set_profiling): one event set per verify call
  bool profiling = false;
  std::vector<std::vector<hipEvent_t>> prof_sets;
};

namespace mochi {
// batcher.cpp: a batcher holds each of its contexts from create to its free
void ctx_hold(mochi_ctx* c) {
  std::lock_guard<std::mutex> lk(c->ref_mu);
  c->batcher_refs++;
}
void ctx_free(mochi_ctx* c);
// Nothing touches c after the unlock unless this release is the one that frees
// it (refs reached 0 with a destroy pending: no other thread may still use c).
void ctx_release(mochi_ctx* c) {
  bool free_now;
  {
    std::lock_guard<std::mutex> lk(c->ref_mu);
    free_now = --c->batcher_refs == 0 && c->destroy_pending;
  }
  if (free_now) ctx_free(c);
}

// the generation of the last context call made by this thread (multi.cpp reads it
// right after its mochi_verify_* returns, on the same thread)
thread_local uint64_t t_ctx_gen = 0;
uint64_t ctx_call_gen() { return t_ctx_gen; }

// Copies the certificate accept bitmap of context call `gen` from the device
// (where that call left it) into dst on `st`, holding the context's lock until
// the copy is done, so no later call can grow or overwrite dev_out under it.
// 1 = not available (a later call ran, the call's device bitmap is not final,
// or it lives on another device): the caller uploads its host bits instead.
int ctx_copy_accept_dev(mochi_ctx* c, uint64_t gen, int device, uint32_t* dst, uint32_t need, hipStream_t st) {
  std::lock_guard<std::mutex> lk(c->mu);
  if (c->gen != gen || !c->acc_dev || c->device != device || c->acc_words < need) return 1;
  if (hipMemcpyAsync(dst, c->acc_dev, 4 * (size_t)need, hipMemcpyDeviceToDevice, st) != hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess)
    return MOCHI_EHIP;
  return MOCHI_OK;
}
}  // namespace mochi

namespace {
// every entry point that launches on the context's buffers, with c->mu held
void new_call(mochi_ctx* c) {
  c->gen++;
  c->acc_dev = nullptr;
  c->acc_words = 0;
  mochi::t_ctx_gen = c->gen;
}
}  // namespace

extern "C" {

int mochi_abi_version(void) { return MOCHI_ABI_VERSION; }

const char* mochi_last_error(void) { return g_err.c_str(); }

int mochi_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

// The grant-prep stream runs at the highest priority, so its blocks take each
// CU the moment k_rsa_pow's block there retires (kernels.hip:launch_verify).
static hipError_t create_prep_stream(hipStream_t* s) {
  int least = 0, greatest = 0;
  if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess)
    return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, greatest);
}

mochi_ctx* mochi_ctx_create(int device, const uint8_t* moduli_be, uint32_t n_keys, uint32_t key_bytes,
                            uint32_t public_exponent) {
  if (!moduli_be || n_keys == 0 || n_keys > MOCHI_MAX_KEYS) {
    fail(MOCHI_EINVAL, "n_keys must be in [1, %d]", MOCHI_MAX_KEYS);
    return nullptr;
  }
  if (key_bytes != MOCHI_RSA_BYTES) {
    fail(MOCHI_EINVAL, "key_bytes must be %d (RSA-2048)", MOCHI_RSA_BYTES);
    return nullptr;
  }
  if (public_exponent != MOCHI_RSA_E) {
    fail(MOCHI_EINVAL, "public_exponent must be 65537");
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    fail(MOCHI_ENODEV, "no HIP device visible");
    return nullptr;
  }
  if (device < 0 || device >= ndev) {
    fail(MOCHI_ENODEV, "device %d out of range (%d visible)", device, ndev);
    return nullptr;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) != hipSuccess || strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    fail(MOCHI_ENODEV, "device %d is not gfx950 (%s)", device, prop.gcnArchName);
    return nullptr;
  }
  std::vector<mochi::KeyEntry> table(n_keys);
  std::vector<mochi::FoldKey> fold(n_keys);
  for (uint32_t k = 0; k < n_keys; k++)
    if (make_key_entry(moduli_be + (size_t)k * MOCHI_RSA_BYTES, &table[k]) != MOCHI_OK ||
        make_fold_key(moduli_be + (size_t)k * MOCHI_RSA_BYTES, &fold[k]) != MOCHI_OK)
      return nullptr;
  mochi_ctx* c = new mochi_ctx;
  c->device = device;
  c->n_keys = n_keys;
  c->chunk_grants = default_chunk_grants();
  int save = 0;
  (void)hipGetDevice(&save);
  bool ok = hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) == hipSuccess &&
            hipStreamCreateWithFlags(&c->s_in, hipStreamNonBlocking) == hipSuccess &&
            create_prep_stream(&c->aux) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_fork, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_join, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_scratch, hipEventDisableTiming) == hipSuccess &&
            hipEventCreateWithFlags(&c->ev_tot, hipEventDisableTiming) == hipSuccess &&
            hipStreamCreateWithFlags(&c->s_out, hipStreamNonBlocking) == hipSuccess &&
            hipMalloc(&c->d_keys, sizeof(mochi::KeyEntry) * n_keys) == hipSuccess &&
            hipMemcpy(c->d_keys, table.data(), sizeof(mochi::KeyEntry) * n_keys, hipMemcpyHostToDevice) == hipSuccess &&
            hipMalloc(&c->d_fold, sizeof(mochi::FoldKey) * n_keys) == hipSuccess &&
            hipMemcpy(c->d_fold, fold.data(), sizeof(mochi::FoldKey) * n_keys, hipMemcpyHostToDevice) == hipSuccess;
  for (int i = 0; i < 8 && ok; i++) ok = hipEventCreate(&c->evs[i / 4][i % 4]) == hipSuccess;
  (void)hipSetDevice(save);
  if (!ok) {
    fail(MOCHI_EHIP, "context setup failed on device %d", device);
    mochi_ctx_destroy(c);
    return nullptr;
  }
  return c;
}

void mochi_ctx_destroy(mochi_ctx* c) {
  if (!c) return;
  {  // a batcher on this context still alive (its deferred teardown not yet done, or
     // the caller closed the context before the batcher): the last release frees it
    std::lock_guard<std::mutex> lk(c->ref_mu);
    if (c->batcher_refs > 0) {
      c->destroy_pending = true;
      return;
    }
  }
  mochi::ctx_free(c);
}

}  // extern "C"

void mochi::ctx_free(mochi_ctx* c) {
  int save = 0;
  (void)hipGetDevice(&save);
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->s_out) (void)hipStreamSynchronize(c->s_out);
  for (auto& set : c->evs)
    for (auto& e : set)
      if (e) (void)hipEventDestroy(e);
  for (auto& e : c->chunk_ev) (void)hipEventDestroy(e);
  for (auto& e : c->tot_ev) (void)hipEventDestroy(e);
  if (c->aux) (void)hipStreamSynchronize(c->aux);
  if (c->s_in) (void)hipStreamDestroy(c->s_in);
  if (c->aux) (void)hipStreamDestroy(c->aux);
  if (c->ev_fork) (void)hipEventDestroy(c->ev_fork);
  if (c->ev_join) (void)hipEventDestroy(c->ev_join);
  if (c->ev_scratch) (void)hipEventDestroy(c->ev_scratch);
  if (c->ev_tot) (void)hipEventDestroy(c->ev_tot);
  if (c->s_out) (void)hipStreamDestroy(c->s_out);
  if (c->d_keys) (void)hipFree(c->d_keys);
  if (c->d_fold) (void)hipFree(c->d_fold);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  delete c;
  (void)hipSetDevice(save);
}

namespace {

int check_batch_header(const mochi_ctx* c, const mochi_batch* b, const mochi_params* p, const mochi_verdicts* o) {
  if (!c || !b || !p || !o) return fail(MOCHI_EINVAL, "null argument");
  if (!o->cert_accept_bits && b->n_certs) return fail(MOCHI_EINVAL, "cert_accept_bits is required");
  if (p->replication_factor == 0) return fail(MOCHI_EINVAL, "replication_factor must be > 0");
  if (b->n_grants && (!b->grant_bytes || !b->grant_off || !b->grant_len || !b->sig || !b->signer || !b->grant_key))
    return fail(MOCHI_EINVAL, "grant arrays must be non-null when n_grants > 0");
  if (!b->cert_grant_off || !b->cert_op_off) return fail(MOCHI_EINVAL, "cert_grant_off / cert_op_off required");
  if (b->n_certs && !b->expected_hash) return fail(MOCHI_EINVAL, "expected_hash required");
  if (b->n_ops && (!b->op_key || !b->op_flags)) return fail(MOCHI_EINVAL, "op arrays required");
  if ((b->cert_mg_off == nullptr) != (b->mg_grant_off == nullptr))
    return fail(MOCHI_EINVAL, "cert_mg_off and mg_grant_off go together");
  if (!b->cert_mg_off && b->n_mgs) return fail(MOCHI_EINVAL, "n_mgs must be 0 without cert_mg_off");
  if ((p->quorum_mode & MOCHI_Q_BIND) && b->n_ops && (!b->op_key_off || !b->op_key_len))
    return fail(MOCHI_EINVAL, "MOCHI_Q_BIND needs op_key_off / op_key_len");
  if (p->quorum_mode & ~(uint32_t)(MOCHI_Q_DISTINCT_SIGNERS | MOCHI_Q_BIND))
    return fail(MOCHI_EINVAL, "unknown quorum_mode bits 0x%x", p->quorum_mode);
  return MOCHI_OK;
}

// Host-side consistency checks (host path only; the device path trusts the caller's device arrays).
int check_batch_host(const mochi_batch* b) {
  if (b->cert_grant_off[0] != 0 || b->cert_grant_off[b->n_certs] != b->n_grants)
    return fail(MOCHI_EINVAL, "cert_grant_off must start at 0 and end at n_grants");
  if (b->cert_op_off[0] != 0 || b->cert_op_off[b->n_certs] != b->n_ops)
    return fail(MOCHI_EINVAL, "cert_op_off must start at 0 and end at n_ops");
  for (uint32_t c = 0; c < b->n_certs; c++) {
    if (b->cert_grant_off[c + 1] < b->cert_grant_off[c] || b->cert_op_off[c + 1] < b->cert_op_off[c])
      return fail(MOCHI_EINVAL, "CSR offsets must be non-decreasing (cert %u)", c);
    if (b->cert_op_off[c + 1] - b->cert_op_off[c] > MOCHI_MAX_OPS_PER_CERT)
      return fail(MOCHI_EINVAL, "cert %u has more than %d ops", c, MOCHI_MAX_OPS_PER_CERT);
  }
  for (uint32_t i = 0; i < b->n_grants; i++) {
    if (b->grant_len[i] > 65536) return fail(MOCHI_EINVAL, "grant %u longer than 65536 bytes", i);
    if (b->grant_off[i] > b->grant_bytes_len || b->grant_len[i] > b->grant_bytes_len - b->grant_off[i])
      return fail(MOCHI_EINVAL, "grant %u lies outside grant_bytes", i);
  }
  for (uint32_t o = 0; o < b->n_ops; o++) {
    if (b->op_key[o] >= MOCHI_MAX_OPS_PER_CERT) return fail(MOCHI_EINVAL, "op_key[%u] >= %d", o, MOCHI_MAX_OPS_PER_CERT);
    if (b->op_key_off && (b->op_key_off[o] > b->grant_bytes_len || b->op_key_len[o] > b->grant_bytes_len - b->op_key_off[o]))
      return fail(MOCHI_EINVAL, "op key %u lies outside grant_bytes", o);
  }
  if (b->cert_mg_off) {
    if (b->cert_mg_off[0] != 0 || b->cert_mg_off[b->n_certs] != b->n_mgs)
      return fail(MOCHI_EINVAL, "cert_mg_off must start at 0 and end at n_mgs");
    if (b->mg_grant_off[0] != 0 || b->mg_grant_off[b->n_mgs] != b->n_grants)
      return fail(MOCHI_EINVAL, "mg_grant_off must start at 0 and end at n_grants");
    for (uint32_t m = 0; m < b->n_mgs; m++)
      if (b->mg_grant_off[m + 1] < b->mg_grant_off[m]) return fail(MOCHI_EINVAL, "mg_grant_off decreases at %u", m);
    for (uint32_t c = 0; c < b->n_certs; c++)
      if (b->cert_mg_off[c + 1] < b->cert_mg_off[c] || b->mg_grant_off[b->cert_mg_off[c]] != b->cert_grant_off[c])
        return fail(MOCHI_EINVAL, "MultiGrants of cert %u do not cover its grants", c);
  }
  return MOCHI_OK;
}

// The last host-path call's spans, from its events (recorded during the call,
// read only when asked).
void resolve_timing(mochi_ctx* c) {
  if (!c->timing_pending) return;
  c->timing_pending = false;
  hipEvent_t* e = c->evs[c->ev_done];
  (void)hipEventElapsedTime(&c->last_ms[0], e[0], e[1]);
  (void)hipEventElapsedTime(&c->last_ms[1], e[1], e[2]);
  (void)hipEventElapsedTime(&c->last_ms[2], e[2], e[3]);
  (void)hipEventElapsedTime(&c->last_total_ms, e[0], e[3]);
}

// Scratch ordering across calls and streams (see mochi_ctx::ev_scratch).
hipError_t scratch_acquire(mochi_ctx* c, hipStream_t st) {
  // on the stream that last released the scratch, stream order already holds
  // (a wait there is one more API call and barrier packet per small batch)
  return c->scratch_used && c->scratch_st != st ? hipStreamWaitEvent(st, c->ev_scratch, 0) : hipSuccess;
}
hipError_t scratch_release(mochi_ctx* c, hipStream_t st) {
  c->scratch_used = true;
  c->scratch_st = st;
  return hipEventRecord(c->ev_scratch, st);
}

int ensure_scratch(mochi_ctx* c, uint32_t N, uint32_t C);

int run_device(mochi_ctx* c, const mochi_batch* b, const mochi_params* p, mochi_verdicts* o, hipStream_t st,
               const uint32_t* op_out_off = nullptr, const uint32_t* grant_same = nullptr,
               const uint8_t* msg_status = nullptr) {
  const uint32_t N = b->n_grants, C = b->n_certs;
  const uint64_t slots = mochi::slot_capacity(N, c->n_keys);
  if (slots > 0xFFFFFFF0ull) return fail(MOCHI_EINVAL, "batch too large");
  int rc;
  if ((uint64_t)N + C > 0xFFFFFFF0ull) return fail(MOCHI_EINVAL, "batch too large");
  if ((rc = ensure_scratch(c, N, C))) return rc;
  mochi::LaunchArgs a;
  memset(&a, 0, sizeof a);
  a.n_grants = N;
  a.n_certs = C;
  a.n_keys = c->n_keys;
  a.n_slots = (uint32_t)slots;
  a.blob = b->grant_bytes;
  a.grant_off = b->grant_off;
  a.grant_len = b->grant_len;
  a.sig = b->sig;
  a.signer = b->signer;
  a.grant_key = b->grant_key;
  a.cert_grant_off = b->cert_grant_off;
  a.cert_op_off = b->cert_op_off;
  a.op_key = b->op_key;
  a.op_flags = b->op_flags;
  a.expected_hash = b->expected_hash;
  a.cert_mg_off = b->cert_mg_off;
  a.mg_grant_off = b->mg_grant_off;
  a.op_object_ts = b->op_object_ts;
  a.op_key_off = b->op_key_off;
  a.op_key_len = b->op_key_len;
  a.quorum_mode = p->quorum_mode;
  const uint32_t R = p->replication_factor;
  a.majority = 2 * (R / 3) + 1;  // ClusterConfiguration.getServerMajority  ClusterConfiguration.java:264-267
  a.strict_gt = p->strict_gt ? 1 : 0;
  a.keys = c->d_keys;
  a.fold = c->d_fold;
  a.digest = c->digest.as<uint32_t>();  // distinct prep results: N + C entries (kernels.h)
  a.n_dist = N + C;
  a.lead = c->lead.as<uint32_t>();
  a.ts = o->grant_ts ? o->grant_ts : c->ts.as<int64_t>();
  a.hash_off = c->hash_off.as<uint64_t>();
  a.hash_len = c->hash_len.as<uint32_t>();
  a.flags = o->grant_flags ? o->grant_flags : c->flags.as<uint8_t>();
  a.count = c->count.as<uint32_t>();
  a.cursor = c->cursor.as<uint32_t>();
  a.total = c->total.as<uint32_t>();
  a.perm = c->perm.as<uint32_t>();
  a.xbuf = c->xbuf.as<uint32_t>();
  a.rare = c->dedup.as<uint8_t>();
  a.small_grants = c->small_grants;
  a.grant_same = grant_same;
  a.grant_valid_bits = o->grant_valid_bits;
  a.cert_accept_bits = o->cert_accept_bits;
  a.cert_reason = o->cert_reason;
  a.cert_fail_op = o->cert_fail_op;
  a.op_decision = o->op_decision;
  a.op_g0 = o->op_g0;
  a.op_ts = o->op_ts;
  a.op_out_off = op_out_off;
  a.msg_status = msg_status;
  a.aux = prep_serial() ? nullptr : c->aux;  // MOCHI_PREP_SERIAL=1: prep on the launch stream (A/B)
  a.ev_fork = c->ev_fork;
  a.ev_join = c->ev_join;
  if (c->profiling) {
    std::vector<hipEvent_t> evs(2 * mochi::kProfStages, nullptr);
    for (auto& e : evs) HIP_TRY(hipEventCreate(&e));
    c->prof_sets.push_back(evs);
    a.prof_events = c->prof_sets.back().data();
  }
  HIP_TRY(scratch_acquire(c, st));
  HIP_TRY(mochi::launch_verify(a, st));
  HIP_TRY(scratch_release(c, st));
  return MOCHI_OK;
}

// ---- host path: chunked H2D / compute / D2H pipeline ------------------------
//
// The batch is cut at certificate boundaries (multiples of 32 certificates, so
// every chunk's accept bits start on a word) into chunks of ~kChunkGrants
// grants.  Chunk j's inputs go up on the copy-in stream, its kernels run on the
// context stream once they have landed, and its verdicts come down on the
// copy-out stream while chunk j+1 computes.  Every chunk has its own input
// region on the device and writes disjoint output slices, so the only
// cross-stream ordering is one event per hand-off.  Sources that are already
// pinned (mochi_host_alloc) are DMA'd in place; others are staged through the
// context's pinned buffer with a parallel memcpy.
bool is_pinned(const void* ptr) {
  if (!ptr) return false;
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, ptr) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

void par_memcpy(void* dst, const void* src, size_t n) {
  constexpr size_t kPar = 8u << 20;
  if (n < kPar) {
    memcpy(dst, src, n);
    return;
  }
  const unsigned hw = std::thread::hardware_concurrency();
  const unsigned nt = hw < 2 ? 1 : hw > 8 ? 8 : hw;
  const size_t per = (n + nt - 1) / nt;
  std::vector<std::thread> th;
  for (unsigned t = 1; t < nt; t++) {
    const size_t lo = t * per;
    if (lo >= n) break;
    const size_t len = per < n - lo ? per : n - lo;
    th.emplace_back([=] { memcpy((char*)dst + lo, (const char*)src + lo, len); });
  }
  memcpy(dst, src, per < n ? per : n);
  for (auto& x : th) x.join();
}

// Verify scratch for N grants of C certificates: per grant (ts, flags, rare,
// lead), per distinct prep result (N + C: digest, hash slice), per slot (perm, z).
int ensure_scratch(mochi_ctx* c, uint32_t N, uint32_t C) {
  const uint64_t slots = mochi::slot_capacity(N, c->n_keys);
  const size_t ND = (size_t)N + C;
  int rc;
  if ((rc = c->digest.ensure(sizeof(uint32_t) * 8 * ND)) || (rc = c->dedup.ensure((size_t)N)) ||
      (rc = c->ts.ensure(sizeof(int64_t) * (size_t)N)) || (rc = c->hash_off.ensure(sizeof(uint64_t) * ND)) ||
      (rc = c->hash_len.ensure(sizeof(uint32_t) * ND)) || (rc = c->flags.ensure((size_t)N)) ||
      (rc = c->lead.ensure(sizeof(uint32_t) * (size_t)N)) ||
      (rc = c->count.ensure(sizeof(uint32_t) * c->n_keys)) || (rc = c->cursor.ensure(sizeof(uint32_t) * c->n_keys)) ||
      (rc = c->total.ensure(mochi::kTotalWords * sizeof(uint32_t))) || (rc = c->perm.ensure(sizeof(uint32_t) * (size_t)slots)) ||
      (rc = c->xbuf.ensure(sizeof(uint32_t) * mochi::kL * (size_t)slots)))
    return rc;
  return MOCHI_OK;
}

// Input segments of one chunk, in mochi_batch order.  The CSR arrays (6, 7,
// 11, 12) are rebased per chunk and therefore always staged.
enum Seg {
  kBlob, kGrantOff, kGrantLen, kSig, kSigner, kGrantKey, kCertGrantOff, kCertOpOff, kOpKey, kOpFlags, kExpHash,
  kCertMgOff, kMgGrantOff, kOpObjTs, kOpKeyOff, kOpKeyLen, kNumSeg
};

int run_host_pipeline(mochi_ctx* c, const mochi_batch* b, const mochi_params* p, mochi_verdicts* o) {
  const uint32_t N = b->n_grants, C = b->n_certs, O = b->n_ops;
  c->acc_dev = nullptr;
  c->acc_words = 0;
  const bool mg = b->cert_mg_off != nullptr;
  // --- plan chunks ---
  struct Chunk {
    uint32_t c0, c1, g0, g1, o0, o1, m0, m1;
    uint64_t lo, hi;  // byte range [lo, hi) of grant_bytes this chunk reads
    size_t seg[kNumSeg];
  };
  std::vector<Chunk> ch;
  uint32_t max_grants = 0, max_certs = 0;
  for (uint32_t c0 = 0; c0 < C || (C == 0 && ch.empty());) {
    uint32_t c1 = c0;
    do c1 = c1 + 32 < C ? c1 + 32 : C;
    while (c1 < C && b->cert_grant_off[c1] - b->cert_grant_off[c0] < c->chunk_grants);
    Chunk k{};
    k.c0 = c0;
    k.c1 = c1;
    k.g0 = b->cert_grant_off[c0];
    k.g1 = b->cert_grant_off[c1];
    k.o0 = b->cert_op_off[c0];
    k.o1 = b->cert_op_off[c1];
    k.m0 = mg ? b->cert_mg_off[c0] : 0;
    k.m1 = mg ? b->cert_mg_off[c1] : 0;
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t g = k.g0; g < k.g1; g++) {
      lo = b->grant_off[g] < lo ? b->grant_off[g] : lo;
      const uint64_t e = b->grant_off[g] + b->grant_len[g];
      hi = e > hi ? e : hi;
    }
    if (b->op_key_off)  // MOCHI_Q_BIND reads the op keys from the blob too
      for (uint32_t x = k.o0; x < k.o1; x++) {
        lo = b->op_key_off[x] < lo ? b->op_key_off[x] : lo;
        const uint64_t e = b->op_key_off[x] + b->op_key_len[x];
        hi = e > hi ? e : hi;
      }
    if (lo == UINT64_MAX) lo = hi = 0;  // nothing read from the blob
    k.lo = lo;
    k.hi = hi;
    if (k.g1 - k.g0 > max_grants) max_grants = k.g1 - k.g0;
    if (k.c1 - k.c0 > max_certs) max_certs = k.c1 - k.c0;
    ch.push_back(k);
    if (C == 0) break;
    c0 = c1;
  }
  const size_t nchunks = ch.size();
  auto seg_bytes = [&](const Chunk& k, int i) -> size_t {
    const size_t ng = k.g1 - k.g0, nc = k.c1 - k.c0, no = k.o1 - k.o0, nm = k.m1 - k.m0;
    switch (i) {
      case kBlob: return (size_t)(k.hi - k.lo);
      case kGrantOff: return sizeof(uint64_t) * ng;
      case kGrantLen: return sizeof(uint32_t) * ng;
      case kSig: return (size_t)MOCHI_RSA_BYTES * ng;
      case kSigner: return sizeof(uint16_t) * ng;
      case kGrantKey: return ng;
      case kCertGrantOff: case kCertOpOff: return sizeof(uint32_t) * (nc + 1);
      case kOpKey: case kOpFlags: return no;
      case kExpHash: return (size_t)MOCHI_TXN_HASH_BYTES * nc;
      case kCertMgOff: return mg ? sizeof(uint32_t) * (nc + 1) : 0;
      case kMgGrantOff: return mg ? sizeof(uint32_t) * (nm + 1) : 0;
      case kOpObjTs: return b->op_object_ts ? sizeof(int64_t) * no : 0;
      case kOpKeyOff: return b->op_key_off ? sizeof(uint64_t) * no : 0;
      default: return b->op_key_len ? sizeof(uint32_t) * no : 0;
    }
  };
  auto seg_src = [&](const Chunk& k, int i) -> const void* {
    switch (i) {
      case kBlob: return b->grant_bytes + k.lo;
      case kGrantOff: return b->grant_off + k.g0;
      case kGrantLen: return b->grant_len + k.g0;
      case kSig: return b->sig + (size_t)MOCHI_RSA_BYTES * k.g0;
      case kSigner: return b->signer + k.g0;
      case kGrantKey: return b->grant_key + k.g0;
      case kOpKey: return b->op_key + k.o0;
      case kOpFlags: return b->op_flags + k.o0;
      case kExpHash: return b->expected_hash + (size_t)MOCHI_TXN_HASH_BYTES * k.c0;
      case kOpObjTs: return b->op_object_ts ? b->op_object_ts + k.o0 : nullptr;
      case kOpKeyOff: return b->op_key_off ? b->op_key_off + k.o0 : nullptr;
      case kOpKeyLen: return b->op_key_len ? b->op_key_len + k.o0 : nullptr;
      default: return nullptr;  // rebased CSR, always staged
    }
  };
  auto rebased = [](int i) { return i == kCertGrantOff || i == kCertOpOff || i == kCertMgOff || i == kMgGrantOff; };
  size_t in_total = 0;
  for (auto& k : ch)
    for (int i = 0; i < kNumSeg; i++) {
      k.seg[i] = in_total;
      in_total = align_up(in_total + seg_bytes(k, i), 256);
    }
  // --- output layout: whole-batch slices ---
  const size_t nbits_g = ((size_t)N + 31) / 32 * 4, nbits_c = ((size_t)C + 31) / 32 * 4;
  size_t out_total = 0;
  auto take = [&](size_t bytes) {
    const size_t off = out_total;
    out_total = align_up(out_total + bytes, 256);
    return off;
  };
  const size_t o_flags = take(N), o_ts = take(o->grant_ts ? sizeof(int64_t) * N : 0), o_acc = take(nbits_c),
               o_reason = take(o->cert_reason ? C : 0), o_fail = take(o->cert_fail_op ? C : 0),
               o_gbits = take(o->grant_valid_bits ? nbits_g : 0), o_dec = take(o->op_decision ? O : 0),
               o_g0 = take(o->op_g0 ? sizeof(uint32_t) * O : 0), o_ots = take(o->op_ts ? sizeof(int64_t) * O : 0);
  int rc;
  if ((rc = c->pin_in.ensure(in_total)) || (rc = c->dev_in.ensure(in_total)) || (rc = c->pin_out.ensure(out_total)) ||
      (rc = c->dev_out.ensure(out_total)) || (rc = ensure_scratch(c, max_grants, max_certs)))
    return rc;
  while (c->chunk_ev.size() < 2 * nchunks) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->chunk_ev.push_back(e);
  }
  bool pinned[kNumSeg];
  for (int i = 0; i < kNumSeg; i++) pinned[i] = !rebased(i) && is_pinned(seg_src(ch[0], i));
  uint8_t* pin = (uint8_t*)c->pin_in.p;
  uint8_t* din = c->dev_in.as<uint8_t>();
  uint8_t* dout = c->dev_out.as<uint8_t>();
  uint8_t* pout = (uint8_t*)c->pin_out.p;
  hipStream_t st = c->stream;
  c->ev_set ^= 1;  // this call's span events: the other set keeps the last call's
  c->ev = c->evs[c->ev_set];
  HIP_TRY(hipEventRecord(c->ev[0], c->s_in));
  for (size_t j = 0; j < nchunks; j++) {
    Chunk& k = ch[j];
    // stage + upload
    uint32_t* cg = (uint32_t*)(pin + k.seg[kCertGrantOff]);
    uint32_t* co = (uint32_t*)(pin + k.seg[kCertOpOff]);
    for (uint32_t x = k.c0; x <= k.c1; x++) {
      cg[x - k.c0] = b->cert_grant_off[x] - k.g0;
      co[x - k.c0] = b->cert_op_off[x] - k.o0;
    }
    if (mg) {
      uint32_t* cm = (uint32_t*)(pin + k.seg[kCertMgOff]);
      uint32_t* mo = (uint32_t*)(pin + k.seg[kMgGrantOff]);
      for (uint32_t x = k.c0; x <= k.c1; x++) cm[x - k.c0] = b->cert_mg_off[x] - k.m0;
      for (uint32_t x = k.m0; x <= k.m1; x++) mo[x - k.m0] = b->mg_grant_off[x] - k.g0;
    }
    for (int i = 0; i < kNumSeg; i++) {
      const size_t n = seg_bytes(k, i);
      if (!n) continue;
      const void* src = pin + k.seg[i];
      if (pinned[i]) src = seg_src(k, i);
      else if (!rebased(i)) par_memcpy(pin + k.seg[i], seg_src(k, i), n);
      HIP_TRY(hipMemcpyAsync(din + k.seg[i], src, n, hipMemcpyHostToDevice, c->s_in));
    }
    HIP_TRY(hipEventRecord(c->chunk_ev[2 * j], c->s_in));
    // compute
    HIP_TRY(hipStreamWaitEvent(st, c->chunk_ev[2 * j], 0));
    if (j == 0) HIP_TRY(hipEventRecord(c->ev[1], st));
    auto at = [&](int i) -> const void* { return seg_bytes(k, i) ? (const void*)(din + k.seg[i]) : nullptr; };
    mochi_batch db;
    memset(&db, 0, sizeof db);
    db.n_grants = k.g1 - k.g0;
    db.n_certs = k.c1 - k.c0;
    db.n_ops = k.o1 - k.o0;
    db.n_mgs = k.m1 - k.m0;
    db.grant_bytes_len = k.hi;
    db.grant_bytes = din + k.seg[kBlob] - k.lo;  // kernels add the absolute grant_off / op_key_off
    db.grant_off = (const uint64_t*)(din + k.seg[kGrantOff]);
    db.grant_len = (const uint32_t*)(din + k.seg[kGrantLen]);
    db.sig = din + k.seg[kSig];
    db.signer = (const uint16_t*)(din + k.seg[kSigner]);
    db.grant_key = din + k.seg[kGrantKey];
    db.cert_grant_off = (const uint32_t*)(din + k.seg[kCertGrantOff]);
    db.cert_op_off = (const uint32_t*)(din + k.seg[kCertOpOff]);
    db.op_key = din + k.seg[kOpKey];
    db.op_flags = din + k.seg[kOpFlags];
    db.expected_hash = din + k.seg[kExpHash];
    db.cert_mg_off = (const uint32_t*)at(kCertMgOff);
    db.mg_grant_off = (const uint32_t*)at(kMgGrantOff);
    db.op_object_ts = (const int64_t*)at(kOpObjTs);
    db.op_key_off = (const uint64_t*)at(kOpKeyOff);
    db.op_key_len = (const uint32_t*)at(kOpKeyLen);
    mochi_verdicts dv;
    memset(&dv, 0, sizeof dv);
    dv.grant_flags = dout + o_flags + k.g0;
    dv.grant_ts = o->grant_ts ? (int64_t*)(dout + o_ts) + k.g0 : nullptr;
    dv.cert_accept_bits = (uint32_t*)(dout + o_acc) + k.c0 / 32;
    dv.cert_reason = o->cert_reason ? dout + o_reason + k.c0 : nullptr;
    dv.cert_fail_op = o->cert_fail_op ? dout + o_fail + k.c0 : nullptr;
    dv.op_decision = o->op_decision ? dout + o_dec + k.o0 : nullptr;
    dv.op_g0 = o->op_g0 ? (uint32_t*)(dout + o_g0) + k.o0 : nullptr;
    dv.op_ts = o->op_ts ? (int64_t*)(dout + o_ots) + k.o0 : nullptr;
    if ((rc = run_device(c, &db, p, &dv, st))) return rc;
    if (j + 1 == nchunks && o->grant_valid_bits && N)
      HIP_TRY(mochi::launch_pack_bits(dout + o_flags, N, MOCHI_GRANT_SIG_OK, (uint32_t*)(dout + o_gbits), st));
    if (j + 1 == nchunks) HIP_TRY(hipEventRecord(c->ev[2], st));
    HIP_TRY(hipEventRecord(c->chunk_ev[2 * j + 1], st));
    // download this chunk's verdict slices
    HIP_TRY(hipStreamWaitEvent(c->s_out, c->chunk_ev[2 * j + 1], 0));
    auto down = [&](size_t off, size_t bytes) -> hipError_t {
      return bytes ? hipMemcpyAsync(pout + off, dout + off, bytes, hipMemcpyDeviceToHost, c->s_out) : hipSuccess;
    };
    if (nchunks == 1 && out_total <= (4u << 20)) {  // one small chunk: one download of the whole region
      HIP_TRY(down(0, out_total));
      continue;
    }
    const size_t ng = k.g1 - k.g0, nc = k.c1 - k.c0, no = k.o1 - k.o0;
    const size_t acc_words = j + 1 == nchunks ? nbits_c / 4 - k.c0 / 32 : nc / 32;
    if (o->grant_flags) HIP_TRY(down(o_flags + k.g0, ng));
    if (o->grant_ts) HIP_TRY(down(o_ts + sizeof(int64_t) * k.g0, sizeof(int64_t) * ng));
    HIP_TRY(down(o_acc + 4 * (size_t)(k.c0 / 32), 4 * acc_words));
    if (o->cert_reason) HIP_TRY(down(o_reason + k.c0, nc));
    if (o->cert_fail_op) HIP_TRY(down(o_fail + k.c0, nc));
    if (o->op_decision) HIP_TRY(down(o_dec + k.o0, no));
    if (o->op_g0) HIP_TRY(down(o_g0 + sizeof(uint32_t) * k.o0, sizeof(uint32_t) * no));
    if (o->op_ts) HIP_TRY(down(o_ots + sizeof(int64_t) * k.o0, sizeof(int64_t) * no));
    if (j + 1 == nchunks && o->grant_valid_bits) HIP_TRY(down(o_gbits, nbits_g));
  }
  HIP_TRY(hipEventRecord(c->ev[3], c->s_out));
  if (hipStreamSynchronize(c->s_out) != hipSuccess)
    return fail(MOCHI_EHIP, "stream sync failed: %s", hipGetErrorString(hipGetLastError()));
  // first upload (not overlapped), compute span, last download (not overlapped),
  // whole call: read from the events when asked (resolve_timing)
  c->ev_done = c->ev_set;
  c->timing_pending = true;
  void* dsts[] = {o->grant_flags, o->grant_ts, o->cert_accept_bits, o->cert_reason, o->cert_fail_op,
                  o->grant_valid_bits, o->op_decision, o->op_g0, o->op_ts};
  const size_t offs[] = {o_flags, o_ts, o_acc, o_reason, o_fail, o_gbits, o_dec, o_g0, o_ots};
  const size_t lens[] = {(size_t)N, sizeof(int64_t) * N, nbits_c, (size_t)C, (size_t)C, nbits_g,
                         (size_t)O, sizeof(uint32_t) * O, sizeof(int64_t) * O};
  for (int i = 0; i < 9; i++)
    if (dsts[i] && lens[i]) memcpy(dsts[i], pout + offs[i], lens[i]);
  c->acc_dev = (const uint32_t*)(dout + o_acc);
  c->acc_words = (uint32_t)(nbits_c / 4);
  return MOCHI_OK;
}

// ---- Write2ToServer wire path -------------------------------------------------
// Decode on the device (w2_decode.hip), then the ordinary verify path over the
// decoded batch, then the per-message status fix-up.  All pointers device.
// Decode, phase 1 (w2_decode.hip): validate + count + CSR scans for the M
// messages of `w`.  cnt: mochi::w2_scratch_words(M) device words (counts, CSR
// offsets and the level-by-level decode state of this batch, so a pipelined
// caller can count chunk j+1 while chunk j verifies);
// the totals (N, O, n_mgs) land in tot_host (pinned) once ev_tot completes.
int w2_count(mochi_ctx* c, const mochi_write2_batch* w, uint8_t* status, uint32_t* cnt, uint32_t* tot_host,
             hipEvent_t ev_tot, hipStream_t st, mochi::W2Args* a) {
  const uint32_t M = w->n_msgs;
  const size_t m1 = (size_t)M + 1;
  size_t scan_bytes = 0;  // a small batch needs none (and the size query is ~7 host API calls)
  if (!mochi::w2_small(M)) HIP_TRY(mochi::w2_scan_temp_bytes(M + 1, &scan_bytes));
  if (scan_bytes > c->w2_scan.cap) {
    HIP_TRY(hipStreamSynchronize(st));  // the scan scratch may be in use by an earlier chunk
    int rc = c->w2_scan.ensure(scan_bytes);
    if (rc) return rc;
  }
  memset(a, 0, sizeof *a);
  a->wire = w->wire;
  a->msg_off = w->msg_off;
  a->msg_len = w->msg_len;
  a->M = M;
  a->flags_off = w->op_flags_off;
  a->flags_in = w->op_flags;
  a->ots_in = w->op_object_ts;
  a->ids = c->ids.as<uint8_t>();
  a->id_off = c->id_off.as<uint32_t>();
  a->n_ids = c->n_ids;
  a->cnt_g = cnt;
  a->cnt_o = cnt + m1;
  a->cnt_m = cnt + 2 * m1;
  a->cert_grant_off = cnt + 3 * m1;
  a->cert_op_off = cnt + 4 * m1;
  a->cert_mg_off = cnt + 5 * m1;
  a->cnt_ce = cnt + 6 * m1;
  a->ce = cnt + (size_t)mochi::kW2MsgArrays * m1;
  a->ce_cap = mochi::kW2MaxCertEntries * (uint32_t)m1;
  a->inl = (uint32_t*)(((uintptr_t)(a->ce + mochi::kW2CeArrays * (size_t)a->ce_cap) + 15) & ~(uintptr_t)15);
  a->inl_ops = a->inl + 4 * (size_t)mochi::kW2InlEntries * m1;
  a->cnt4 = a->inl_ops + 2 * (size_t)mochi::kW2InlOps * m1;  // 16-byte aligned: the two above are multiples of 4 words
  a->off4 = a->cnt4 + 4 * m1;
  a->status = status;
  a->scan_temp = c->w2_scan.p;
  a->scan_temp_bytes = c->w2_scan.cap;
  HIP_TRY(mochi::launch_w2_count(*a, st));
  // decoded grants, ops and MultiGrants: the packed scan's last element
  HIP_TRY(hipMemcpyAsync(tot_host, a->off4 + 4 * (size_t)M, 12, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipEventRecord(ev_tot, st));
  return MOCHI_OK;
}

// Grow a decode buffer; if it must be reallocated, first let the stream drain
// (an earlier chunk's kernels may still read the old allocation).
int grow(DevBuf& b, size_t bytes, hipStream_t st) {
  if (bytes <= b.cap) return MOCHI_OK;
  HIP_TRY(hipStreamSynchronize(st));
  return b.ensure(bytes);
}

// Decode, phase 2: emit the SoA batch (N grants, O ops, NM MultiGrants from
// phase 1), then the verify path and the per-message status fix-up.  Per-op
// outputs follow the caller's op_flags_off layout (`op_out_off`, device).
int w2_verify(mochi_ctx* c, const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* o,
              mochi::W2Args& a, uint32_t N, uint32_t O, uint32_t NM, const uint32_t* op_out_off, hipStream_t st,
              bool decode_only) {
  int rc;
  if ((rc = grow(c->w2_goff, 8 * (size_t)N, st)) || (rc = grow(c->w2_glen, 4 * (size_t)N, st)) ||
      (rc = grow(c->w2_sig, (size_t)MOCHI_RSA_BYTES * N, st)) || (rc = grow(c->w2_signer, 2 * (size_t)N, st)) ||
      (rc = grow(c->w2_gkey, N, st)) || (rc = grow(c->w2_okey, O, st)) || (rc = grow(c->w2_oflags, O, st)) ||
      (rc = grow(c->w2_sigsrc, 8 * (size_t)N, st)) || (rc = grow(c->w2_mgo, 4 * ((size_t)NM + 1), st)) ||
      (rc = grow(c->w2_ots, 8 * (size_t)O, st)) || (rc = grow(c->w2_okoff, 8 * (size_t)O, st)) ||
      (rc = grow(c->w2_oklen, 4 * (size_t)O, st)) || (rc = grow(c->w2_same, 4 * (size_t)N, st)))
    return rc;
  if (!decode_only) {  // the verify scratch grows only once the stream has drained
    const uint64_t slots = mochi::slot_capacity(N, c->n_keys);
    if (sizeof(uint32_t) * mochi::kL * slots > c->xbuf.cap || sizeof(uint32_t) * 8 * ((size_t)N + a.M) > c->digest.cap ||
        sizeof(uint32_t) * (size_t)N > c->lead.cap)
      HIP_TRY(hipStreamSynchronize(st));
    if ((rc = ensure_scratch(c, N, a.M))) return rc;
  }
  a.N = N;
  a.sig_src = c->w2_sigsrc.as<uint64_t>();
  a.grant_off = c->w2_goff.as<uint64_t>();
  a.grant_len = c->w2_glen.as<uint32_t>();
  a.sig = c->w2_sig.as<uint8_t>();
  a.signer = c->w2_signer.as<uint16_t>();
  a.grant_key = c->w2_gkey.as<uint8_t>();
  a.op_key = c->w2_okey.as<uint8_t>();
  a.op_flags = c->w2_oflags.as<uint8_t>();
  a.op_object_ts = c->w2_ots.as<int64_t>();
  a.op_key_off = c->w2_okoff.as<uint64_t>();
  a.op_key_len = c->w2_oklen.as<uint32_t>();
  a.mg_grant_off = c->w2_mgo.as<uint32_t>();
  a.grant_same = c->w2_same.as<uint32_t>();
  HIP_TRY(mochi::launch_w2_emit(a, st));
  if (decode_only) return MOCHI_OK;
  mochi_batch db;
  memset(&db, 0, sizeof db);
  db.n_grants = N;
  db.n_certs = a.M;
  db.n_ops = O;
  db.n_mgs = NM;
  db.grant_bytes_len = w->wire_len;
  db.grant_bytes = w->wire;
  db.grant_off = a.grant_off;
  db.grant_len = a.grant_len;
  db.sig = a.sig;
  db.signer = a.signer;
  db.grant_key = a.grant_key;
  db.cert_grant_off = a.cert_grant_off;
  db.cert_op_off = a.cert_op_off;
  db.op_key = a.op_key;
  db.op_flags = a.op_flags;
  db.expected_hash = w->expected_hash;
  db.cert_mg_off = a.cert_mg_off;
  db.mg_grant_off = a.mg_grant_off;
  db.op_object_ts = a.op_object_ts;
  db.op_key_off = a.op_key_off;
  db.op_key_len = a.op_key_len;
  mochi_verdicts dv;
  memset(&dv, 0, sizeof dv);
  dv.cert_accept_bits = o->cert_accept_bits;
  dv.cert_reason = o->cert_reason;
  dv.cert_fail_op = o->cert_fail_op;
  dv.op_decision = o->op_decision;
  dv.op_g0 = o->op_g0;
  dv.op_ts = o->op_ts;
  // the status fix-up of undecoded messages runs inside k_tally (one launch
  // fewer at the end of the call); MOCHI_W2_FIXUP_KERNEL=1 (A/B): as its own kernel
  const bool fused = !fixup_kernel();
  if ((rc = run_device(c, &db, p, &dv, st, op_out_off, a.grant_same, fused ? a.status : nullptr))) return rc;
  if (!fused)
    HIP_TRY(mochi::launch_w2_fixup(a, o->cert_accept_bits, o->cert_reason, o->cert_fail_op, o->op_decision, o->op_g0,
                                   o->op_ts, st));
  return MOCHI_OK;
}

// Device-resident wire batch, one shot (mochi_verify_write2_device).
int run_write2_device(mochi_ctx* c, const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* o,
                      uint8_t* status, hipStream_t st) {
  const uint32_t M = w->n_msgs;
  if (c->n_ids != c->n_keys) return fail(MOCHI_EINVAL, "server ids not set (mochi_ctx_set_server_ids)");
  int rc;
  if ((rc = c->w2_cnt.ensure(4 * mochi::w2_scratch_words(M))) || (rc = c->w2_tot.ensure(16)) ||
      (!status && (rc = c->w2_status.ensure(M ? M : 1))))
    return rc;
  HIP_TRY(scratch_acquire(c, st));
  mochi::W2Args a;
  uint32_t* tot = (uint32_t*)c->w2_tot.p;
  if ((rc = w2_count(c, w, status ? status : c->w2_status.as<uint8_t>(), c->w2_cnt.as<uint32_t>(), tot, c->ev_tot, st, &a)))
    return rc;
  HIP_TRY(hipEventSynchronize(c->ev_tot));
  if ((rc = w2_verify(c, w, p, o, a, tot[0], tot[1], tot[2], w->op_flags_off, st, false))) return rc;
  HIP_TRY(scratch_release(c, st));
  return MOCHI_OK;
}

int check_write2_header(const mochi_ctx* c, const mochi_write2_batch* w, const mochi_params* p,
                        const mochi_verdicts* o) {
  if (!c || !w || !p || !o) return fail(MOCHI_EINVAL, "null argument");
  if (o->grant_valid_bits || o->grant_flags || o->grant_ts)
    return fail(MOCHI_EINVAL, "grant-level outputs are not produced on the Write2 wire path");
  if (w->n_msgs && (!o->cert_accept_bits || !w->wire || !w->msg_off || !w->msg_len || !w->expected_hash))
    return fail(MOCHI_EINVAL, "wire / msg_off / msg_len / expected_hash / cert_accept_bits required");
  if (w->op_flags_off && !w->op_flags) return fail(MOCHI_EINVAL, "op_flags required with op_flags_off");
  if ((o->op_decision || o->op_g0 || o->op_ts) && !w->op_flags_off)
    return fail(MOCHI_EINVAL, "per-op outputs on the wire path need op_flags_off (their layout)");
  if (w->op_object_ts && !w->op_flags_off) return fail(MOCHI_EINVAL, "op_object_ts needs op_flags_off");
  if ((p->quorum_mode & ~(uint32_t)(MOCHI_Q_DISTINCT_SIGNERS | MOCHI_Q_BIND)) != 0)
    return fail(MOCHI_EINVAL, "unknown quorum_mode bits 0x%x", p->quorum_mode);
  if (p->replication_factor == 0) return fail(MOCHI_EINVAL, "replication_factor must be > 0");
  return MOCHI_OK;
}

}  // namespace

extern "C" {

int mochi_verify_batch_device(mochi_ctx* c, const mochi_batch* b, const mochi_params* p, mochi_verdicts* o,
                              void* stream) {
  int rc = check_batch_header(c, b, p, o);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(c->device) != hipSuccess) return fail(MOCHI_EHIP, "hipSetDevice(%d)", c->device);
  new_call(c);
  rc = run_device(c, b, p, o, (hipStream_t)stream);  // NULL = the null stream, as in HIP
  (void)hipSetDevice(save);
  return rc;
}

int mochi_verify_batch(mochi_ctx* c, const mochi_batch* b, const mochi_params* p, mochi_verdicts* o) {
  int rc = check_batch_header(c, b, p, o);
  if (rc) return rc;
  if ((rc = check_batch_host(b))) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(c->device) != hipSuccess) return fail(MOCHI_EHIP, "hipSetDevice(%d)", c->device);
  new_call(c);
  rc = run_host_pipeline(c, b, p, o);
  (void)hipSetDevice(save);
  return rc;
}

void* mochi_host_alloc(uint64_t bytes) {
  void* ptr = nullptr;
  if (hipHostMalloc(&ptr, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
    fail(MOCHI_ENOMEM, "hipHostMalloc(%llu) failed", (unsigned long long)bytes);
    return nullptr;
  }
  return ptr;
}

void mochi_host_free(void* ptr) {
  if (ptr) (void)hipHostFree(ptr);
}

int mochi_ctx_set_small_batch(mochi_ctx* c, uint32_t grants) {
  if (!c) return fail(MOCHI_EINVAL, "null context");
  std::lock_guard<std::mutex> lk(c->mu);
  c->small_grants = grants;
  return MOCHI_OK;
}

int mochi_ctx_set_chunk_grants(mochi_ctx* c, uint32_t grants) {
  if (!c) return fail(MOCHI_EINVAL, "null context");
  std::lock_guard<std::mutex> lk(c->mu);
  c->chunk_grants = grants ? grants : default_chunk_grants();
  return MOCHI_OK;
}

int mochi_ctx_last_total_ms(mochi_ctx* c, float* total_ms) {
  if (!c || !total_ms) return fail(MOCHI_EINVAL, "null argument");
  resolve_timing(c);
  *total_ms = c->last_total_ms;
  return MOCHI_OK;
}

int mochi_ctx_set_server_ids(mochi_ctx* c, const uint8_t* ids, const uint32_t* id_off, uint32_t n_ids) {
  if (!c || !ids || !id_off) return fail(MOCHI_EINVAL, "null argument");
  if (n_ids != c->n_keys) return fail(MOCHI_EINVAL, "n_ids (%u) must equal the key count (%u)", n_ids, c->n_keys);
  if (id_off[0] != 0) return fail(MOCHI_EINVAL, "id_off[0] must be 0");
  for (uint32_t i = 0; i < n_ids; i++)
    if (id_off[i + 1] < id_off[i] || id_off[i + 1] - id_off[i] > 256)
      return fail(MOCHI_EINVAL, "server id %u: bad length", i);
  std::lock_guard<std::mutex> lk(c->mu);
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(c->device) != hipSuccess) return fail(MOCHI_EHIP, "hipSetDevice(%d)", c->device);
  const size_t nb = id_off[n_ids];
  int rc = c->ids.ensure(nb ? nb : 1);
  if (!rc) rc = c->id_off.ensure(4 * ((size_t)n_ids + 1));
  if (!rc && nb && hipMemcpy(c->ids.p, ids, nb, hipMemcpyHostToDevice) != hipSuccess) rc = fail(MOCHI_EHIP, "copy ids");
  if (!rc && hipMemcpy(c->id_off.p, id_off, 4 * ((size_t)n_ids + 1), hipMemcpyHostToDevice) != hipSuccess)
    rc = fail(MOCHI_EHIP, "copy id_off");
  if (!rc) {
    c->n_ids = n_ids;
    c->server_ids.clear();
    for (uint32_t i = 0; i < n_ids; i++) c->server_ids.emplace_back((const char*)ids + id_off[i], id_off[i + 1] - id_off[i]);
  }
  (void)hipSetDevice(save);
  return rc;
}

int mochi_verify_write2_device(mochi_ctx* c, const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* o,
                               uint8_t* msg_status, void* stream) {
  int rc = check_write2_header(c, w, p, o);
  if (rc) return rc;
  std::lock_guard<std::mutex> lk(c->mu);
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(c->device) != hipSuccess) return fail(MOCHI_EHIP, "hipSetDevice(%d)", c->device);
  new_call(c);
  rc = run_write2_device(c, w, p, o, msg_status, (hipStream_t)stream);
  (void)hipSetDevice(save);
  return rc;
}

static int verify_write2_host(mochi_ctx* c, const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* o,
                              uint8_t* msg_status, mochi_write2_decoded* dec);

int mochi_verify_write2(mochi_ctx* c, const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* o,
                        uint8_t* msg_status) {
  int rc = check_write2_header(c, w, p, o);
  if (rc) return rc;
  return verify_write2_host(c, w, p, o, msg_status, nullptr);
}

int mochi_write2_decode(mochi_ctx* c, const mochi_write2_batch* w, mochi_write2_decoded* out) {
  if (!out) return fail(MOCHI_EINVAL, "null argument");
  memset(out, 0, sizeof *out);
  mochi_params p = {1, 1, 0, 0};
  mochi_verdicts o;
  memset(&o, 0, sizeof o);
  uint32_t dummy = 0;
  o.cert_accept_bits = &dummy;
  int rc = check_write2_header(c, w, &p, &o);
  if (rc) return rc;
  return verify_write2_host(c, w, &p, &o, nullptr, out);
}

void mochi_write2_decoded_free(mochi_write2_decoded* d) {
  if (!d) return;
  free(d->grant_off);
  free(d->grant_len);
  free(d->sig);
  free(d->signer);
  free(d->grant_key);
  free(d->cert_grant_off);
  free(d->cert_op_off);
  free(d->op_key);
  free(d->op_flags);
  free(d->msg_status);
  free(d->cert_mg_off);
  free(d->mg_grant_off);
  free(d->op_key_off);
  free(d->op_key_len);
  memset(d, 0, sizeof *d);
}

// ---- Write2 wire path: the messages the device decoder declines -------------
//
// MOCHI_MSG_FALLBACK messages (repeated / merged fields, non-canonical Grant
// bytes, more than 32 MultiGrants or 64 grants per MultiGrant) are decoded on
// the host with full protobuf-java semantics (w2_host.cpp) into an SoA batch and
// verified through the same device path as every other certificate; their
// verdicts replace the UNDECIDED placeholder.  Messages the host decoder cannot
// express (more than MOCHI_MAX_OPS_PER_CERT operations, a grant over 64 KiB,
// op_flags_off disagreeing with the operation count) stay UNDECIDED.
static int decide_fallback(mochi_ctx* c, const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* o,
                           const std::vector<uint32_t>& msgs) {
  const uint32_t* ofo = w->op_flags_off;
  std::vector<uint32_t> take;
  std::vector<mochi_host::Message> dec;
  for (uint32_t m : msgs) {
    mochi_host::Message d;
    if (mochi_host::decode_full(w->wire + w->msg_off[m], w->msg_len[m], c->server_ids, d) != MOCHI_MSG_OK) continue;
    if (ofo && ofo[m + 1] - ofo[m] != d.ops.size()) continue;
    bool fits = true;
    for (auto& mg : d.mgs)
      for (auto& g : mg.grants) fits &= g.bytes.size() <= 65536;
    if (!fits) continue;
    take.push_back(m);
    dec.push_back(std::move(d));
  }
  if (take.empty()) return MOCHI_OK;
  std::vector<uint8_t> blob, sig, gkey, opk, opf, hashes;
  std::vector<uint64_t> goff, okoff;
  std::vector<uint32_t> glen, cgo{0}, coo{0}, cmo{0}, mgo{0}, oklen;
  std::vector<uint16_t> signer;
  std::vector<int64_t> ots;
  for (size_t i = 0; i < take.size(); i++) {
    const uint32_t m = take[i];
    const mochi_host::Message& d = dec[i];
    for (auto& mg : d.mgs) {
      for (auto& g : mg.grants) {
        goff.push_back(blob.size());
        glen.push_back((uint32_t)g.bytes.size());
        blob.insert(blob.end(), g.bytes.begin(), g.bytes.end());
        sig.insert(sig.end(), g.sig, g.sig + MOCHI_RSA_BYTES);
        signer.push_back(mg.signer);
        gkey.push_back(g.slot);
      }
      mgo.push_back((uint32_t)goff.size());
    }
    cmo.push_back((uint32_t)mgo.size() - 1);
    cgo.push_back((uint32_t)goff.size());
    for (size_t j = 0; j < d.ops.size(); j++) {
      const auto& op = d.ops[j];
      opk.push_back(op.slot);
      const uint8_t fl = ofo ? w->op_flags[ofo[m] + j] : (uint8_t)(MOCHI_OP_LOCAL | MOCHI_OP_HAS_SVOC);
      opf.push_back((uint8_t)(fl | (op.not_write ? MOCHI_OP_NOT_WRITE : 0)));
      ots.push_back(ofo && w->op_object_ts ? w->op_object_ts[ofo[m] + j] : 0);
      okoff.push_back(blob.size());
      oklen.push_back((uint32_t)op.key_bytes.size());
      blob.insert(blob.end(), op.key_bytes.begin(), op.key_bytes.end());
    }
    coo.push_back((uint32_t)opk.size());
    hashes.insert(hashes.end(), w->expected_hash + (size_t)m * MOCHI_TXN_HASH_BYTES,
                  w->expected_hash + (size_t)(m + 1) * MOCHI_TXN_HASH_BYTES);
  }
  if (blob.empty()) blob.push_back(0);
  mochi_batch b;
  memset(&b, 0, sizeof b);
  b.n_grants = (uint32_t)goff.size();
  b.n_certs = (uint32_t)take.size();
  b.n_ops = (uint32_t)opk.size();
  b.n_mgs = (uint32_t)mgo.size() - 1;
  b.grant_bytes_len = blob.size();
  b.grant_bytes = blob.data();
  b.grant_off = goff.data();
  b.grant_len = glen.data();
  b.sig = sig.data();
  b.signer = signer.data();
  b.grant_key = gkey.data();
  b.cert_grant_off = cgo.data();
  b.cert_op_off = coo.data();
  b.op_key = opk.data();
  b.op_flags = opf.data();
  b.expected_hash = hashes.data();
  b.cert_mg_off = cmo.data();
  b.mg_grant_off = mgo.data();
  b.op_object_ts = ots.data();
  b.op_key_off = okoff.data();
  b.op_key_len = oklen.data();
  const size_t C = take.size(), O = opk.size();
  std::vector<uint32_t> acc((C + 31) / 32), og0(O + 1);
  std::vector<uint8_t> reason(C), fail(C), odec(O + 1);
  std::vector<int64_t> ots_out(O + 1);
  mochi_verdicts v;
  memset(&v, 0, sizeof v);
  v.cert_accept_bits = acc.data();
  v.cert_reason = reason.data();
  v.cert_fail_op = fail.data();
  v.op_decision = odec.data();
  v.op_g0 = og0.data();
  v.op_ts = ots_out.data();
  resolve_timing(c);
  float saved[4] = {c->last_ms[0], c->last_ms[1], c->last_ms[2], c->last_total_ms};
  const int rc = run_host_pipeline(c, &b, p, &v);
  c->last_ms[0] = saved[0], c->last_ms[1] = saved[1], c->last_ms[2] = saved[2], c->last_total_ms = saved[3];
  c->timing_pending = false;
  if (rc) return rc;
  for (size_t i = 0; i < C; i++) {
    const uint32_t m = take[i];
    const bool a = (acc[i >> 5] >> (i & 31)) & 1u;
    if (a) o->cert_accept_bits[m >> 5] |= 1u << (m & 31);
    else o->cert_accept_bits[m >> 5] &= ~(1u << (m & 31));
    if (o->cert_reason) o->cert_reason[m] = reason[i];
    if (o->cert_fail_op) o->cert_fail_op[m] = fail[i];
    if (ofo)
      for (uint32_t j = 0; j < coo[i + 1] - coo[i]; j++) {
        const size_t src = coo[i] + j, dst = ofo[m] + j;
        if (o->op_decision) o->op_decision[dst] = odec[src];
        if (o->op_g0) o->op_g0[dst] = og0[src];
        if (o->op_ts) o->op_ts[dst] = ots_out[src];
      }
  }
  return MOCHI_OK;
}

// ---- Write2 wire path, host memory: chunked pipeline -------------------------
//
// Messages are cut into chunks of whole messages (multiples of 32, so each
// chunk's accept bits start on a word) of ~chunk_grants * 256 wire bytes.
// For chunk j:
// stage + upload (copy-in stream), then on the context stream the decode count
// phase and its totals; chunk j-2's emit + verify + fix-up is enqueued once ITS
// totals are on the host, so the host waits only for count kernels while the
// device verifies earlier chunks and the copy engines move the next one.
// Verdicts come down per chunk on the copy-out stream.
static int verify_write2_host(mochi_ctx* c, const mochi_write2_batch* w, const mochi_params* p, mochi_verdicts* o,
                              uint8_t* msg_status, mochi_write2_decoded* dec) {
  constexpr size_t kW2Lag = 2;  // chunks counted ahead of the one being verified
  int rc;
  const uint32_t M = w->n_msgs;
  for (uint32_t m = 0; m < M; m++)
    if (w->msg_off[m] > w->wire_len || w->msg_len[m] > w->wire_len - w->msg_off[m])
      return fail(MOCHI_EINVAL, "message %u lies outside wire", m);
  if (w->op_flags_off) {  // the device trusts these offsets: validate them here
    if (w->op_flags_off[0] != 0) return fail(MOCHI_EINVAL, "op_flags_off[0] must be 0");
    for (uint32_t m = 0; m < M; m++)
      if (w->op_flags_off[m + 1] < w->op_flags_off[m]) return fail(MOCHI_EINVAL, "op_flags_off decreases at %u", m);
  }
  if (c->n_ids != c->n_keys) return fail(MOCHI_EINVAL, "server ids not set (mochi_ctx_set_server_ids)");
  std::lock_guard<std::mutex> lk(c->mu);
  new_call(c);
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(c->device) != hipSuccess) return fail(MOCHI_EHIP, "hipSetDevice(%d)", c->device);
  struct Restore {
    int d;
    ~Restore() { (void)hipSetDevice(d); }
  } restore{save};
  const uint32_t* ofo = w->op_flags_off;
  const size_t O_in = ofo ? ofo[M] : 0;
  // --- chunks ---
  struct Chunk {
    uint32_t m0, m1;
    uint64_t lo, hi;  // wire byte range
    size_t seg[7], cnt;
  };
  std::vector<Chunk> ch;
  // ~67 MB of wire bytes per chunk at the default chunk_grants (measured on one
  // box, 250k messages: 45.5 GB/s at 67 MB, 43.5 at 134 MB, 40.3 at 34 MB; a
  // ramp of smaller chunks at fill and drain measured 37.7: every chunk pays
  // the verify path's latency floor, ~0.6 ms, whatever its size)
  const uint64_t target = dec ? UINT64_MAX : (uint64_t)c->chunk_grants * 256;
  for (uint32_t m0 = 0; m0 < M || ch.empty();) {
    uint32_t m1 = m0;
    uint64_t bytes = 0;
    do {
      const uint32_t next = m1 + 32 < M ? m1 + 32 : M;
      for (uint32_t m = m1; m < next; m++) bytes += w->msg_len[m];
      m1 = next;
    } while (m1 < M && bytes < target);
    Chunk k{};
    k.m0 = m0;
    k.m1 = m1;
    uint64_t lo = UINT64_MAX, hi = 0;
    for (uint32_t m = m0; m < m1; m++) {
      lo = w->msg_off[m] < lo ? w->msg_off[m] : lo;
      hi = w->msg_off[m] + w->msg_len[m] > hi ? w->msg_off[m] + w->msg_len[m] : hi;
    }
    if (lo == UINT64_MAX) lo = hi = 0;
    k.lo = lo;
    k.hi = hi;
    ch.push_back(k);
    if (M == 0) break;
    m0 = m1;
  }
  const size_t nch = ch.size();
  // --- input segments: wire slice, msg_off, msg_len, op_flags_off (rebased), op_flags, op_object_ts, hash ---
  auto seg_bytes = [&](const Chunk& k, int i) -> size_t {
    const size_t nm = k.m1 - k.m0, no = ofo ? ofo[k.m1] - ofo[k.m0] : 0;
    switch (i) {
      case 0: return (size_t)(k.hi - k.lo);
      case 1: return 8 * nm;
      case 2: return 4 * nm;
      case 3: return ofo ? 4 * (nm + 1) : 0;
      case 4: return ofo ? no : 0;
      case 5: return ofo && w->op_object_ts ? 8 * no : 0;
      default: return (size_t)MOCHI_TXN_HASH_BYTES * nm;
    }
  };
  auto seg_src = [&](const Chunk& k, int i) -> const void* {
    switch (i) {
      case 0: return w->wire + k.lo;
      case 1: return w->msg_off + k.m0;
      case 2: return w->msg_len + k.m0;
      case 3: return nullptr;  // rebased, staged
      case 4: return ofo ? w->op_flags + ofo[k.m0] : nullptr;
      case 5: return ofo && w->op_object_ts ? w->op_object_ts + ofo[k.m0] : nullptr;
      default: return w->expected_hash + (size_t)MOCHI_TXN_HASH_BYTES * k.m0;
    }
  };
  size_t in_total = 0, cnt_total = 0;
  for (auto& k : ch) {
    for (int i = 0; i < 7; i++) {
      k.seg[i] = in_total;
      in_total = align_up(in_total + seg_bytes(k, i), 256);
    }
    k.cnt = cnt_total;
    cnt_total += mochi::w2_scratch_words(k.m1 - k.m0);
  }
  const size_t nbits = ((size_t)M + 31) / 32 * 4;
  size_t out_total = 0;
  auto take = [&](size_t bytes) {
    const size_t off = out_total;
    out_total = align_up(out_total + bytes, 256);
    return off;
  };
  const size_t o_acc = take(nbits), o_reason = take(M), o_fail = take(M), o_status = take(M ? M : 1),
               o_dec = take(o->op_decision ? O_in : 0), o_g0 = take(o->op_g0 ? 4 * O_in : 0),
               o_ots = take(o->op_ts ? 8 * O_in : 0);
  if ((rc = c->pin_in.ensure(in_total)) || (rc = c->dev_in.ensure(in_total)) || (rc = c->pin_out.ensure(out_total)) ||
      (rc = c->dev_out.ensure(out_total)) || (rc = c->w2_cnt.ensure(4 * cnt_total)) ||
      (rc = c->w2_tot.ensure(16 * nch)))
    return rc;
  while (c->chunk_ev.size() < 2 * nch) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->chunk_ev.push_back(e);
  }
  while (c->tot_ev.size() < nch) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->tot_ev.push_back(e);
  }
  uint8_t* pin = (uint8_t*)c->pin_in.p;
  uint8_t* din = c->dev_in.as<uint8_t>();
  uint8_t* dout = c->dev_out.as<uint8_t>();
  uint8_t* pout = (uint8_t*)c->pin_out.p;
  uint32_t* tot = (uint32_t*)c->w2_tot.p;
  hipStream_t st = c->stream;
  // sources already in pinned memory (mochi_host_alloc) are DMA'd in place;
  // the rebased op_flags_off CSR (segment 3) is always staged
  // One small chunk (a batcher flush): every segment staged and ONE upload and
  // ONE download of the whole region -- a copy costs ~5 us of its own on the
  // GPU whatever its size, and a 2-message batch moved 5 + 7 of them.
  const bool one_copy = nch == 1 && in_total <= (4u << 20);
  // ... and both copies on the launch stream: nothing to overlap them with, and
  // a cross-stream hand-off is one more event record, wait and barrier packet
  const bool on_st = one_copy && !copy_streams();  // MOCHI_COPY_STREAMS=1 (A/B): the copy streams anyway
  hipStream_t s_in = on_st ? st : c->s_in, s_out = on_st ? st : c->s_out;
  bool pinned[7];
  for (int i = 0; i < 7; i++) pinned[i] = !one_copy && i != 3 && is_pinned(seg_src(ch[0], i));
  std::vector<mochi_write2_batch> dws(nch);
  std::vector<mochi::W2Args> args(nch);
  HIP_TRY(scratch_acquire(c, st));
  c->ev_set ^= 1;  // this call's span events: the other set keeps the last call's
  c->ev = c->evs[c->ev_set];
  HIP_TRY(hipEventRecord(c->ev[0], s_in));
  // phase 2 + download of chunk j (its totals must be on the host)
  auto finish = [&](size_t j) -> int {
    Chunk& k = ch[j];
    HIP_TRY(hipEventSynchronize(c->tot_ev[j]));
    const uint32_t* t = tot + 4 * j;
    const uint32_t nm = k.m1 - k.m0, o0 = ofo ? ofo[k.m0] : 0;
    mochi_verdicts dv;
    memset(&dv, 0, sizeof dv);
    dv.cert_accept_bits = (uint32_t*)(dout + o_acc) + k.m0 / 32;
    dv.cert_reason = dout + o_reason + k.m0;
    dv.cert_fail_op = dout + o_fail + k.m0;
    dv.op_decision = o->op_decision ? dout + o_dec + o0 : nullptr;
    dv.op_g0 = o->op_g0 ? (uint32_t*)(dout + o_g0) + o0 : nullptr;
    dv.op_ts = o->op_ts ? (int64_t*)(dout + o_ots) + o0 : nullptr;
    int r = w2_verify(c, &dws[j], p, &dv, args[j], t[0], t[1], t[2], dws[j].op_flags_off, st, dec != nullptr);
    if (r) return r;
    if (dec) return MOCHI_OK;
    if (j + 1 == nch) HIP_TRY(hipEventRecord(c->ev[2], st));
    if (!on_st) {
      HIP_TRY(hipEventRecord(c->chunk_ev[2 * j + 1], st));
      HIP_TRY(hipStreamWaitEvent(s_out, c->chunk_ev[2 * j + 1], 0));
    }
    auto down = [&](size_t off, size_t bytes) -> hipError_t {
      return bytes ? hipMemcpyAsync(pout + off, dout + off, bytes, hipMemcpyDeviceToHost, s_out) : hipSuccess;
    };
    if (one_copy) return (int)(down(0, out_total) == hipSuccess ? MOCHI_OK : fail(MOCHI_EHIP, "download failed"));
    const size_t no = ofo ? ofo[k.m1] - o0 : 0;
    const size_t acc_words = j + 1 == nch ? nbits / 4 - k.m0 / 32 : nm / 32;
    HIP_TRY(down(o_acc + 4 * (size_t)(k.m0 / 32), 4 * acc_words));
    HIP_TRY(down(o_reason + k.m0, nm));
    HIP_TRY(down(o_fail + k.m0, nm));
    HIP_TRY(down(o_status + k.m0, nm));
    if (o->op_decision) HIP_TRY(down(o_dec + o0, no));
    if (o->op_g0) HIP_TRY(down(o_g0 + 4 * (size_t)o0, 4 * no));
    if (o->op_ts) HIP_TRY(down(o_ots + 8 * (size_t)o0, 8 * no));
    return MOCHI_OK;
  };
  for (size_t j = 0; j < nch; j++) {
    Chunk& k = ch[j];
    const uint32_t nm = k.m1 - k.m0;
    if (ofo) {
      uint32_t* f = (uint32_t*)(pin + k.seg[3]);
      for (uint32_t m = k.m0; m <= k.m1; m++) f[m - k.m0] = ofo[m] - ofo[k.m0];
    }
    size_t staged_end = 0;
    for (int i = 0; i < 7; i++) {
      const size_t n = seg_bytes(k, i);
      if (!n) continue;
      const void* src = pin + k.seg[i];
      if (pinned[i]) src = seg_src(k, i);  // DMA'd in place (e.g. the batcher's pinned batch)
      else if (i != 3) par_memcpy(pin + k.seg[i], seg_src(k, i), n);
      if (one_copy) staged_end = k.seg[i] + n > staged_end ? k.seg[i] + n : staged_end;
      else HIP_TRY(hipMemcpyAsync(din + k.seg[i], src, n, hipMemcpyHostToDevice, s_in));
    }
    if (one_copy && staged_end) HIP_TRY(hipMemcpyAsync(din, pin, staged_end, hipMemcpyHostToDevice, s_in));
    if (!on_st) HIP_TRY(hipEventRecord(c->chunk_ev[2 * j], s_in));
    mochi_write2_batch& dw = dws[j];
    memset(&dw, 0, sizeof dw);
    dw.n_msgs = nm;
    dw.wire_len = k.hi;
    dw.wire = din + k.seg[0] - k.lo;  // message offsets stay absolute
    dw.msg_off = (const uint64_t*)(din + k.seg[1]);
    dw.msg_len = (const uint32_t*)(din + k.seg[2]);
    dw.op_flags_off = ofo ? (const uint32_t*)(din + k.seg[3]) : nullptr;
    dw.op_flags = ofo ? din + k.seg[4] : nullptr;
    dw.op_object_ts = seg_bytes(k, 5) ? (const int64_t*)(din + k.seg[5]) : nullptr;
    dw.expected_hash = din + k.seg[6];
    if (!on_st) HIP_TRY(hipStreamWaitEvent(st, c->chunk_ev[2 * j], 0));
    if (j == 0) HIP_TRY(hipEventRecord(c->ev[1], st));
    if ((rc = w2_count(c, &dw, dout + o_status + k.m0, c->w2_cnt.as<uint32_t>() + k.cnt, tot + 4 * j, c->tot_ev[j], st,
                       &args[j])))
      return rc;
    // the verify of chunk j - kW2Lag: its totals are read on the host, so the
    // host waits for its count; with two chunks of lag the stream still holds
    // work while it waits
    if (j >= kW2Lag && (rc = finish(j - kW2Lag))) return rc;
  }
  for (size_t j = nch > kW2Lag ? nch - kW2Lag : 0; j < nch; j++)
    if ((rc = finish(j))) return rc;
  HIP_TRY(scratch_release(c, st));
  if (dec) {
    // decode-only (one chunk): copy the decoded SoA back (tests / inspection)
    const mochi::W2Args& da = args[0];
    const uint32_t N = tot[0], O = tot[1], NM = tot[2];
    dec->n_msgs = M;
    dec->n_grants = N;
    dec->n_ops = O;
    dec->n_mgs = NM;
    dec->grant_off = (uint64_t*)malloc(8 * (size_t)N + 8);
    dec->grant_len = (uint32_t*)malloc(4 * (size_t)N + 4);
    dec->sig = (uint8_t*)malloc((size_t)MOCHI_RSA_BYTES * N + 1);
    dec->signer = (uint16_t*)malloc(2 * (size_t)N + 2);
    dec->grant_key = (uint8_t*)malloc((size_t)N + 1);
    dec->cert_grant_off = (uint32_t*)malloc(4 * ((size_t)M + 1));
    dec->cert_op_off = (uint32_t*)malloc(4 * ((size_t)M + 1));
    dec->op_key = (uint8_t*)malloc((size_t)O + 1);
    dec->op_flags = (uint8_t*)malloc((size_t)O + 1);
    dec->msg_status = (uint8_t*)malloc((size_t)M + 1);
    dec->cert_mg_off = (uint32_t*)malloc(4 * ((size_t)M + 1));
    dec->mg_grant_off = (uint32_t*)malloc(4 * ((size_t)NM + 1));
    dec->op_key_off = (uint64_t*)malloc(8 * (size_t)O + 8);
    dec->op_key_len = (uint32_t*)malloc(4 * (size_t)O + 4);
    struct {
      void* dst;
      const void* src;
      size_t n;
    } cp[] = {{dec->grant_off, da.grant_off, 8 * (size_t)N},     {dec->grant_len, da.grant_len, 4 * (size_t)N},
              {dec->sig, da.sig, (size_t)MOCHI_RSA_BYTES * N},   {dec->signer, da.signer, 2 * (size_t)N},
              {dec->grant_key, da.grant_key, N},                 {dec->cert_grant_off, da.cert_grant_off, 4 * ((size_t)M + 1)},
              {dec->cert_op_off, da.cert_op_off, 4 * ((size_t)M + 1)}, {dec->op_key, da.op_key, O},
              {dec->op_flags, da.op_flags, O},                   {dec->msg_status, da.status, M},
              {dec->cert_mg_off, da.cert_mg_off, 4 * ((size_t)M + 1)}, {dec->mg_grant_off, da.mg_grant_off, 4 * ((size_t)NM + 1)},
              {dec->op_key_off, da.op_key_off, 8 * (size_t)O},   {dec->op_key_len, da.op_key_len, 4 * (size_t)O}};
    for (auto& x : cp)
      if (x.n) HIP_TRY(hipMemcpyAsync(x.dst, x.src, x.n, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    return MOCHI_OK;
  }
  HIP_TRY(hipEventRecord(c->ev[3], s_out));
  HIP_TRY(hipStreamSynchronize(s_out));
  c->ev_done = c->ev_set;
  c->timing_pending = true;  // read from the events when asked (mochi_ctx_last_timing): four API calls off the call's path
  std::vector<uint32_t> fallback;
  for (uint32_t m = 0; m < M; m++)
    if (pout[o_status + m] == MOCHI_MSG_FALLBACK) fallback.push_back(m);
  memcpy(o->cert_accept_bits, pout + o_acc, nbits);
  if (o->cert_reason) memcpy(o->cert_reason, pout + o_reason, M);
  if (o->cert_fail_op) memcpy(o->cert_fail_op, pout + o_fail, M);
  if (msg_status) memcpy(msg_status, pout + o_status, M);
  if (o->op_decision) memcpy(o->op_decision, pout + o_dec, O_in);
  if (o->op_g0) memcpy(o->op_g0, pout + o_g0, 4 * O_in);
  if (o->op_ts) memcpy(o->op_ts, pout + o_ots, 8 * O_in);
  c->acc_dev = (const uint32_t*)(dout + o_acc);
  c->acc_words = (uint32_t)(nbits / 4);
  if (fallback.empty()) return MOCHI_OK;
  rc = decide_fallback(c, w, p, o, fallback);
  c->acc_dev = nullptr;  // the host decided some verdicts (and the fallback batch reused dev_out)
  c->acc_words = 0;
  return rc;
}

int mochi_fold_matrix(const uint8_t* modulus_be, int8_t* img, uint32_t* cadd) {
  if (!modulus_be || !img || !cadd) return fail(MOCHI_EINVAL, "null argument");
  if (!(modulus_be[0] & 0x80) || !(modulus_be[255] & 1)) return fail(MOCHI_EINVAL, "modulus must be odd, 2048 bits");
  std::vector<mochi::FoldKey> f(1);
  int rc = make_fold_key(modulus_be, f.data());
  if (rc) return rc;
  memcpy(img, f[0].img, sizeof f[0].img);
  memcpy(cadd, f[0].cadd, sizeof f[0].cadd);
  return MOCHI_OK;
}

int mochi_rsa_public_op(mochi_ctx* c, uint32_t n, const uint8_t* sig_be, const uint16_t* signer, uint8_t* out_be,
                        uint32_t* out_z) {
  if (!c || (n && (!sig_be || !signer || !out_be))) return fail(MOCHI_EINVAL, "null argument");
  for (uint32_t i = 0; i < n; i++)
    if (signer[i] >= c->n_keys) return fail(MOCHI_EINVAL, "signer[%u] out of range", i);
  if (n == 0) return MOCHI_OK;
  std::lock_guard<std::mutex> lk(c->mu);
  new_call(c);
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(c->device) != hipSuccess) return fail(MOCHI_EHIP, "hipSetDevice(%d)", c->device);
  const uint64_t slots = mochi::slot_capacity(n, c->n_keys);
  const size_t sig_bytes = (size_t)MOCHI_RSA_BYTES * n, y_bytes = sizeof(uint32_t) * 64 * (size_t)n;
  int rc;
  if ((rc = c->dev_in.ensure(align_up(sig_bytes, 256) + sizeof(uint16_t) * n)) || (rc = c->dev_out.ensure(y_bytes)) ||
      (rc = c->digest.ensure(sizeof(uint32_t) * 8 * (size_t)n)) || (rc = c->flags.ensure(n)) ||
      (rc = c->count.ensure(sizeof(uint32_t) * c->n_keys)) || (rc = c->cursor.ensure(sizeof(uint32_t) * c->n_keys)) ||
      (rc = c->total.ensure(mochi::kTotalWords * sizeof(uint32_t))) || (rc = c->perm.ensure(sizeof(uint32_t) * (size_t)slots)) ||
      (rc = c->xbuf.ensure(sizeof(uint32_t) * mochi::kL * (size_t)slots))) {
    (void)hipSetDevice(save);
    return rc;
  }
  hipStream_t st = c->stream;
  uint8_t* din = c->dev_in.as<uint8_t>();
  uint16_t* dsigner = (uint16_t*)(din + align_up(sig_bytes, 256));
  mochi::LaunchArgs a;
  memset(&a, 0, sizeof a);
  a.n_grants = n;
  a.n_keys = c->n_keys;
  a.n_slots = (uint32_t)slots;
  a.sig = din;
  a.signer = dsigner;
  a.keys = c->d_keys;
  a.fold = c->d_fold;
  a.digest = c->digest.as<uint32_t>();
  a.flags = c->flags.as<uint8_t>();
  a.count = c->count.as<uint32_t>();
  a.cursor = c->cursor.as<uint32_t>();
  a.total = c->total.as<uint32_t>();
  a.perm = c->perm.as<uint32_t>();
  a.xbuf = c->xbuf.as<uint32_t>();
  a.dbg_y = c->dev_out.as<uint32_t>();
  a.skip_prep_tally = true;
  std::vector<uint32_t> y(64 * (size_t)n), perm, z;
  bool ok = hipMemcpyAsync(din, sig_be, sig_bytes, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemcpyAsync(dsigner, signer, sizeof(uint16_t) * n, hipMemcpyHostToDevice, st) == hipSuccess &&
            hipMemsetAsync(a.digest, 0, sizeof(uint32_t) * 8 * (size_t)n, st) == hipSuccess &&
            hipMemsetAsync(a.flags, 0, n, st) == hipSuccess && mochi::launch_verify(a, st) == hipSuccess &&
            hipMemcpyAsync(y.data(), a.dbg_y, y_bytes, hipMemcpyDeviceToHost, st) == hipSuccess;
  if (ok && out_z) {
    perm.resize(slots);
    z.resize((size_t)mochi::kL * slots);
    ok = hipMemcpyAsync(perm.data(), a.perm, sizeof(uint32_t) * slots, hipMemcpyDeviceToHost, st) == hipSuccess &&
         hipMemcpyAsync(z.data(), a.xbuf, sizeof(uint32_t) * z.size(), hipMemcpyDeviceToHost, st) == hipSuccess;
  }
  ok = ok && hipStreamSynchronize(st) == hipSuccess;
  (void)hipSetDevice(save);
  if (!ok) return fail(MOCHI_EHIP, "rsa_public_op failed: %s", hipGetErrorString(hipGetLastError()));
  for (uint32_t g = 0; g < n; g++)
    for (int i = 0; i < 64; i++) {
      const uint32_t w = y[(size_t)g * 64 + i];
      uint8_t* o = out_be + (size_t)g * 256 + 256 - 4 * (i + 1);
      o[0] = (uint8_t)(w >> 24);
      o[1] = (uint8_t)(w >> 16);
      o[2] = (uint8_t)(w >> 8);
      o[3] = (uint8_t)w;
    }
  if (out_z)
    for (uint64_t sl = 0; sl < slots; sl++) {
      const uint32_t g = perm[sl];
      if (g == 0xFFFFFFFFu) continue;
      for (int j = 0; j < mochi::kL; j++) out_z[(size_t)g * mochi::kL + j] = z[(size_t)j * slots + sl];
    }
  return MOCHI_OK;
}

int mochi_ctx_set_profiling(mochi_ctx* c, int on) {
  if (!c) return fail(MOCHI_EINVAL, "null ctx");
  std::lock_guard<std::mutex> lk(c->mu);
  c->profiling = on != 0;
  return MOCHI_OK;
}

int mochi_ctx_read_profile(mochi_ctx* c, float* stage_ms, uint32_t n_stages, uint32_t* n_calls) {
  if (!c || !stage_ms) return fail(MOCHI_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(c->mu);
  for (uint32_t i = 0; i < n_stages; i++) stage_ms[i] = 0.f;
  uint32_t calls = 0;
  for (auto& evs : c->prof_sets) {
    for (auto e : evs)
      if (hipEventSynchronize(e) != hipSuccess) return fail(MOCHI_EHIP, "hipEventSynchronize failed");
    for (uint32_t i = 0; i < n_stages && i < (uint32_t)mochi::kProfStages; i++) {
      float ms = 0.f;
      (void)hipEventElapsedTime(&ms, evs[2 * i], evs[2 * i + 1]);  // (start, end) of stage i
      stage_ms[i] += ms;
    }
    for (auto e : evs) (void)hipEventDestroy(e);
    calls++;
  }
  c->prof_sets.clear();
  if (n_calls) *n_calls = calls;
  return MOCHI_OK;
}

int mochi_ctx_last_timing(mochi_ctx* c, float* h2d_ms, float* kernels_ms, float* d2h_ms) {
  if (!c) return fail(MOCHI_EINVAL, "null ctx");
  resolve_timing(c);
  if (h2d_ms) *h2d_ms = c->last_ms[0];
  if (kernels_ms) *kernels_ms = c->last_ms[1];
  if (d2h_ms) *d2h_ms = c->last_ms[2];
  return MOCHI_OK;
}

// Client-side aggregation: MochiDBClient.java:148-175 (reads) / 355-382 (Write2).
int mochi_tally_responses(uint32_t n_requests, const uint32_t* resp_off, const uint32_t* n_ops,
                          const uint32_t* resp_n_ops, const uint64_t* status_off, const uint8_t* status,
                          const uint64_t* chosen_off, uint32_t replication_factor, int32_t* chosen, uint8_t* reason,
                          uint32_t* accept_bits) {
  if (!resp_off || !n_ops || !resp_n_ops || !status_off || !status || !chosen_off || !accept_bits)
    return fail(MOCHI_EINVAL, "null argument");
  const uint32_t M = 2 * (replication_factor / 3) + 1;  // getServerMajority
  memset(accept_bits, 0, ((size_t)n_requests + 31) / 32 * 4);
  std::vector<uint32_t> cnt;
  for (uint32_t r = 0; r < n_requests; r++) {
    const uint32_t k = n_ops[r];
    cnt.assign(k, 0);
    int32_t* ch = chosen ? chosen + chosen_off[r] : nullptr;
    if (ch)
      for (uint32_t j = 0; j < k; j++) ch[j] = -1;
    uint8_t why = 0;
    for (uint32_t q = resp_off[r]; q < resp_off[r + 1]; q++) {
      if (resp_n_ops[q] != k) {  // operations.size() != transactionOps.size()
        why = 1;
        break;
      }
      const uint8_t* st = status + status_off[q];
      for (uint32_t j = 0; j < k; j++)
        if (st[j] != 1) {  // != WRONG_SHARD
          cnt[j]++;
          if (ch) ch[j] = (int32_t)(q - resp_off[r]);
        }
    }
    for (uint32_t j = 0; j < k && !why; j++)
      if (cnt[j] < M) why = 2;  // consistentTRCount[index] < getServerMajority()
    if (reason) reason[r] = why;
    if (!why) accept_bits[r >> 5] |= 1u << (r & 31);
  }
  return MOCHI_OK;
}

int mochi_write1_classify(uint32_t n_requests, const uint32_t* resp_off, const uint8_t* resp_kind,
                          const uint32_t* resp_server, const uint32_t* resp_grant_off, const uint8_t* grant_key,
                          const int64_t* grant_ts, const uint8_t* grant_status, uint8_t* decision) {
  if (!resp_off || !resp_kind || !resp_server || !resp_grant_off || !decision)
    return fail(MOCHI_EINVAL, "null argument");
  if (resp_grant_off[resp_off[n_requests]] > resp_grant_off[0] && (!grant_key || !grant_ts || !grant_status))
    return fail(MOCHI_EINVAL, "null grant arrays");
  std::vector<uint32_t> ok_servers;
  for (uint32_t r = 0; r < n_requests; r++) {
    const uint32_t q0 = resp_off[r], q1 = resp_off[r + 1];
    if (q1 < q0) return fail(MOCHI_EINVAL, "resp_off not monotone at request %u", r);
    // one pass: REQUESTFAILED dominates, then any WRONG_SHARD grant in an OK/REFUSED multigrant
    bool failed = false, wrong_shard = false, all_ok = true;
    for (uint32_t q = q0; q < q1; q++) {
      const uint8_t kind = resp_kind[q];
      all_ok &= kind == MOCHI_W1_OK;
      failed |= kind == MOCHI_W1_REQUEST_FAILED;
      if (kind == MOCHI_W1_OK || kind == MOCHI_W1_REFUSED)
        for (uint32_t g = resp_grant_off[q]; g < resp_grant_off[q + 1]; g++) wrong_shard |= grant_status[g] == 1;
    }
    uint8_t d;
    if (failed) d = MOCHI_W1_THROW_FAILED;
    else if (wrong_shard) d = MOCHI_W1_THROW_UNSUPPORTED;
    else {
      // uniformity over the surviving OK multigrant of every serverId (the
      // last one, HashMap.put): walk backwards, skip ids already taken
      int64_t ts0[256];
      uint8_t seen[256];
      memset(seen, 0, sizeof seen);
      ok_servers.clear();
      bool uniform = true;
      for (uint32_t q = q1; q-- > q0 && uniform;) {
        if (resp_kind[q] != MOCHI_W1_OK) continue;
        bool dup = false;
        for (uint32_t sid : ok_servers) dup |= sid == resp_server[q];
        if (dup) continue;
        ok_servers.push_back(resp_server[q]);
        for (uint32_t g = resp_grant_off[q]; g < resp_grant_off[q + 1]; g++) {
          const uint8_t k = grant_key[g];
          if (k == 0xFF) continue;
          if (!seen[k]) {
            seen[k] = 1;
            ts0[k] = grant_ts[g];
          } else if (ts0[k] != grant_ts[g]) {
            uniform = false;
            break;
          }
        }
      }
      d = !uniform ? MOCHI_W1_RETRY : all_ok ? MOCHI_W1_PROCEED : MOCHI_W1_THROW_REFUSED;
    }
    decision[r] = d;
  }
  return MOCHI_OK;
}

}  // extern "C"

// ---- device signer (rsa_sign.hip) --------------------------------------------
struct mochi_signer {
  int device = 0;
  hipStream_t stream = nullptr;
  void* d_key = nullptr;
  std::mutex mu;
  DevBuf dev_in, dev_sig;
  PinnedBuf pin_in, pin_out;
  // fault check: the verify path under the signer's own public key
  mochi_ctx* check = nullptr;
  DevBuf zeros, flags, misc;  // signer index / key slot zeros, SIG_OK flags, [0] rejected [1..] CSR zeros
  uint32_t fault_idx = 0xFFFFFFFFu;
};

namespace {

int bn_limbs(const BIGNUM* v, uint32_t* x, int n_limbs) {
  std::vector<uint8_t> le((size_t)n_limbs * 28 / 8 + 8, 0);
  if (BN_num_bytes(v) > (int)le.size() - 8 || BN_bn2lebinpad(v, le.data(), (int)le.size()) < 0) return 0;
  for (int j = 0; j < n_limbs; j++) {
    const int bit = j * 28, by = bit >> 3, sh = bit & 7;
    uint64_t w = 0;
    for (int b = 0; b < 5; b++) w |= (uint64_t)le[by + b] << (8 * b);
    x[j] = (uint32_t)(w >> sh) & 0x0FFFFFFFu;
  }
  return 1;
}

// -m^{-1} mod 2^28 from m's lowest 28-bit limb (odd): Newton on 32 bits
uint32_t neg_inv28(uint32_t lo) {
  uint32_t inv = 1;
  for (int i = 0; i < 6; i++) inv *= 2u - lo * inv;
  return (0u - inv) & 0x0FFFFFFFu;
}

}  // namespace

extern "C" {

mochi_signer* mochi_signer_create(int device, const char* pem) {
  if (!pem) {
    fail(MOCHI_EINVAL, "null key");
    return nullptr;
  }
  BIO* bio = BIO_new_mem_buf(pem, -1);
  EVP_PKEY* pk = bio ? PEM_read_bio_PrivateKey(bio, nullptr, nullptr, nullptr) : nullptr;
  if (bio) BIO_free(bio);
  BIGNUM *p = nullptr, *q = nullptr, *dp = nullptr, *dq = nullptr, *qi = nullptr;
  bool ok = pk && EVP_PKEY_get_bits(pk) == 2048 && EVP_PKEY_get_bn_param(pk, OSSL_PKEY_PARAM_RSA_FACTOR1, &p) &&
            EVP_PKEY_get_bn_param(pk, OSSL_PKEY_PARAM_RSA_FACTOR2, &q) &&
            EVP_PKEY_get_bn_param(pk, OSSL_PKEY_PARAM_RSA_EXPONENT1, &dp) &&
            EVP_PKEY_get_bn_param(pk, OSSL_PKEY_PARAM_RSA_EXPONENT2, &dq) &&
            EVP_PKEY_get_bn_param(pk, OSSL_PKEY_PARAM_RSA_COEFFICIENT1, &qi);
  if (pk) EVP_PKEY_free(pk);
  ok = ok && BN_num_bits(p) <= 1024 && BN_num_bits(q) <= 1024 && BN_num_bits(dp) <= 1024 && BN_num_bits(dq) <= 1024 &&
       BN_num_bits(dp) >= 2 && BN_num_bits(dq) >= 2;
  constexpr int kLh = 37;
  uint32_t lp[kLh], lq[kLh], r3p[kLh], r3q[kLh], qir[kLh], wdp[32], wdq[32], cpad[74];
  BN_CTX* bc = BN_CTX_new();
  BIGNUM *R = BN_new(), *t = BN_new(), *three = BN_new(), *cp = nullptr;
  uint8_t cb[256];
  memset(cb, 0xFF, sizeof cb);
  static const uint8_t kDigestInfo[19] = {0x30, 0x31, 0x30, 0x0d, 0x06, 0x09, 0x60, 0x86, 0x48, 0x01,
                                          0x65, 0x03, 0x04, 0x02, 0x01, 0x05, 0x00, 0x04, 0x20};
  cb[0] = 0x00;
  cb[1] = 0x01;
  cb[256 - 32 - 19 - 1] = 0x00;
  memcpy(cb + 256 - 32 - 19, kDigestInfo, 19);
  memset(cb + 256 - 32, 0, 32);
  cp = BN_bin2bn(cb, 256, nullptr);
  ok = ok && bc && R && t && three && cp && BN_set_bit(R, 28 * kLh) && BN_set_word(three, 3);
  ok = ok && bn_limbs(p, lp, kLh) && bn_limbs(q, lq, kLh);
  ok = ok && BN_mod_exp(t, R, three, p, bc) && bn_limbs(t, r3p, kLh);
  ok = ok && BN_mod_exp(t, R, three, q, bc) && bn_limbs(t, r3q, kLh);
  ok = ok && BN_mod_mul(t, qi, R, p, bc) && bn_limbs(t, qir, kLh);
  ok = ok && bn_limbs(cp, cpad, 74);
  uint8_t le[128];
  ok = ok && BN_bn2lebinpad(dp, le, 128) == 128;
  if (ok)
    for (int i = 0; i < 32; i++) wdp[i] = (uint32_t)le[4 * i] | (uint32_t)le[4 * i + 1] << 8 | (uint32_t)le[4 * i + 2] << 16 | (uint32_t)le[4 * i + 3] << 24;
  ok = ok && BN_bn2lebinpad(dq, le, 128) == 128;
  if (ok)
    for (int i = 0; i < 32; i++) wdq[i] = (uint32_t)le[4 * i] | (uint32_t)le[4 * i + 1] << 8 | (uint32_t)le[4 * i + 2] << 16 | (uint32_t)le[4 * i + 3] << 24;
  std::vector<uint8_t> host(mochi::sign_key_bytes());
  if (ok)
    mochi::sign_key_set(host.data(), lp, lq, r3p, r3q, qir, wdp, wdq, cpad, neg_inv28(lp[0]), neg_inv28(lq[0]),
                        (uint32_t)BN_num_bits(dp), (uint32_t)BN_num_bits(dq));
  for (BIGNUM* b : {p, q, dp, dq, qi, R, t, three, cp}) BN_clear_free(b);
  BN_CTX_free(bc);
  if (!ok) {
    fail(MOCHI_EINVAL, "not an RSA-2048 private key with CRT parameters");
    return nullptr;
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
    fail(MOCHI_ENODEV, "device %d not available", device);
    return nullptr;
  }
  mochi_signer* s = new mochi_signer;
  s->device = device;
  int save = 0;
  (void)hipGetDevice(&save);
  ok = hipSetDevice(device) == hipSuccess && hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking) == hipSuccess &&
       hipMalloc(&s->d_key, host.size()) == hipSuccess &&
       hipMemcpy(s->d_key, host.data(), host.size(), hipMemcpyHostToDevice) == hipSuccess;
  memset(host.data(), 0, host.size());
  (void)hipSetDevice(save);
  if (!ok) {
    fail(MOCHI_EHIP, "signer setup failed");
    mochi_signer_destroy(s);
    return nullptr;
  }
  uint8_t n_be[MOCHI_RSA_BYTES];
  if (mochi_pem_modulus(pem, n_be) != MOCHI_OK ||
      !(s->check = mochi_ctx_create(device, n_be, 1, MOCHI_RSA_BYTES, MOCHI_RSA_E))) {
    fail(MOCHI_EINVAL, "signer: public-key check context failed");
    mochi_signer_destroy(s);
    return nullptr;
  }
  if (s->misc.ensure(256) || hipMemset(s->misc.p, 0, 256) != hipSuccess) {
    fail(MOCHI_EHIP, "signer scratch");
    mochi_signer_destroy(s);
    return nullptr;
  }
  return s;
}

void mochi_signer_destroy(mochi_signer* s) {
  if (!s) return;
  int save = 0;
  (void)hipGetDevice(&save);
  (void)hipSetDevice(s->device);
  if (s->stream) (void)hipStreamSynchronize(s->stream);
  if (s->d_key) {
    (void)hipMemset(s->d_key, 0, mochi::sign_key_bytes());  // private key material
    (void)hipFree(s->d_key);
  }
  if (s->stream) (void)hipStreamDestroy(s->stream);
  if (s->check) mochi_ctx_destroy(s->check);
  delete s;
  (void)hipSetDevice(save);
}

}  // extern "C"

namespace {
// Verify n freshly made signatures with the signer's public key on the same
// stream (k_grant_prep + k_rsa_pow + k_rsa_final, ~1/50 of the signing work)
// and withhold every one that fails (RSA-CRT fault attack, Boneh-DeMillo-Lipton).
int signer_check(mochi_signer* s, const uint8_t* grant_bytes, const uint64_t* grant_off, const uint32_t* grant_len,
                 uint32_t n, uint8_t* sig, hipStream_t st) {
  if (!n) return MOCHI_OK;
  int rc;
  if ((rc = s->zeros.ensure(2 * (size_t)n)) || (rc = s->flags.ensure(n))) return rc;
  HIP_TRY(hipMemsetAsync(s->zeros.p, 0, 2 * (size_t)n, st));
  mochi_batch db;
  memset(&db, 0, sizeof db);
  db.n_grants = n;
  db.grant_bytes = grant_bytes;
  db.grant_off = grant_off;
  db.grant_len = grant_len;
  db.sig = sig;
  db.signer = s->zeros.as<uint16_t>();
  db.grant_key = s->zeros.as<uint8_t>();
  uint32_t* misc = s->misc.as<uint32_t>();
  db.cert_grant_off = misc + 1;  // one zero: no certificates
  db.cert_op_off = misc + 1;
  mochi_params p = {1, 1, 0, 0};
  mochi_verdicts dv;
  memset(&dv, 0, sizeof dv);
  dv.grant_flags = s->flags.as<uint8_t>();
  dv.cert_accept_bits = misc + 2;
  if ((rc = run_device(s->check, &db, &p, &dv, st))) return rc;
  HIP_TRY(mochi::launch_withhold(s->flags.as<uint8_t>(), n, sig, misc, st));
  return MOCHI_OK;
}
}  // namespace

extern "C" {

int mochi_signer_set_fault(mochi_signer* s, uint32_t grant_index) {
  if (!s) return fail(MOCHI_EINVAL, "null signer");
  std::lock_guard<std::mutex> lk(s->mu);
  s->fault_idx = grant_index;
  return MOCHI_OK;
}

int mochi_signer_rejected(mochi_signer* s, uint64_t* rejected) {
  if (!s || !rejected) return fail(MOCHI_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  int save = 0;
  (void)hipGetDevice(&save);
  uint32_t v = 0;
  const bool ok = hipSetDevice(s->device) == hipSuccess && hipDeviceSynchronize() == hipSuccess &&
                  hipMemcpy(&v, s->misc.p, 4, hipMemcpyDeviceToHost) == hipSuccess &&
                  hipMemset(s->misc.p, 0, 4) == hipSuccess;
  (void)hipSetDevice(save);
  if (!ok) return fail(MOCHI_EHIP, "signer counter read failed");
  *rejected = v;
  return MOCHI_OK;
}

int mochi_sign_batch_device(mochi_signer* s, const uint8_t* grant_bytes, const uint64_t* grant_off,
                            const uint32_t* grant_len, uint32_t n, uint8_t* sig_out, void* stream) {
  if (!s || (n && (!grant_bytes || !grant_off || !grant_len || !sig_out))) return fail(MOCHI_EINVAL, "null argument");
  std::lock_guard<std::mutex> lk(s->mu);
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(s->device) != hipSuccess) return fail(MOCHI_EHIP, "hipSetDevice");
  const hipError_t e = mochi::launch_rsa_sign(grant_bytes, grant_off, grant_len, n, s->d_key, sig_out, s->fault_idx,
                                              (hipStream_t)stream);
  int rc = e == hipSuccess ? MOCHI_OK : fail(MOCHI_EHIP, "k_rsa_sign: %s", hipGetErrorString(e));
  if (!rc) {
    std::lock_guard<std::mutex> ck(s->check->mu);
    rc = signer_check(s, grant_bytes, grant_off, grant_len, n, sig_out, (hipStream_t)stream);
  }
  (void)hipSetDevice(save);
  return rc;
}

int mochi_sign_batch(mochi_signer* s, const uint8_t* grant_bytes, uint64_t grant_bytes_len, const uint64_t* grant_off,
                     const uint32_t* grant_len, uint32_t n, uint8_t* sig_out) {
  if (!s || (n && (!grant_bytes || !grant_off || !grant_len || !sig_out))) return fail(MOCHI_EINVAL, "null argument");
  for (uint32_t i = 0; i < n; i++)
    if (grant_off[i] > grant_bytes_len || grant_len[i] > grant_bytes_len - grant_off[i])
      return fail(MOCHI_EINVAL, "grant %u lies outside grant_bytes", i);
  if (n == 0) return MOCHI_OK;
  std::lock_guard<std::mutex> lk(s->mu);
  int save = 0;
  (void)hipGetDevice(&save);
  if (hipSetDevice(s->device) != hipSuccess) return fail(MOCHI_EHIP, "hipSetDevice");
  const size_t o_off = align_up(grant_bytes_len, 256), o_len = o_off + align_up(8 * (size_t)n, 256),
               total = o_len + align_up(4 * (size_t)n, 256), sig_bytes = (size_t)MOCHI_RSA_BYTES * n;
  int rc;
  if ((rc = s->pin_in.ensure(total)) || (rc = s->dev_in.ensure(total)) || (rc = s->pin_out.ensure(sig_bytes)) ||
      (rc = s->dev_sig.ensure(sig_bytes))) {
    (void)hipSetDevice(save);
    return rc;
  }
  uint8_t* pin = (uint8_t*)s->pin_in.p;
  par_memcpy(pin, grant_bytes, grant_bytes_len);
  memcpy(pin + o_off, grant_off, 8 * (size_t)n);
  memcpy(pin + o_len, grant_len, 4 * (size_t)n);
  uint8_t* din = s->dev_in.as<uint8_t>();
  hipStream_t st = s->stream;
  hipError_t e = hipMemcpyAsync(din, pin, total, hipMemcpyHostToDevice, st);
  if (e == hipSuccess)
    e = mochi::launch_rsa_sign(din, (const uint64_t*)(din + o_off), (const uint32_t*)(din + o_len), n, s->d_key,
                               s->dev_sig.as<uint8_t>(), s->fault_idx, st);
  if (e == hipSuccess) {
    std::lock_guard<std::mutex> ck(s->check->mu);
    if (signer_check(s, din, (const uint64_t*)(din + o_off), (const uint32_t*)(din + o_len), n,
                     s->dev_sig.as<uint8_t>(), st) != MOCHI_OK)
      e = hipErrorUnknown;
  }
  if (e == hipSuccess) e = hipMemcpyAsync(s->pin_out.p, s->dev_sig.p, sig_bytes, hipMemcpyDeviceToHost, st);
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  if (e == hipSuccess) memcpy(sig_out, s->pin_out.p, sig_bytes);
  (void)hipSetDevice(save);
  return e == hipSuccess ? MOCHI_OK : fail(MOCHI_EHIP, "sign batch: %s", hipGetErrorString(e));
}

}  // extern "C"
