// rsa_sign.hip — k_rsa_sign: producer-side SHA256withRSA on the device, one
// signature per lane, for the Write1 signing site the reference leaves as a
// TODO (InMemoryDataStore.java:283-295 builds the MultiGrant;
// MochiProtocol.proto:123 "// TODO: add signature").  Every lane signs with the
// SAME server key (a server signs its own grants), so the key, the CRT primes
// and the private exponents are wave-uniform: scalar loads / SGPR operands,
// uniform branches on the exponent bits.
//
//   H  = SHA-256(grant)                       (sha256_dev.h)
//   EM = Cpad + H                             (RFC 8017 §9.2, Cpad precomputed)
//   m1 = EM^dP mod p,  m2 = EM^dQ mod q       (37-limb Montgomery, mont_crt.h)
//   h  = qInv (m1 - m2) mod p,  s = m2 + h q  (Garner)
//
// PKCS#1 v1.5 signatures are deterministic, so s is bit-for-bit what OpenSSL's
// EVP_DigestSign gives (tests/test_gpu_sign.py).  Exponentiation is a fixed
// 4-bit window over the uniform exponent: ~1,020 squarings + 255 multiplies +
// 16 table products per half, 2,072 / 2,738 v_mad_u64_u32 each (~5.8M per
// signature).  The operation sequence depends only on the exponent's length,
// neither on the message nor on the exponent's bits.
#include "../../include/mochi_hip.h"
#include "kernels.h"
#include "mont_crt.h"
#include "sha256_dev.h"

namespace mochi {

constexpr int kLh = 37;  // 37 * 28 = 1036 bits > 1024-bit primes, R = 2^1036 > 4p

struct SignKey {
  uint32_t p[kLh], q[kLh];
  uint32_t r3p[kLh], r3q[kLh];  // R^3 mod p, R^3 mod q
  uint32_t qinv_r[kLh];         // qInv * R mod p
  uint32_t dp[32], dq[32];      // CRT exponents, 32-bit words little-endian
  uint32_t cpad[kL];            // EM with a zero digest, 74 limbs
  uint32_t p0inv, q0inv, dp_bits, dq_bits;
};

namespace {

// Fixed 4-bit-window exponentiation: T[j] = base^j (Montgomery form, T[0] = R
// mod p), then for every window below the top one 4 squarings and ONE
// multiply by T[window] -- including window 0, so the operation sequence
// depends only on the exponent's length, not on its bits.  ~1,020 squarings +
// 255 multiplies + 16 table products per 1024-bit half, vs ~1,023 + ~512 for
// square-and-multiply.  T lives in per-lane private (scratch) memory.  The
// window value is a digit of the SECRET exponent, so T is never indexed by it:
// every multiply reads all 16 entries in a fixed order and keeps one with a
// mask computed in VGPRs (v_cmp / v_cndmask, no branch on the digit), so the
// addresses, the instruction stream and its timing are the same for every
// digit.  Cost (measured, round 4): 16 x 37 scratch loads per multiply make
// the signer memory-bound on its scratch table (PMC: frac_wait_any 0.62) and
// halved its rate, 5.26e6 -> 2.68e6 signatures/s; the
// producer side is not the verify path, and constant-time lookups are the
// point.
template <int L>
__device__ __forceinline__ void table_select(uint32_t (&out)[L], const uint32_t (&tbl)[16][L], uint32_t w) {
  uint32_t wv = w;
  asm volatile("" : "+v"(wv));  // the digit as a per-lane value: compares stay vector, never a scalar branch
#pragma unroll
  for (int j = 0; j < L; j++) out[j] = 0;
#pragma unroll
  for (uint32_t v = 0; v < 16; v++) {
    const uint32_t m = 0u - (uint32_t)(wv == v);
#pragma unroll
    for (int j = 0; j < L; j++) out[j] |= tbl[v][j] & m;
  }
}

template <int L>
__device__ __forceinline__ void mont_pow(uint32_t (&acc)[L], const uint32_t (&base)[L], cptr r3, cptr e,
                                         uint32_t ebits, cptr n, uint32_t n0inv) {
  uint32_t tbl[16][L];
  uint32_t t[L];
  {
    // T[0] = R mod p: MontMul(R^3, 1) = R^2, MontMul(R^2, 1) = R  (both < 2p)
    uint32_t one[L] = {};
    one[0] = 1;
    const uint32_t unused[L] = {};
    mont_mul_n<L, true>(t, one, r3, unused, n, n0inv);
    mont_mul_n<L, false>(t, t, nullptr, one, n, n0inv);
  }
#pragma unroll
  for (int j = 0; j < L; j++) {
    tbl[0][j] = t[j];
    tbl[1][j] = base[j];
    t[j] = base[j];
  }
#pragma unroll 1
  for (int w = 2; w < 16; w++) {
    mont_mul_n<L, false>(t, t, nullptr, base, n, n0inv);
#pragma unroll
    for (int j = 0; j < L; j++) tbl[w][j] = t[j];
  }
  const int nwin = (int)(ebits + 3) >> 2;  // ebits >= 2
  auto window = [&](int i) -> uint32_t { return (e[i >> 3] >> ((i & 7) * 4)) & 15u; };
  const uint32_t top = window(nwin - 1);  // != 0: the exponent's top bit lies in it
  table_select<L>(acc, tbl, top);
#pragma unroll 1
  for (int i = nwin - 2; i >= 0; i--) {
#pragma unroll 1
    for (int s = 0; s < 4; s++) mont_sqr_n<L>(acc, n, n0inv);
    table_select<L>(t, tbl, window(i));
    mont_mul_n<L, false>(acc, acc, nullptr, t, n, n0inv);
  }
}

// EM^d mod prime (canonical, < prime) for the prime's key constants.
__device__ __forceinline__ void crt_half(uint32_t (&out)[kLh], const uint32_t (&hl)[10], cptr cpad, cptr pr,
                                         uint32_t p0inv, cptr r3, cptr d, uint32_t dbits) {
  uint32_t base[kLh], acc[kLh];
  // EM * R^-1 mod p by REDC of the 74-limb EM (EM < 2^2048 < R*p)
  redc_wide<kLh>(base, [&](auto kc) -> uint64_t {
    constexpr int k = decltype(kc)::value;
    if constexpr (k < 10) return (uint64_t)hl[k] + cpad[k];
    else return cpad[k];
  }, pr, p0inv);
  const uint32_t unused[kLh] = {};
  mont_mul_n<kLh, true>(base, base, r3, unused, pr, p0inv);  // EM * R (Montgomery form)
  mont_pow<kLh>(acc, base, r3, d, dbits, pr, p0inv);
  redc_wide<kLh>(out, [&](auto kc) -> uint64_t {  // out of Montgomery form
    constexpr int k = decltype(kc)::value;
    if constexpr (k < kLh) return acc[k];
    else return 0;
  }, pr, p0inv);
  reduce_once<kLh>(out, pr);
}

__global__ __launch_bounds__(256, 3) void k_rsa_sign(const uint8_t* __restrict__ blob,
                                                     const uint64_t* __restrict__ goff,
                                                     const uint32_t* __restrict__ glen, uint32_t n,
                                                     const SignKey* __restrict__ key, uint8_t* __restrict__ sig,
                                                     uint32_t fault_idx) {
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  if (g >= n) return;
  uint32_t hl[10];
  {
    uint32_t h[8];
    sha256(blob + goff[g], glen[g], h);
    // H as an integer: digest word 0 is its most significant 32 bits
    uint32_t hw[8];
#pragma unroll
    for (int i = 0; i < 8; i++) hw[i] = h[7 - i];
#pragma unroll
    for (int j = 0; j < 10; j++) {
      const int bit = j * kLimbBits, wi = bit >> 5, sh = bit & 31;
      const uint64_t v = ((uint64_t)(wi + 1 < 8 ? hw[wi + 1] : 0u) << 32) | hw[wi];
      hl[j] = (uint32_t)(v >> sh) & kLimbMask;
    }
  }
  const cptr cpad = as_const(key->cpad);
  const cptr p = as_const(key->p), q = as_const(key->q);
  uint32_t m1[kLh], m2[kLh];
  crt_half(m1, hl, cpad, p, *as_const(&key->p0inv), as_const(key->r3p), as_const(key->dp), *as_const(&key->dp_bits));
  crt_half(m2, hl, cpad, q, *as_const(&key->q0inv), as_const(key->r3q), as_const(key->dq), *as_const(&key->dq_bits));
  if (g == fault_idx) m1[0] ^= 1u;  // test hook (mochi_signer_set_fault): a transient fault in one CRT half
  // Garner: h = qInv (m1 - m2 mod p) mod p
  uint32_t d[kLh];
#pragma unroll
  for (int j = 0; j < kLh; j++) d[j] = m2[j];
  reduce_once<kLh>(d, p);  // m2 < q < 2p
  int32_t br = 0;
#pragma unroll
  for (int j = 0; j < kLh; j++) {
    const int32_t t = (int32_t)m1[j] - (int32_t)d[j] - br;
    br = t < 0 ? 1 : 0;
    d[j] = (uint32_t)t & kLimbMask;
  }
  if (br) {  // m1 < m2 mod p: add p back
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kLh; j++) {
      const uint32_t t = d[j] + p[j] + c;
      d[j] = t & kLimbMask;
      c = t >> kLimbBits;
    }
  }
  const uint32_t unused[kLh] = {};
  mont_mul_n<kLh, true>(d, d, as_const(key->qinv_r), unused, p, *as_const(&key->p0inv));
  reduce_once<kLh>(d, p);
  // s = m2 + h q  (< p q = n < 2^2048), 74 limbs
  uint32_t s[kL];
  uint64_t carry = 0;
  static_for<0, kL>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    constexpr int lo = k - kLh + 1 > 0 ? k - kLh + 1 : 0;
    constexpr int hi = k < kLh - 1 ? k : kLh - 1;
    uint64_t acc0 = carry, acc1 = 0;
    if constexpr (k < kLh) acc1 = m2[k];
    static_for<lo, hi + 1>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      if constexpr (i & 1) acc1 = mad64(d[i], q[k - i], acc1);
      else acc0 = mad64(d[i], q[k - i], acc0);
    });
    const uint64_t acc = acc0 + acc1;
    s[k] = (uint32_t)acc & kLimbMask;
    carry = acc >> kLimbBits;
  });
  uint32_t w[64];
  limbs_to_words(s, w);
  uint4* out = (uint4*)(sig + (size_t)g * MOCHI_RSA_BYTES);
#pragma unroll
  for (int q4 = 0; q4 < 16; q4++)
    out[q4] = make_uint4(__builtin_bswap32(w[63 - 4 * q4]), __builtin_bswap32(w[62 - 4 * q4]),
                         __builtin_bswap32(w[61 - 4 * q4]), __builtin_bswap32(w[60 - 4 * q4]));
}

}  // namespace

size_t sign_key_bytes() { return sizeof(SignKey); }

// Host-side: fill a SignKey from big-endian CRT components (OpenSSL BN work in capi.cpp).
void sign_key_set(void* dst, const uint32_t* p, const uint32_t* q, const uint32_t* r3p, const uint32_t* r3q,
                  const uint32_t* qinv_r, const uint32_t* dp, const uint32_t* dq, const uint32_t* cpad, uint32_t p0inv,
                  uint32_t q0inv, uint32_t dp_bits, uint32_t dq_bits) {
  SignKey* k = (SignKey*)dst;
  for (int j = 0; j < kLh; j++) {
    k->p[j] = p[j];
    k->q[j] = q[j];
    k->r3p[j] = r3p[j];
    k->r3q[j] = r3q[j];
    k->qinv_r[j] = qinv_r[j];
  }
  for (int j = 0; j < 32; j++) {
    k->dp[j] = dp[j];
    k->dq[j] = dq[j];
  }
  for (int j = 0; j < kL; j++) k->cpad[j] = cpad[j];
  k->p0inv = p0inv;
  k->q0inv = q0inv;
  k->dp_bits = dp_bits;
  k->dq_bits = dq_bits;
}

hipError_t launch_rsa_sign(const uint8_t* blob, const uint64_t* goff, const uint32_t* glen, uint32_t n,
                           const void* key, uint8_t* sig, uint32_t fault_idx, hipStream_t st) {
  if (n)
    hipLaunchKernelGGL(k_rsa_sign, dim3((n + 255) / 256), dim3(256), 0, st, blob, goff, glen, n,
                       (const SignKey*)key, sig, fault_idx);
  return hipGetLastError();
}

}  // namespace mochi
