// rsa_pow.hip — k_rsa_pow: the RSA-2048 squaring chain z = s^(2^16) mod n
// (z < 2^2064, not fully reduced), one signature per lane, with the modular
// reduction on the matrix cores (fold.h):
//
//   per squaring   t = x^2          VALU product scanning, 2,775 v_mad_u64_u32
//                  x = t_lo + W t_hi  v_mfma_i32_32x32x32_i8, 10 M-tiles x 10 K-steps
//                                   x 2 N-tiles (the wave's 64 signatures)
//
// versus 8,251 v_mad_u64_u32 per squaring for a Montgomery squaring on the
// VALU alone (mont.h): the m*n half of Montgomery's work, a product with the
// fixed modulus, becomes a product with a fixed matrix — shared by every
// signature of the signer, so it is GEMM-shaped.
//
// Lanes and MFMA fragments: lane l owns signature l of the wave.  An N-tile is
// 32 signatures, and a 32x32x32 B fragment gives lane l (half h = l >> 5) the
// K slots 16h..16h+15 of column l & 31, so one v_permlane32_swap per operand
// register pair turns "own t_hi limbs 8s+0..3 | 8s+4..7" into the two N-tiles'
// operands; one swap per accumulator pair turns the D fragments (half h = rows
// 4h + 8u + 0..3 = limb 2u + h of the M-tile) back into "own even | own odd".
//
// Group = 512 slots of ONE signer (buckets are 512-aligned), block = 8 waves
// = one group at a time; the signer's 100 KB image is staged in LDS; 2 waves
// per SIMD; persistent blocks, one per CU.
#include "fold.h"
#include "rsa_common.h"

namespace mochi {
namespace {

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));

__device__ __forceinline__ void swap32(int& a, int& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}

// d = a * b + c, signed 32 x 32 + 64 (one v_mad_i64_i32; hipcc otherwise
// sign-extends, shifts and adds in four instructions)
__device__ __forceinline__ int64_t mad_i64(int32_t a, int32_t b, int64_t c) {
  int64_t d;
  uint64_t cc;
  asm("v_mad_i64_i32 %0, %1, %2, %3, %4" : "=v"(d), "=s"(cc) : "v"(a), "s"(b), "v"(c));
  return d;
}

__device__ __forceinline__ void fold_sqr(uint32_t (&x)[kL], const v4i* __restrict__ wl, cptr cadd) {
  // ---- t = x^2: product scanning, cross products once, column sum doubled ----
  uint32_t t[2 * kL];
  {
    uint64_t carry = 0;
    static_for<0, 2 * kL - 1>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      constexpr int lo = k - kL + 1 > 0 ? k - kL + 1 : 0;
      constexpr int xhi = k > 0 ? (k - 1) / 2 : -1;
      uint64_t x0 = 0, x1 = 0;
      static_for<lo, xhi + 1>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        if constexpr (i & 1) x1 = mad64(x[i], x[k - i], x1);
        else x0 = mad64(x[i], x[k - i], x0);
      });
      uint64_t xs = x0 + x1;
      asm("" : "+v"(xs));  // double the column sum once (else hipcc doubles every x_i: extra mads and registers)
      uint64_t acc = carry + (xs << 1);
      if constexpr ((k & 1) == 0) acc = mad64(x[k >> 1], x[k >> 1], acc);
      t[k] = (uint32_t)acc & kLimbMask;
      asm volatile("" : "+v"(t[k]));  // materialise the 28-bit limb (else the 64-bit column stays live)
      carry = acc >> kLimbBits;
      // column by column: left alone the scheduler hoists later columns' mads
      // and keeps ~40 64-bit column sums live
      __builtin_amdgcn_sched_barrier(0);
    });
    t[2 * kL - 1] = (uint32_t)carry;
  }
  // ---- B operands: t_hi bytes biased to signed (b - 128), split over the halves ----
  v4i b0[kFoldKS], b1[kFoldKS];
  static_for<0, kFoldKS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<0, 4>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int jp = 8 * s + i, jq = 8 * s + 4 + i;
      int p = (int)0x80808080u, q = (int)0x80808080u;
      if constexpr (jp < kFoldNH) p = (int)(t[kFoldF + jp] ^ 0x80808080u);
      if constexpr (jq < kFoldNH) q = (int)(t[kFoldF + jq] ^ 0x80808080u);
      swap32(p, q);  // p: N-tile 0 (signatures 0..31), q: N-tile 1 (32..63)
      b0[s][i] = p;
      b1[s][i] = q;
    });
  });
  // ---- x = t_lo + fold(t_hi), M-tile by M-tile, carries low to high ----
  int64_t carry = 0;
  static_for<0, kFoldMT>([&](auto mc) {
    constexpr int mt = decltype(mc)::value;
    __builtin_amdgcn_sched_barrier(0);
    v16i d0 = {}, d1 = {};
    v4i a = wl[(mt * kFoldKS) * 64];
    static_for<0, kFoldKS>([&](auto sc) {  // one K-step of weights in flight
      constexpr int s = decltype(sc)::value;
      v4i an = a;
      if constexpr (s + 1 < kFoldKS) an = wl[(mt * kFoldKS + s + 1) * 64];
      d0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b0[s], d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b1[s], d1, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      a = an;
    });
    static_for<0, 16>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      int e = d0[v], o = d1[v];
      swap32(e, o);  // e: own even limbs, o: own odd limbs
      d0[v] = e;
      d1[v] = o;
    });
    static_for<0, 8>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      constexpr int q = 8 * mt + r, u = r >> 1;
      if constexpr (q < kL) {
        const v16i& d = (r & 1) ? d1 : d0;
        // limb q = c0 + 2^8 c1 + 2^16 (c2 + 2^8 c3) + t_lo + cadd + carry; the
        // first four terms of p stay in int32 (|c0 + 2^8 c1| < 1.27e9, t_lo and
        // cadd < 2^28), h * 2^16 + p + carry is two v_mad_i64_i32
        int p = d[4 * u] + (d[4 * u + 1] << 8);
        if constexpr (q < kFoldF) p += (int)t[q];
        p += (int)cadd[q];
        const int h = d[4 * u + 2] + (d[4 * u + 3] << 8);
        const int64_t v = mad_i64(h, 65536, mad_i64(p, 1, carry));
        x[q] = (uint32_t)v & kLimbMask;
        carry = v >> kLimbBits;
      }
    });
  });
}

// Persistent: one block per CU walks a contiguous range of 512-slot groups, so
// the CU never idles between blocks (a block's 8 waves would otherwise all wait
// for its slowest before the next block could take the LDS) and the signer's
// image is staged only when the key changes along the range (block-uniform).
__global__ __launch_bounds__(512, 1) void k_rsa_pow(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                                    const uint8_t* __restrict__ sig,
                                                    const uint16_t* __restrict__ signer,
                                                    const FoldKey* __restrict__ fold, uint32_t* __restrict__ zout) {
  __shared__ v4i w[kFoldImgBytes / 16];
  const uint32_t n_groups = (n_slots + kBucketAlign - 1) / kBucketAlign;
  const uint32_t g_begin = (uint32_t)((uint64_t)blockIdx.x * n_groups / gridDim.x);
  const uint32_t g_end = (uint32_t)((uint64_t)(blockIdx.x + 1) * n_groups / gridDim.x);
  uint32_t cur_key = 0xFFFFFFFFu;
  for (uint32_t grp = g_begin; grp < g_end; grp++) {
    const uint32_t base = grp * kBucketAlign;
    // buckets are 512-aligned and padded only at their tail: a group whose
    // first slot is empty is all padding (every thread reads the same slot)
    const uint32_t g_lead = __builtin_amdgcn_readfirstlane(perm[base]);
    if (g_lead == 0xFFFFFFFFu) continue;
    const uint32_t key = __builtin_amdgcn_readfirstlane((uint32_t)signer[g_lead]);
    if (key != cur_key) {  // block-uniform: every wave walks the same groups
      __syncthreads();     // the old image is no longer read
      const v4i* src = (const v4i*)fold[key].img;
      for (uint32_t i = threadIdx.x; i < kFoldImgBytes / 16; i += blockDim.x) w[i] = src[i];
      __syncthreads();
      cur_key = key;
    }
    const uint32_t slot = base + threadIdx.x;
    const uint32_t g = slot < n_slots ? perm[slot] : 0xFFFFFFFFu;
    const bool active = g != 0xFFFFFFFFu;
    if (__ballot(active) == 0) continue;  // this wave's quarter of the group is padding
    uint32_t x[kL];
    {
      uint32_t wd[64];
      load_sig_words(sig, active ? g : g_lead, wd);  // inactive lanes shadow the lead grant (never stored)
      words_to_limbs(wd, x);
    }
    const cptr c = as_const(fold[key].cadd);
#pragma unroll 1
    for (int it = 0; it < 16; it++) {
      cptr ci = c;
      asm volatile("" : "+s"(ci));  // keep the 74 cadd loads inside the loop (SGPR pressure if hoisted)
      fold_sqr(x, w + (threadIdx.x & 63), ci);
    }
    if (active) {
#pragma unroll
      for (int j = 0; j < kL; j++) zout[(size_t)j * n_slots + slot] = x[j];
    }
  }
}

}  // namespace

void launch_rsa_pow(const LaunchArgs& a, hipStream_t st) {
  // one persistent block per CU (the 100 KB image allows one block per CU)
  static int n_cu[64] = {0};
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev >= 0 && dev < 64 && n_cu[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    n_cu[dev] = v;
  }
  const uint32_t cus = dev >= 0 && dev < 64 ? (uint32_t)n_cu[dev] : 256u;
  const uint32_t groups = (a.n_slots + kBucketAlign - 1) / kBucketAlign;
  const uint32_t blocks = groups < cus ? groups : cus;
  if (blocks)
    hipLaunchKernelGGL(k_rsa_pow, dim3(blocks), dim3(kBucketAlign), 0, st, a.perm, a.n_slots, a.sig, a.signer, a.fold,
                       a.xbuf);
}

}  // namespace mochi
