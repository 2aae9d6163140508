// fold_pow.hip — prototype: RSA-2048 squaring chain with the modular reduction
// on the matrix cores (model: fold_ref.py).
//
// Per squaring and lane (one signature per lane, 64 per wave):
//   t = x^2              VALU product scanning, 28-bit limbs, 2,775 v_mad_u64_u32
//   x = t_lo + W * t_hi  t_hi's 300 bytes times the key's fold matrix on
//                        v_mfma_i32_32x32x32_i8 (10 M-tiles x 10 K-steps x 2 N-tiles)
// The wave's 64 signatures form two 32-column N-tiles; v_permlane32_swap moves
// half of every operand / accumulator register across the wave halves so each
// lane keeps exactly its own signature's limbs.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace {

constexpr int kL = 74, kF = 73, kNH = 75, kKS = 10, kMT = 10;
constexpr uint32_t kM28 = (1u << 28) - 1;
#ifndef COMBINE_MAD
#define COMBINE_MAD 0
#endif
#ifndef MT_BARRIER
#define MT_BARRIER 1
#endif
#ifndef PRIO
#define PRIO 0
#endif
#ifndef DESYNC
#define DESYNC 0
#endif
#ifndef SQ_ONLY
#define SQ_ONLY 0
#endif
#ifndef MF_ONLY
#define MF_ONLY 0
#endif
#ifndef COLGROUP
#define COLGROUP 1
#endif
constexpr int kColGroup = COLGROUP;

typedef int v4i __attribute__((ext_vector_type(4)));
typedef int v16i __attribute__((ext_vector_type(16)));
typedef const __attribute__((address_space(4))) uint32_t* cptr32;

template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) { return (uint64_t)a * b + c; }

__device__ __forceinline__ void swap32(int& a, int& b) {
  auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
  a = r[0];
  b = r[1];
}

#ifndef STAMPS
#define STAMPS 0
#endif
__device__ __forceinline__ uint64_t stamp() {
#if STAMPS
  return __builtin_amdgcn_s_memtime();
#else
  return 0;
#endif
}

__device__ __forceinline__ void fold_sqr(uint32_t (&x)[kL], const v4i* __restrict__ wl, cptr32 corr, uint64_t (&acc)[3]) {
  const uint64_t s0 = stamp();
  uint32_t t[2 * kL];
#if MF_ONLY
#pragma unroll
  for (int q = 0; q < 2 * kL; q++) t[q] = (x[q % kL] + q) & kM28;
  if (0)
#endif
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
      t[k] = (uint32_t)acc & kM28;
      asm volatile("" : "+v"(t[k]));  // materialize the 28-bit limb (else the 64-bit column stays live)
      carry = acc >> 28;
      // product scanning, column by column: left alone the scheduler hoists
      // later columns' mads and keeps ~40 64-bit column sums live
      if constexpr ((k & (kColGroup - 1)) == kColGroup - 1) __builtin_amdgcn_sched_barrier(0);
    });
    t[2 * kL - 1] = (uint32_t)carry;
  }
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t s1 = stamp();
  acc[0] += s1 - s0;
#if SQ_ONLY
#pragma unroll
  for (int q = 0; q < kL; q++) x[q] = t[q] ^ t[q + 74];
  return;
#endif
#if PRIO
  __builtin_amdgcn_s_setprio(3);  // MFMA phase: issue MFMAs first, the partner wave's VALU fills the gaps
#endif
  // signature-side operands: bytes of t_hi biased to signed (b - 128)
  v4i b0[kKS], b1[kKS];
  static_for<0, kKS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<0, 4>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int jp = 8 * s + i, jq = 8 * s + 4 + i;
      int p = (int)0x80808080u, q = (int)0x80808080u;
      if constexpr (jp < kNH) p = (int)(t[kF + jp] ^ 0x80808080u);
      if constexpr (jq < kNH) q = (int)(t[kF + jq] ^ 0x80808080u);
      swap32(p, q);
      b0[s][i] = p;
      b1[s][i] = q;
    });
  });
  int64_t carry = 0;
  __builtin_amdgcn_sched_barrier(0);
  const uint64_t s2 = stamp();
  acc[1] += s2 - s1;
  static_for<0, kMT>([&](auto mc) {
    constexpr int mt = decltype(mc)::value;
#if MT_BARRIER
    __builtin_amdgcn_sched_barrier(0);
#endif
    v16i d0 = {}, d1 = {};
    // one K-step of weights in flight: a group = load(s+1), two MFMAs on s
    v4i a = wl[(mt * kKS) * 64];
    static_for<0, kKS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      v4i an = a;
      if constexpr (s + 1 < kKS) an = wl[(mt * kKS + s + 1) * 64];
      d0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b0[s], d0, 0, 0, 0);
      d1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b1[s], d1, 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
      a = an;
    });
    static_for<0, 16>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      int a = d0[v], b = d1[v];
      swap32(a, b);
      d0[v] = a;
      d1[v] = b;
    });
    static_for<0, 8>([&](auto rc) {
      constexpr int r = decltype(rc)::value;  // limb 8mt + r: even from d0, odd from d1
      constexpr int q = 8 * mt + r, u = r >> 1;
      if constexpr (q < kL) {
        const v16i& d = (r & 1) ? d1 : d0;
        // |c0 + 256 c1| < 1.27e9 and t_lo < 2^28: the low part stays in int32
        // (adding t_lo after widening keeps 73 zero-extended pairs live)
        int p = d[4 * u] + (d[4 * u + 1] << 8);
        if constexpr (q < kF) p += (int)t[q];
        const int h = d[4 * u + 2] + (d[4 * u + 3] << 8);
        const int64_t v = (int64_t)h * 65536 + ((int64_t)p + (int64_t)corr[q] + carry);
        x[q] = (uint32_t)v & kM28;
        carry = v >> 28;
      }
    });
  });
#if PRIO
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_setprio(0);
#endif
  __builtin_amdgcn_sched_barrier(0);
  acc[2] += stamp() - s2;
}

__device__ uint64_t g_stamps[6];

__global__ __launch_bounds__(512, 1) void k_fold_pow(const uint32_t* __restrict__ xin, const v4i* __restrict__ wimg,
                                                     const uint32_t* __restrict__ corr, uint32_t* __restrict__ zout,
                                                     uint32_t n, int iters) {
  __shared__ v4i w[kMT * kKS * 64];
#if STAMPS
  const uint64_t t_begin = stamp();
#endif
  for (int i = threadIdx.x; i < kMT * kKS * 64; i += blockDim.x) w[i] = wimg[i];
  __syncthreads();
  const uint32_t idx = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = idx < n;
  uint32_t x[kL];
  uint64_t acc[3] = {0, 0, 0};
#pragma unroll
  for (int j = 0; j < kL; j++) x[j] = active ? xin[(size_t)j * n + idx] : 0u;
  const cptr32 c = (cptr32)corr;
#if DESYNC
  // the second wave of every SIMD starts ~half a squaring late so the two
  // waves' MFMA phases do not coincide
  if (threadIdx.x >= 256) {
    __builtin_amdgcn_s_sleep(127);
    __builtin_amdgcn_s_sleep(80);
  }
#endif
#pragma unroll 1
  for (int it = 0; it < iters; it++) {
    cptr32 ci = c;
    asm volatile("" : "+s"(ci));  // keep the 74 corr loads inside the loop (148 SGPRs if hoisted)
    fold_sqr(x, w + (threadIdx.x & 63), ci, acc);
  }
  if (active) {
#pragma unroll
    for (int j = 0; j < kL; j++) zout[(size_t)j * n + idx] = x[j];
  }
#if STAMPS
  if ((threadIdx.x & 63) == 0) {  // per-phase cycles summed over waves (vector atomics)
    atomicAdd((unsigned long long*)&g_stamps[0], (unsigned long long)acc[0]);
    atomicAdd((unsigned long long*)&g_stamps[1], (unsigned long long)acc[1]);
    atomicAdd((unsigned long long*)&g_stamps[2], (unsigned long long)acc[2]);
    atomicAdd((unsigned long long*)&g_stamps[3], 1ull);
    atomicAdd((unsigned long long*)&g_stamps[4], (unsigned long long)(stamp() - t_begin));  // wave lifetime
  }
#endif
}

}  // namespace

extern "C" int fold_stamps(uint64_t* out, int reset) {
  if (reset) {
    uint64_t z[6] = {0, 0, 0, 0, 0, 0};
    return hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof z) != hipSuccess;
  }
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), 6 * sizeof(uint64_t)) != hipSuccess;
}

extern "C" int fold_pow(const uint32_t* xin, const void* wimg, const uint32_t* corr, uint32_t* zout, uint32_t n,
                        int iters, void* stream) {
  hipLaunchKernelGGL(k_fold_pow, dim3((n + 511) / 512), dim3(512), 0, (hipStream_t)stream, xin, (const v4i*)wimg,
                     corr, zout, n, iters);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
