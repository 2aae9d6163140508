// fold_dev.h — the modular fold on the matrix cores, shared by k_rsa_pow
// (rsa_pow.hip: 16 squarings) and k_rsa_final (rsa_final.hip: the multiply
// by s and the EMSA check).  Layout and bounds: fold.h.
//
// Given a 148-limb t (radix 2^28, t < 2^4144), fold_reduce writes the 74
// normalised limbs of
//     x = t_lo + sum_{j<75, b<4} byte_b(t_{73+j}) * R_{j,b} + cadd - h
// where t_lo = limbs 0..72, cadd is a per-key 74-limb constant (k_rsa_pow:
// the -128 bias correction; k_rsa_final: that plus n - Cpad) and h (k_rsa_final
// only) a 10-limb value subtracted in the low limbs.  The sum is
// v_mfma_i32_32x32x32_i8: 10 M-tiles x 10 K-steps x 2 N-tiles (the wave's 64
// signatures; lane l owns signature l).
//
// Fragments: a 32x32x32 B fragment gives lane l (half h = l >> 5) the K slots
// 16h..16h+15 of column l & 31, so one v_permlane32_swap per operand register
// pair turns "own t_hi limbs 8s+0..3 | 8s+4..7" into the two N-tiles'
// operands; one swap per accumulator pair turns the D fragments (half h =
// rows 4h + 8u + 0..3 = limb 2u + h of the M-tile) back into "own even | own
// odd" limbs.  A fragments are read from LDS (the key's image) one K-step ahead.
#pragma once
#include <atomic>

#include "fold.h"
#include "kara_dev.h"
#include "mont.h"

namespace mochi {

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

constexpr int kHL = 10;  // a SHA-256 digest in radix 2^28

// global-address-space pointers (keep global_load with an SGPR base + VGPR
// offset where an asm barrier would otherwise erase the address space)
typedef __attribute__((address_space(1))) char gchar;
typedef __attribute__((address_space(1))) uint32_t guint;

// BIASED: t_hi limbs (t[kFoldF..]) arrive already XOR kFoldBias.  t_lo limbs
// may be signed (Karatsuba's t[37..72], |t| < 2^29: kara_dev.h).
template <bool SUB_H, bool BIASED = false>
__device__ __forceinline__ void fold_reduce(const uint32_t (&t)[2 * kL], uint32_t (&x)[kL],
                                            const v4i* __restrict__ wl, cptr cadd, const uint32_t* hl) {
  // tile 0's first A fragment: issued before the B operands are formed (their
  // ~150 VALU ops cover the LDS latency); every later tile's first fragment is
  // prefetched by the previous tile's last K-step
  v4i a = wl[0];
  // ---- B operands: t_hi bytes biased to signed (b - 128), split over the halves ----
  v4i b0[kFoldKS], b1[kFoldKS];
  static_for<0, kFoldKS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<0, 4>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int jp = 8 * s + i, jq = 8 * s + 4 + i;
      int p = 0, q = 0;  // padding K slots: their weights are zero
      if constexpr (jp < kFoldNH) p = (int)(BIASED ? t[kFoldF + jp] : t[kFoldF + jp] ^ kFoldBias);
      if constexpr (jq < kFoldNH) q = (int)(BIASED ? t[kFoldF + jq] : t[kFoldF + jq] ^ kFoldBias);
      swap32(p, q);  // p: N-tile 0 (signatures 0..31), q: N-tile 1 (32..63)
      b0[s][i] = p;
      b1[s][i] = q;
    });
  });
  // ---- x = t_lo + fold(t_hi) + cadd (- h), M-tile by M-tile, carries low to high ----
  int64_t carry = 0;
  // one M-tile: 10 K-steps x 2 N-tiles, the next A fragment read one step ahead
  auto mfma_step = [&](auto mc, auto sc, v16i& d0, v16i& d1) {
    constexpr int mt = decltype(mc)::value, s = decltype(sc)::value;
    v4i an = a;
    if constexpr (mt * kFoldKS + s + 1 < kFoldMT * kFoldKS) an = wl[(mt * kFoldKS + s + 1) * 64];
    d0 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b0[s], d0, 0, 0, 0);
    d1 = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b1[s], d1, 0, 0, 0);
    a = an;
  };
  // the limbs of M-tile mt from its accumulators
  auto assemble = [&](auto mc, const v16i& d0, const v16i& d1) {
    constexpr int mt = decltype(mc)::value;
    // the two halves of each limb (c0 + 2^8 c1 and c2 + 2^8 c3) in the MFMA's
    // own layout -- half h of the wave holds limb 2u + h of both N-tiles'
    // signatures, all four digits in one lane (rows 4h + 8u + 0..3) -- then one
    // swap per half turns "limb 2u+h of signatures l and l+32" into "limbs 2u
    // and 2u+1 of my own signature": 8 swaps per tile instead of 16 on the digits
    int p0[4], h0[4], p1[4], h1[4];
    static_for<0, 4>([&](auto uc) {
      constexpr int u = decltype(uc)::value;
      p0[u] = d0[4 * u] + (d0[4 * u + 1] << 8);
      h0[u] = d0[4 * u + 2] + (d0[4 * u + 3] << 8);
      p1[u] = d1[4 * u] + (d1[4 * u + 1] << 8);
      h1[u] = d1[4 * u + 2] + (d1[4 * u + 3] << 8);
      swap32(p0[u], p1[u]);  // p0: own limb 2u, p1: own limb 2u + 1
      swap32(h0[u], h1[u]);
    });
    static_for<0, 8>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      constexpr int q = 8 * mt + r, u = r >> 1;
      if constexpr (q < kL) {
        // limb q = c0 + 2^8 c1 + 2^16 (c2 + 2^8 c3) + t_lo + cadd (- h) + carry;
        // p = c0 + 2^8 c1 + t_lo + cadd (- h) stays in int32: |c0 + 2^8 c1| <=
        // 257 * 300 * 2^14 = 1,263,206,400, |t_lo| < 2^29 (signed Karatsuba
        // limbs), cadd and h < 2^28, so -1.80e9 < p < 2.07e9 < 2^31
        // (tests/fold_model.py asserts it); h * 2^16 + p + carry is two
        // v_mad_i64_i32
        int p = (r & 1) ? p1[u] : p0[u];
        if constexpr (q < kFoldF) p += (int)t[q];
        p += (int)cadd[q];
        if constexpr (SUB_H && q < kHL) p -= (int)hl[q];
        const int h = (r & 1) ? h1[u] : h0[u];
        const int64_t v = mad_i64(h, 65536, mad_i64(p, 1, carry));
        x[q] = (uint32_t)v & kLimbMask;
        carry = v >> kLimbBits;
      }
    });
  };
  static_for<0, kFoldMT>([&](auto mc) {
    __builtin_amdgcn_sched_barrier(0);
    v16i d0 = {}, d1 = {};
    static_for<0, kFoldKS>([&](auto sc) {  // one K-step of weights in flight
      mfma_step(mc, sc, d0, d1);
      __builtin_amdgcn_sched_barrier(0);
    });
    assemble(mc, d0, d1);
  });
}

// ---------------------------------------------------------------------------
// The fold split over a block's four waves for the latency kernels of small
// batches (k_rsa_pow_lat, k_rsa_final_lat): every wave holds the same 64 slots;
// t sits in the LDS exchange rows xr (lane-major), wave w folds M-tiles w, w+4,
// w+8 and writes each output limb's two int32 halves (p, h) back into the rows;
// the limb arithmetic is fold_reduce's, split by tile (bit-exact with it).
// ---------------------------------------------------------------------------
#ifndef MOCHI_LAT_SEQ_TILES
#define MOCHI_LAT_SEQ_TILES 0  // A/B: the latency kernels' M-tiles one after the other
#endif
constexpr uint32_t kLatChunk = 64;
constexpr int kLatRows = 2 * kL + 1;  // 149 rows: H + M, then t (148), then the (p, h) pairs (148)

// The (p, h) halves of output limb q of an M-tile from its accumulators (the
// MFMA layout: half h of the wave holds limb 2u + h of both N-tiles'
// signatures; one swap per half turns them into this lane's own limbs)
template <int MT, bool SUB_H>
__device__ __forceinline__ void lat_assemble(const v16i& d0, const v16i& d1, cptr cadd,
                                             const uint32_t (*xr)[kLatChunk], uint32_t lane, const uint32_t (&hl)[kHL],
                                             int (&po)[8], int (&ho)[8]) {
  int p0[4], h0[4], p1[4], h1[4];
  static_for<0, 4>([&](auto uc) {
    constexpr int u = decltype(uc)::value;
    p0[u] = d0[4 * u] + (d0[4 * u + 1] << 8);
    h0[u] = d0[4 * u + 2] + (d0[4 * u + 3] << 8);
    p1[u] = d1[4 * u] + (d1[4 * u + 1] << 8);
    h1[u] = d1[4 * u + 2] + (d1[4 * u + 3] << 8);
    swap32(p0[u], p1[u]);  // p0: own limb 2u, p1: own limb 2u + 1
    swap32(h0[u], h1[u]);
  });
  static_for<0, 8>([&](auto rc) {
    constexpr int r = decltype(rc)::value;
    constexpr int q = 8 * MT + r, u = r >> 1;
    if constexpr (q < kL) {
      int p = (r & 1) ? p1[u] : p0[u];
      if constexpr (q < kFoldF) p += (int)xr[q][lane];  // t_lo (signed Karatsuba limbs)
      p += (int)cadd[q];
      if constexpr (SUB_H && q < kHL) p -= (int)hl[q];  // k_rsa_final_lat: - H, as fold_reduce<true>
      po[r] = p;
      ho[r] = (r & 1) ? h1[u] : h0[u];
    }
  });
}

// The M-tiles MT0, MT0 + 4, MT0 + 8 (< 10) of one wave, their K-steps
// interleaved (4-6 independent MFMA chains: alone on its SIMD a wave would
// otherwise wait out each chain's latency), then -- once the block has finished
// reading t (barrier 3, inside) -- the (p, h) pairs stored at rows 2q, 2q + 1.
// !kTwo: slots 32-63 of the chunk are empty (a bucket fills from its start), so
// the second N-tile (signatures 32-63) is skipped -- half the MFMAs; lanes
// 32-63 then carry garbage, and they are never stored (a batcher flush of a few
// messages has 1-2 grants per signer bucket).
template <int MT0, bool kTwo, bool SUB_H = false>
__device__ __forceinline__ void lat_fold(const v4i* wl, cptr cadd, uint32_t (*xr)[kLatChunk], uint32_t lane,
                                         const uint32_t (&hl)[kHL]) {
  constexpr int NT = MT0 + 8 < kFoldMT ? 3 : 2;
  v4i b0[kFoldKS], b1[kFoldKS];
  static_for<0, kFoldKS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<0, 4>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int jp = 8 * s + i, jq = 8 * s + 4 + i;
      int p = 0, q = 0;  // t_hi arrives biased (kara_combine); padding K slots have zero weights
      if constexpr (jp < kFoldNH) p = (int)xr[kFoldF + jp][lane];
      if constexpr (jq < kFoldNH) q = (int)xr[kFoldF + jq][lane];
      swap32(p, q);
      b0[s][i] = p;
      b1[s][i] = q;
    });
  });
  v16i d0[NT], d1[NT];
  static_for<0, NT>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    d0[j] = v16i{};
    d1[j] = v16i{};
  });
#if MOCHI_LAT_SEQ_TILES
  static_for<0, NT>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    static_for<0, kFoldKS>([&](auto sc) {
      constexpr int s = decltype(sc)::value;
      const v4i a = wl[((MT0 + 4 * j) * kFoldKS + s) * 64];
      d0[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b0[s], d0[j], 0, 0, 0);
      if constexpr (kTwo) d1[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b1[s], d1[j], 0, 0, 0);
      __builtin_amdgcn_sched_barrier(0);
    });
  });
#else
  static_for<0, kFoldKS>([&](auto sc) {
    constexpr int s = decltype(sc)::value;
    static_for<0, NT>([&](auto jc) {
      constexpr int j = decltype(jc)::value;
      const v4i a = wl[((MT0 + 4 * j) * kFoldKS + s) * 64];
      d0[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b0[s], d0[j], 0, 0, 0);
      if constexpr (kTwo) d1[j] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b1[s], d1[j], 0, 0, 0);
    });
  });
#endif
  int po[3][8] = {}, ho[3][8] = {};
  static_for<0, NT>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    lat_assemble<MT0 + 4 * j, SUB_H>(d0[j], d1[j], cadd, xr, lane, hl, po[j], ho[j]);
  });
  __syncthreads();  // barrier 3: every wave is done reading t
  static_for<0, NT>([&](auto jc) {
    constexpr int j = decltype(jc)::value;
    constexpr int mt = MT0 + 4 * j;
    static_for<0, 8>([&](auto rc) {
      constexpr int r = decltype(rc)::value;
      constexpr int q = 8 * mt + r;
      if constexpr (q < kL) {
        xr[2 * q][lane] = (uint32_t)po[j][r];
        xr[2 * q + 1][lane] = (uint32_t)ho[j][r];
      }
    });
  });
}


// Persistent walk over 512-slot groups of one signer (buckets are 512-aligned):
// block b takes a contiguous range of groups; fn(base, key) runs per non-empty
// group after the signer's fold image is staged in `w` (restaged only when the
// key changes along the range — block-uniform).
// ctr (optional): groups are taken from this device counter (zeroed before the
// launch) instead of a contiguous range -- a CU that starts late or clocks lower
// does fewer; the next index is fetched one group ahead, so the atomic's round
// trip runs under the current group
template <typename F>
__device__ __forceinline__ void for_groups(const uint32_t* __restrict__ perm, uint32_t n_slots,
                                           const uint16_t* __restrict__ signer, const FoldKey* __restrict__ fold,
                                           v4i* w, F&& fn, uint32_t* ctr = nullptr) {
  const uint32_t n_groups = (n_slots + kBucketAlign - 1) / kBucketAlign;
  __shared__ uint32_t s_grp[2];
  const bool dyn = ctr != nullptr;  // kernel argument: uniform
  uint32_t grp, g_end, it = 0;
  if (dyn) {
    if (threadIdx.x == 0) s_grp[0] = atomicAdd(ctr, 1u);
    __syncthreads();
    grp = __builtin_amdgcn_readfirstlane(s_grp[0]);
    g_end = n_groups;
  } else {
    grp = (uint32_t)((uint64_t)blockIdx.x * n_groups / gridDim.x);
    g_end = (uint32_t)((uint64_t)(blockIdx.x + 1) * n_groups / gridDim.x);
  }
  uint32_t cur_key = 0xFFFFFFFFu;
  while (grp < g_end) {
    uint32_t nxt = 0;
    if (dyn && threadIdx.x == 0) nxt = atomicAdd(ctr, 1u);
    const uint32_t base = grp * kBucketAlign;
    // buckets are 512-aligned and padded only at their tail: a group whose
    // first slot is empty is all padding (every thread reads the same slot)
    const uint32_t g_lead = __builtin_amdgcn_readfirstlane(perm[base]);
    if (g_lead != 0xFFFFFFFFu) {
      const uint32_t key = __builtin_amdgcn_readfirstlane((uint32_t)signer[g_lead]);
      if (key != cur_key) {
        __syncthreads();  // the old image is no longer read
        const v4i* src = (const v4i*)fold[key].img;
        for (uint32_t i = threadIdx.x; i < kFoldImgBytes / 16; i += blockDim.x) w[i] = src[i];
        __syncthreads();
        cur_key = key;
      }
      fn(base, key, g_lead);
    }
    if (dyn) {
      it ^= 1;
      if (threadIdx.x == 0) s_grp[it] = nxt;
      __syncthreads();
      grp = __builtin_amdgcn_readfirstlane(s_grp[it]);
    } else {
      grp++;
    }
  }
}

// one persistent 512-thread block per CU (the 100 KB image allows one per CU).
// The CU count is cached per device in atomics: several host threads launch
// concurrently (batcher flushers, multi-GPU workers, pipelined contexts).
inline uint32_t fold_grid(uint32_t n_slots) {
  static std::atomic<int> n_cu[64];  // zero-initialised (static storage)
  int dev = 0;
  (void)hipGetDevice(&dev);
  uint32_t cus = 256u;
  if (dev >= 0 && dev < 64) {
    int v = n_cu[dev].load(std::memory_order_relaxed);
    if (v == 0) {
      if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
      n_cu[dev].store(v, std::memory_order_relaxed);  // every writer stores the same value
    }
    cus = (uint32_t)v;
  }
  const uint32_t groups = (n_slots + kBucketAlign - 1) / kBucketAlign;
  return groups < cus ? groups : cus;
}

}  // namespace mochi
