// Integer-VALU peak microbenchmark for gfx950 (MI355X).
//
// Measures the sustained chip-wide issue rate of the instructions a
// multi-precision Montgomery multiply can be built from, so that the
// verify kernel's roofline (P_MAC = measured peak
// v_mad_u64_u32 rate of one MI355X) is a measured number, not a guess.
//
// Each kernel runs 8 independent dependency chains per lane of one
// instruction kind, issued through inline asm so the compiler cannot fold
// or re-associate them.  Build: make -C microbench ; run: ./microbench/int_peak
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

constexpr int kChains = 8;
constexpr int kUnroll = 8;   // asm statements per chain per iteration

// v_mad_u64_u32: 32x32 -> 64 multiply + 64-bit accumulate, carry out to SGPR pair.
__global__ __launch_bounds__(256) void k_mad_u64(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = seed * (threadIdx.x + 1), b = seed ^ (threadIdx.x * 0x9E3779B9u);
  uint64_t acc[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) acc[i] = (uint64_t)(i + threadIdx.x) << 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
#pragma unroll
      for (int i = 0; i < kChains; i++) {
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(c) : "v"(a), "v"(b));
      }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// Comba step: v_mad_u64_u32 with carry-out + v_addc_co_u32 into a third word.
__global__ __launch_bounds__(256) void k_comba(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = seed * (threadIdx.x + 1), b = seed ^ (threadIdx.x * 0x9E3779B9u);
  uint64_t acc[kChains];
  uint32_t hi[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) { acc[i] = (uint64_t)(i + threadIdx.x) << 7; hi[i] = 0; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
#pragma unroll
      for (int i = 0; i < kChains; i++) {
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %3, %4, %0\n\tv_addc_co_u32_e64 %2, %1, %2, 0, %1"
                     : "+v"(acc[i]), "=&s"(c), "+v"(hi[i]) : "v"(a), "v"(b));
      }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s ^= acc[i] ^ hi[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define SIMPLE_KERNEL(NAME, ASM)                                                        \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed, int iters) { \
    uint32_t a = seed * (threadIdx.x + 1), b = seed ^ (threadIdx.x * 0x9E3779B9u);      \
    uint32_t acc[kChains];                                                              \
    _Pragma("unroll") for (int i = 0; i < kChains; i++) acc[i] = i + threadIdx.x;      \
    for (int it = 0; it < iters; it++) {                                                \
      _Pragma("unroll") for (int u = 0; u < kUnroll; u++)                               \
      _Pragma("unroll") for (int i = 0; i < kChains; i++)                               \
        asm volatile(ASM : "+v"(acc[i]) : "v"(a), "v"(b));                              \
    }                                                                                   \
    uint64_t s = 0;                                                                     \
    _Pragma("unroll") for (int i = 0; i < kChains; i++) s ^= acc[i];                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                     \
  }

SIMPLE_KERNEL(k_mul_lo, "v_mul_lo_u32 %0, %1, %0")
SIMPLE_KERNEL(k_mul_hi, "v_mul_hi_u32 %0, %1, %0")
SIMPLE_KERNEL(k_mad_u24, "v_mad_u32_u24 %0, %1, %2, %0")
SIMPLE_KERNEL(k_mulhi_u24, "v_mul_hi_u32_u24 %0, %1, %0")
SIMPLE_KERNEL(k_add, "v_add_u32 %0, %1, %0")
SIMPLE_KERNEL(k_add3, "v_add3_u32 %0, %1, %2, %0")
SIMPLE_KERNEL(k_dot2_u16, "v_dot2_u32_u16 %0, %1, %2, %0")

__global__ __launch_bounds__(256) void k_fma_f64(uint64_t* out, uint32_t seed, int iters) {
  double a = 1.0 + 1e-9 * threadIdx.x, b = 0.999999 + 1e-12 * seed;
  double acc[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) acc[i] = i + threadIdx.x;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
#pragma unroll
      for (int i = 0; i < kChains; i++) asm volatile("v_fma_f64 %0, %1, %2, %0" : "+v"(acc[i]) : "v"(a), "v"(b));
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}


SIMPLE_KERNEL(k_add_e64, "v_add_u32_e64 %0, %1, %0")
SIMPLE_KERNEL(k_mul_u24_e32, "v_mul_u32_u24_e32 %0, %1, %0")
SIMPLE_KERNEL(k_mulhi_u24_e32, "v_mul_hi_u32_u24_e32 %0, %1, %0")
SIMPLE_KERNEL(k_fmac_f32, "v_fmac_f32_e32 %0, %1, %2")
SIMPLE_KERNEL(k_fma_f32, "v_fma_f32 %0, %1, %2, %0")
SIMPLE_KERNEL(k_alignbit, "v_alignbit_b32 %0, %1, %0, 7")
SIMPLE_KERNEL(k_and_or, "v_and_or_b32 %0, %1, %2, %0")

// Comba step with the carry routed through VCC so the addc is a 4-byte VOP2.
__global__ __launch_bounds__(256) void k_comba_vcc(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = seed * (threadIdx.x + 1), b = seed ^ (threadIdx.x * 0x9E3779B9u);
  uint64_t acc[kChains];
  uint32_t hi[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) { acc[i] = (uint64_t)(i + threadIdx.x) << 7; hi[i] = 0; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
#pragma unroll
      for (int i = 0; i < kChains; i++) {
        asm volatile("v_mad_u64_u32 %0, vcc, %2, %3, %0\n\tv_addc_co_u32_e32 %1, vcc, 0, %1, vcc"
                     : "+v"(acc[i]), "+v"(hi[i]) : "v"(a), "v"(b) : "vcc");
      }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s ^= acc[i] ^ hi[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// v_mad_u64_u32 with one operand from an SGPR (wave-uniform modulus limb).
__global__ __launch_bounds__(256) void k_mad_u64_sgpr(uint64_t* out, uint32_t seed, int iters) {
  uint32_t a = seed * (threadIdx.x + 1);
  uint32_t bs = __builtin_amdgcn_readfirstlane(seed * 7u);
  uint64_t acc[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) acc[i] = (uint64_t)(i + threadIdx.x) << 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
#pragma unroll
      for (int i = 0; i < kChains; i++) {
        uint64_t c;
        asm volatile("v_mad_u64_u32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(c) : "v"(a), "s"(bs));
      }
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

#define SIMPLE64_KERNEL(NAME, ASM)                                                      \
  __global__ __launch_bounds__(256) void NAME(uint64_t* out, uint32_t seed, int iters) { \
    uint32_t a = seed * (threadIdx.x + 1);                                              \
    uint64_t b = ((uint64_t)seed << 32) ^ (threadIdx.x * 0x9E3779B97F4A7C15ull);        \
    uint64_t acc[kChains];                                                              \
    _Pragma("unroll") for (int i = 0; i < kChains; i++) acc[i] = (uint64_t)(i + threadIdx.x) << 20; \
    for (int it = 0; it < iters; it++) {                                                \
      _Pragma("unroll") for (int u = 0; u < kUnroll; u++)                               \
      _Pragma("unroll") for (int i = 0; i < kChains; i++)                               \
        asm volatile(ASM : "+v"(acc[i]) : "v"(a), "v"(b));                              \
    }                                                                                   \
    uint64_t s = 0;                                                                     \
    _Pragma("unroll") for (int i = 0; i < kChains; i++) s ^= acc[i];                    \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                     \
  }

// the glue of k_rsa_pow's x^2 columns and fold reassembly (rsa_pow.hip, fold_dev.h)
SIMPLE64_KERNEL(k_lshl_add_u64, "v_lshl_add_u64 %0, %0, 1, %2")
SIMPLE64_KERNEL(k_lshrrev_b64, "v_lshrrev_b64 %0, 28, %0")
SIMPLE64_KERNEL(k_ashrrev_i64, "v_ashrrev_i64 %0, 28, %0")
SIMPLE_KERNEL(k_and, "v_and_b32 %0, %1, %0")
SIMPLE_KERNEL(k_xor, "v_xor_b32 %0, %1, %0")
SIMPLE_KERNEL(k_lshl_add_u32, "v_lshl_add_u32 %0, %1, 8, %0")

__global__ __launch_bounds__(256) void k_mad_i64(uint64_t* out, uint32_t seed, int iters) {
  int32_t a = (int32_t)(seed * (threadIdx.x + 1)), b = (int32_t)(seed ^ (threadIdx.x * 0x9E3779B9u));
  int64_t acc[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) acc[i] = (int64_t)(i + threadIdx.x) << 7;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
#pragma unroll
      for (int i = 0; i < kChains; i++) {
        uint64_t c;
        asm volatile("v_mad_i64_i32 %0, %1, %2, %3, %0" : "+v"(acc[i]), "=s"(c) : "v"(a), "v"(b));
      }
  }
  int64_t s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s ^= acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = (uint64_t)s;
}

__global__ __launch_bounds__(256) void k_permlane32_swap(uint64_t* out, uint32_t seed, int iters) {
  uint32_t x[kChains], y[kChains];
#pragma unroll
  for (int i = 0; i < kChains; i++) { x[i] = seed + i + threadIdx.x; y[i] = seed ^ i; }
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int u = 0; u < kUnroll; u++)
#pragma unroll
      for (int i = 0; i < kChains; i++) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(x[i]), "+v"(y[i]));
  }
  uint64_t s = 0;
#pragma unroll
  for (int i = 0; i < kChains; i++) s ^= x[i] ^ y[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef void (*kfn)(uint64_t*, uint32_t, int);

static double run(const char* name, kfn f, int insts_per_step, uint64_t* d, int blocks, int iters) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 12345u, iters);  // warmup
  CHECK(hipDeviceSynchronize());
  float best = 1e30f;
  for (int r = 0; r < 5; r++) {
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(f, dim3(blocks), dim3(256), 0, 0, d, 12345u + r, iters);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  double steps = (double)blocks * 256 * iters * kUnroll * kChains;
  double rate = steps / (best * 1e-3);  // lane-ops per second
  printf("{\"inst\": \"%s\", \"lane_ops_per_s\": %.4e, \"insts_per_step\": %d, \"ms\": %.3f}\n", name, rate,
         insts_per_step, best);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return rate;
}

int main(int argc, char** argv) {
  int dev = 0;
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, dev));
  int blocks = p.multiProcessorCount * 8;
  int iters = argc > 1 ? atoi(argv[1]) : 2000;
  printf("{\"device\": \"%s\", \"cus\": %d, \"clock_khz\": %d, \"blocks\": %d}\n", p.gcnArchName,
         p.multiProcessorCount, p.clockRate, blocks);
  uint64_t* d;
  CHECK(hipMalloc(&d, (size_t)blocks * 256 * sizeof(uint64_t)));
  run("v_mad_u64_u32", k_mad_u64, 1, d, blocks, iters);
  run("v_mad_u64_u32 sgpr-operand", k_mad_u64_sgpr, 1, d, blocks, iters);
  run("v_mad_u64_u32 @4 waves/SIMD", k_mad_u64, 1, d, blocks / 2, iters);
  run("v_mad_u64_u32 @2 waves/SIMD", k_mad_u64, 1, d, blocks / 4, iters);
  run("mad_u64+addc_e64 (comba step)", k_comba, 2, d, blocks, iters);
  run("mad_u64+addc_e32 vcc (comba step)", k_comba_vcc, 2, d, blocks, iters);
  run("v_mul_lo_u32", k_mul_lo, 1, d, blocks, iters);
  run("v_mul_hi_u32", k_mul_hi, 1, d, blocks, iters);
  run("v_mad_u32_u24", k_mad_u24, 1, d, blocks, iters);
  run("v_mul_u32_u24_e32", k_mul_u24_e32, 1, d, blocks, iters);
  run("v_mul_hi_u32_u24_e32", k_mulhi_u24_e32, 1, d, blocks, iters);
  run("v_add_u32_e32", k_add, 1, d, blocks, iters);
  run("v_add_u32_e64", k_add_e64, 1, d, blocks, iters);
  run("v_add3_u32", k_add3, 1, d, blocks, iters);
  run("v_fmac_f32_e32", k_fmac_f32, 1, d, blocks, iters);
  run("v_fma_f32", k_fma_f32, 1, d, blocks, iters);
  run("v_alignbit_b32", k_alignbit, 1, d, blocks, iters);
  run("v_and_or_b32", k_and_or, 1, d, blocks, iters);
  run("v_dot2_u32_u16", k_dot2_u16, 1, d, blocks, iters);
  run("v_fma_f64", k_fma_f64, 1, d, blocks, iters);
  run("v_lshl_add_u64", k_lshl_add_u64, 1, d, blocks, iters);
  run("v_lshrrev_b64", k_lshrrev_b64, 1, d, blocks, iters);
  run("v_ashrrev_i64", k_ashrrev_i64, 1, d, blocks, iters);
  run("v_mad_i64_i32", k_mad_i64, 1, d, blocks, iters);
  run("v_and_b32", k_and, 1, d, blocks, iters);
  run("v_xor_b32", k_xor, 1, d, blocks, iters);
  run("v_lshl_add_u32", k_lshl_add_u32, 1, d, blocks, iters);
  run("v_permlane32_swap_b32", k_permlane32_swap, 1, d, blocks, iters);
  CHECK(hipFree(d));
  return 0;
}
