// mem_dev.h — the two places a grant's bytes are read from by the byte-level
// device code (proto_dev.h, sha256_dev.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mochi {

typedef uint32_t mem_v4u __attribute__((ext_vector_type(4)));

// Where the bytes are: HBM (generic 64-bit addresses) or a copy staged in LDS
// (32-bit LDS addresses: ds_read instead of a gathered global load per lane,
// k_grant_prep).  A staged copy keeps each byte's offset within its dword.
// (the explicit global address space: global_load, not flat_load, from an
// address that went through an integer)
struct GlobalMem {
  using addr_t = uintptr_t;
  static __device__ __forceinline__ uint32_t ld32(addr_t a) {
    return *(const __attribute__((address_space(1))) uint32_t*)a;
  }
  static __device__ __forceinline__ mem_v4u ld128(addr_t a) {
    return *(const __attribute__((address_space(1))) mem_v4u*)a;
  }
};
struct LdsMem {
  using addr_t = uint32_t;
  static __device__ __forceinline__ uint32_t ld32(addr_t a) {
    return *(const __attribute__((address_space(3))) uint32_t*)(size_t)a;
  }
  static __device__ __forceinline__ mem_v4u ld128(addr_t a) {
    return *(const __attribute__((address_space(3))) mem_v4u*)(size_t)a;
  }
};

}  // namespace mochi
