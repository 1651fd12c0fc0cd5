// Common device helpers for the ldnn gfx950 (CDNA4) kernels.
//
// Every kernel in csrc/kernels/ is written for gfx950 only: wave64, MFMA bf16
// matrix cores, 160 KiB LDS per CU, 8 XCDs.  No CUDA shims, no dual paths.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ldnn {

typedef uint16_t bf16_t;  // raw bf16 bits as stored in HBM

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef uint16_t u16x4 __attribute__((ext_vector_type(4)));
typedef uint16_t u16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int kWave = 64;  // CDNA wavefront width (never 32)
constexpr int kNumXcd = 8;

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

// Plain cast lowers to v_cvt_pk_bf16_f32 (RNE, keeps NaN a NaN).
__device__ __forceinline__ uint16_t f2bf(float f) { return __builtin_bit_cast(uint16_t, (__bf16)f); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Bijective XCD-aware remap of a 1-D workgroup id: workgroups b and b+8 share
// an XCD (round-robin dispatch), so give each XCD a contiguous run of logical
// tiles.  Pure speed choice: any placement is still correct.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int q = nwg / kNumXcd, r = nwg % kNumXcd;
  const int xcd = bid % kNumXcd, idx = bid / kNumXcd;
  const int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

}  // namespace ldnn
