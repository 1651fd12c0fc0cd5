// Division by a runtime-constant divisor as a multiply-high + shift (host and
// device), for the implicit-GEMM row / tap decompositions in conv_lds.hip.
// n / d == (umulhi(n, m) + n) >> s for 0 <= n < 2^31, with s = ceil(log2 d) and
// m = floor(2^32 (2^s - d) / d) + 1.  Checked exhaustively over divisors and
// edge numerators by tests/native/host_selftest.cpp (host ASan/UBSan build).
#pragma once

#include <cstdint>

#include <hip/hip_runtime.h>

namespace ldnn {
namespace convlds {

struct FastDiv {
  uint32_t m, s;
};

inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  if (d == 0) d = 1;  // an empty parity class: never divided by
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

__host__ __device__ __forceinline__ int fdiv(int n, const FastDiv& f) {
  const uint32_t hi = (uint32_t)(((uint64_t)(uint32_t)n * f.m) >> 32);
  return (int)((hi + (uint32_t)n) >> f.s);
}

}  // namespace convlds
}  // namespace ldnn
