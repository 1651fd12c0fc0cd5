// Host-side self test of the native planning code, built with AddressSanitizer and
// UndefinedBehaviorSanitizer on the HOST half of hipcc's compile (the device code is
// built normally and never launched; no GPU is touched).  SURVEY §5 "race detection /
// sanitizers": this covers the C++ that sizes grids, split-K slices and workspaces --
// the code whose integer overflow or off-by-one would become an out-of-bounds kernel.
//
//   scripts/host_sanitize.sh   (driven by tests/test_native_host_sanitized.py)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ldnn_fastdiv.h"
#include "ldnn_kernels.h"

static int g_fail = 0;
#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++g_fail;                                                               \
    }                                                                         \
  } while (0)

static void fastdiv() {
  using namespace ldnn::convlds;
  std::vector<uint32_t> ns = {0u, 1u, 2u, 3u, 63u, 64u, 65u, 4095u, 4096u, 65535u, 65536u, 1000003u,
                              (1u << 24) + 1, (1u << 30) - 1, 1u << 30, 2147483646u, 2147483647u};
  uint64_t x = 88172645463325252ull;
  for (int i = 0; i < 2000; ++i) {  // xorshift: numerators over the whole int range
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    ns.push_back((uint32_t)(x & 0x7fffffffu));
  }
  for (uint32_t d = 1; d <= 4096; ++d) {
    const FastDiv f = make_fastdiv(d);
    for (uint32_t n : ns) CHECK(fdiv((int)n, f) == (int)(n / d));
    for (uint32_t k = 1; k < 64; ++k) {  // around every small multiple of d
      const uint64_t m = (uint64_t)k * d;
      if (m + 1 < (1u << 31)) {
        CHECK(fdiv((int)(m - 1), f) == (int)((m - 1) / d));
        CHECK(fdiv((int)m, f) == (int)(m / d));
        CHECK(fdiv((int)(m + 1), f) == (int)((m + 1) / d));
      }
    }
  }
  for (uint32_t d : {50176u, 200704u, 802816u, 1u << 20, (1u << 31) - 1}) {  // big row counts
    const FastDiv f = make_fastdiv(d);
    for (uint32_t n : ns) CHECK(fdiv((int)n, f) == (int)(n / d));
  }
}

static void conv_plans() {
  int shapes = 0;
  for (int N : {1, 3, 64, 256})
    for (int H : {1, 2, 4, 7, 14, 32, 56, 112})
      for (int C : {8, 16, 32, 64, 128, 512, 1024})
        for (int K : {64, 128, 256, 1024})
          for (int R : {1, 3, 5, 7})
            for (int st : {1, 2}) {
              const int pad = R / 2;
              ldnn::ConvShape s{};
              s.N = N; s.H = H; s.W = H; s.C = C; s.K = K; s.R = R; s.S = R; s.stride = st; s.pad = pad;
              s.P = (H + 2 * pad - R) / st + 1;
              s.Q = s.P;
              if (s.P <= 0) continue;
              for (int op = 0; op < 3; ++op) {
                const ldnn::ConvWorkspace w = ldnn::conv2d_lds_workspace(s, op);
                if (w.counters > 0) {  // in-launch combine: one 64 KiB slab per (tile, slice)
                  CHECK(w.slab_bytes > 0 && w.slab_bytes % 65536 == 0);
                  CHECK(w.slab_bytes / 65536 >= (size_t)2 * w.counters);
                }
                if (op == 2 && w.slab_bytes > 0)  // wgrad partial slabs: whole [K][RSC] fp32 copies
                  CHECK(w.slab_bytes % ((size_t)K * R * R * C * 4) == 0);
                if (op < 2 && w.slab_bytes > 0 && w.counters == 0) {  // small-M slab split-K: whole outputs
                  const size_t out = op == 0 ? (size_t)N * s.P * s.Q * K * 4 : (size_t)N * H * H * C * 4;
                  CHECK(w.slab_bytes % out == 0 && w.slab_bytes / out >= 2 && w.slab_bytes / out <= 32);
                  CHECK(op == 0 || st == 1);  // stride-2 dgrad classes keep the in-launch combine
                }
              }
              ++shapes;
            }
  std::printf("conv plans: %d shapes\n", shapes);
}

static void small_kernels() {
  for (int B : {1, 16, 17, 255, 4096, 65536})
    for (int K : {8, 64, 784, 4096, 8192}) {
      const int sp = ldnn::head_wgrad_splits(B, K);
      CHECK(sp >= 1 && sp <= 64);
      CHECK(ldnn::head_dgrad_ws_floats(B, K) == (size_t)((B + 15) / 16) * K);
    }
  for (int C : {8, 64, 1024, 4096}) CHECK(ldnn::bn_workspace_floats(C) >= 4 * C);
}

int main() {
  fastdiv();
  conv_plans();
  small_kernels();
  if (g_fail) {
    std::fprintf(stderr, "host selftest: %d failures\n", g_fail);
    return 1;
  }
  std::printf("HOST_SELFTEST_OK\n");
  return 0;
}
