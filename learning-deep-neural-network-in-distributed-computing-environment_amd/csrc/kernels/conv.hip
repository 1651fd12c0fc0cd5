// Implicit-GEMM 2-D convolution for gfx950: forward,
// backward-data (dgrad) and backward-weight (wgrad) as bf16 MFMA GEMMs whose
// operand tiles are GATHERED from NHWC activations while they are staged into
// LDS -- no im2col buffer is ever materialised.
//
// Layouts (channels innermost, padded to a multiple of 8 so every gather is a
// 16-byte vector of 8 channels):
//   x  [N][H][W][C]      activations (NHWC, bf16)
//   w  [K][R][S][C]      weights (KRSC, the bf16 shadow of the fp32 master)
//   y  [N][P][Q][K]      outputs (NHWC)
//
// GEMM views (M x Ngemm, reduction Kd):
//   fwd   y [NPQ][K]   = A(m=npq, k=rsc) . B(k=rsc, n=k_out)   A gathered from x (zero padding = zeros),
//                                                            B = w as a [K][RSC] k-contiguous matrix
//   dgrad dx[NHW][C]   = A(m=nhw, k=rsk) . B(k=rsk, n=c)      A gathered from dy: p = (h+pad-r)/stride
//                                                            when divisible (zero-insertion form of the
//                                                            transposed conv, handles stride 2 exactly),
//                                                            B gathered from w rows (k,r,s)
//   wgrad dw[K][RSC]   = A(m=k_out, k=npq) . B(k=npq, n=rsc)  A = dy as a [NPQ][K] matrix (k-strided),
//                                                            B gathered from x; fp32 out, split-K over NPQ
//
// The main loop is the 128x128x64 register-staged MFMA tile of gemm.hip (same
// LDS images, fragment reads and fused epilogue), with the global address of
// each 16-byte chunk produced by a per-operand gather policy.  This generic
// kernel serves the shapes outside the LDS-DMA fast path of conv_lds.hip
// (stems with C < 64, 5x5 LeNet convs, K % 64 != 0 dgrads); the dispatchers
// below try the fast path first.
#include "ldnn_common.h"
#include "ldnn_gemm_tile.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

struct ConvArgs {
  ConvShape s;
  const bf16_t* x;
  const bf16_t* w;
  const bf16_t* dy;
  void* out;
  const float* bias;
  int M, N, Kd;  // GEMM view
  int ldc;
  float beta;
};

// ---- gather policies: at(a, row, k) -> address of 8 consecutive elements, or null (= zeros)
// KC policies: the 8 elements run along the reduction dim k (fixed GEMM row).
// Strided policies: the 8 elements run along the GEMM row dim (fixed k).

struct FwdA {  // x gathered, row = output pixel npq, k = (r, s, c)
  static constexpr bool KC = true;
  __device__ static const bf16_t* at(const ConvArgs& a, int m, int k) {
    const ConvShape& s = a.s;
    const int q = m % s.Q, t = m / s.Q, p = t % s.P, n = t / s.P;
    const int c = k % s.C, rs = k / s.C, r = rs / s.S, sx = rs % s.S;
    const int ih = p * s.stride - s.pad + r, iw = q * s.stride - s.pad + sx;
    if (ih < 0 || ih >= s.H || iw < 0 || iw >= s.W) return nullptr;
    return a.x + (((size_t)n * s.H + ih) * s.W + iw) * s.C + c;
  }
};

struct FwdB {  // weights [K][RSC]
  static constexpr bool KC = true;
  __device__ static const bf16_t* at(const ConvArgs& a, int n, int k) {
    return a.w + (size_t)n * a.Kd + k;
  }
};

struct DgradA {  // dy gathered, row = input pixel nhw, k = (r, s, kout)
  static constexpr bool KC = true;
  __device__ static const bf16_t* at(const ConvArgs& a, int m, int k) {
    const ConvShape& s = a.s;
    const int wq = m % s.W, t = m / s.W, h = t % s.H, n = t / s.H;
    const int ko = k % s.K, rs = k / s.K, r = rs / s.S, sx = rs % s.S;
    const int ph = h + s.pad - r, pw = wq + s.pad - sx;
    if (ph < 0 || pw < 0) return nullptr;
    if (s.stride > 1 && ((ph % s.stride) || (pw % s.stride))) return nullptr;
    const int p = ph / s.stride, q = pw / s.stride;
    if (p >= s.P || q >= s.Q) return nullptr;
    return a.dy + (((size_t)n * s.P + p) * s.Q + q) * s.K + ko;
  }
};

struct DgradB {  // weights: k = (r, s, kout) row, 8 consecutive input channels
  static constexpr bool KC = false;
  __device__ static const bf16_t* at(const ConvArgs& a, int c, int k) {
    const ConvShape& s = a.s;
    const int ko = k % s.K, rs = k / s.K, r = rs / s.S, sx = rs % s.S;
    return a.w + (((size_t)ko * s.R + r) * s.S + sx) * s.C + c;
  }
};

struct WgradA {  // dy as [NPQ][K]: k = npq, 8 consecutive output channels
  static constexpr bool KC = false;
  __device__ static const bf16_t* at(const ConvArgs& a, int m, int k) { return a.dy + (size_t)k * a.s.K + m; }
};

struct WgradB {  // x gathered: k = npq, 8 consecutive j = (r, s, c..c+7)
  static constexpr bool KC = false;
  __device__ static const bf16_t* at(const ConvArgs& a, int j, int k) {
    const ConvShape& s = a.s;
    const int q = k % s.Q, t = k / s.Q, p = t % s.P, n = t / s.P;
    const int c = j % s.C, rs = j / s.C, r = rs / s.S, sx = rs % s.S;
    const int ih = p * s.stride - s.pad + r, iw = q * s.stride - s.pad + sx;
    if (ih < 0 || ih >= s.H || iw < 0 || iw >= s.W) return nullptr;
    return a.x + (((size_t)n * s.H + ih) * s.W + iw) * s.C + c;
  }
};

constexpr int BM = 128, BN = 128;
constexpr int kThreads = 256;
constexpr int kTileBytes = 128 * BK * 2;

template <class OP>
__device__ __forceinline__ void load_tile(u32x4 (&r)[4], const ConvArgs& a, int rows, int r0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + kThreads * i;
    int row, k;
    if constexpr (OP::KC) {
      k = (c & 7) * 8;
      row = c >> 3;
    } else {
      const int half = c & 1, klo = (c >> 1) & 3, rb = (c >> 3) & 7, khi = c >> 6;
      k = khi * 4 + klo;
      row = rb * 16 + half * 8;
    }
    const int gr = r0 + row, gk = k0 + k;
    const bf16_t* ptr = (gr < rows && gk < a.Kd) ? OP::at(a, gr, gk) : nullptr;
    r[i] = ptr ? *reinterpret_cast<const u32x4*>(ptr) : u32x4{0u, 0u, 0u, 0u};
  }
}

template <bool KC>
__device__ __forceinline__ void store_tile(const u32x4 (&r)[4], char* lds, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + kThreads * i;
    int row, k;
    if constexpr (KC) {
      k = (c & 7) * 8;
      row = c >> 3;
    } else {
      const int half = c & 1, klo = (c >> 1) & 3, rb = (c >> 3) & 7, khi = c >> 6;
      k = khi * 4 + klo;
      row = rb * 16 + half * 8;
    }
    *reinterpret_cast<u32x4*>(lds + lds_offset<KC, 128>(row, k)) = r[i];
  }
}

template <class OA, class OB, int EPI, bool OUT_F32>
__global__ __launch_bounds__(kThreads, 2) void conv_gemm_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[4 * kTileBytes];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int m0, n0;
  tile_coords(a.M, a.N, BM, BN, m0, n0);

  floatx4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk_all = (a.Kd + BK - 1) / BK;
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
  const int kbase = kt0 * BK;
  u32x4 ra[4], rb[4];
  load_tile<OA>(ra, a, a.M, m0, kbase, tid);
  load_tile<OB>(rb, a, a.N, n0, kbase, tid);
  store_tile<OA::KC>(ra, smem, tid);
  store_tile<OB::KC>(rb, smem + kTileBytes, tid);
  __syncthreads();
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = (kt + 1) < nk;
    if (more) {
      load_tile<OA>(ra, a, a.M, m0, kbase + (kt + 1) * BK, tid);
      load_tile<OB>(rb, a, a.N, n0, kbase + (kt + 1) * BK, tid);
    }
    const char* la = smem + cur * 2 * kTileBytes;
    const char* lb = la + kTileBytes;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag<OA::KC, 128>(la, wm * 4 + i, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag<OB::KC, 128>(lb, wn * 4 + j, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[j][i], 0, 0, 0);
    }
    if (more) {
      char* nb = smem + (cur ^ 1) * 2 * kTileBytes;
      store_tile<OA::KC>(ra, nb, tid);
      store_tile<OB::KC>(rb, nb + kTileBytes, tid);
    }
    __syncthreads();
  }
  if constexpr (OUT_F32 && EPI == EPI_NONE) {
    if (gridDim.y > 1) {  // split-K partial sums
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int m = m0 + wm * 64 + i * 16 + (lane & 15);
          if (n < a.N && m < a.M) {
            float* c = reinterpret_cast<float*>(a.out) + (size_t)m * a.ldc + n;
#pragma unroll
            for (int r = 0; r < 4; ++r) atomicAdd(c + r, acc[j][i][r]);
          }
        }
      }
      return;
    }
  }
  GemmParams p{};
  p.C = a.out;
  p.M = a.M;
  p.N = a.N;
  p.ldc = a.ldc;
  p.bias = a.bias;
  p.beta = a.beta;
  epilogue<EPI, OUT_F32, 4, 4>(p, acc, m0 + wm * 64, n0 + wn * 64, lane);
}

inline int splitk_for(int tiles, int Kd) {
  if (tiles >= 128) return 1;
  int sk = (512 + tiles - 1) / tiles;
  const int max_by_k = Kd / 512;
  if (sk > max_by_k) sk = max_by_k;
  return sk < 2 ? 1 : (sk > 64 ? 64 : sk);
}

// Small-channel dgrad (C == 8: the padded input channels of LeNet's second conv or a small
// stem's; K * R * S * 8 <= kDgradC8MaxW): the MFMA kernels compute a 128-wide output tile
// for these 8 columns (LeNet-5 b256 conv2 dgrad: 27 us for 0.3 GFLOP).  Here one thread
// computes the 8 channels of one input pixel on the VALU from the taps' dy vectors, with
// the [K][R][S][8] weights staged once per workgroup in LDS as fp32 (every lane of a wave
// reads the same address: LDS broadcasts): 22 us.  (Measured alternatives, all slower:
// 4 pixels per thread 48 us and 4 channels per thread 29 us -- the loop is load-latency
// bound -- and the weights through scalar loads as SGPR operands 35 us.)
// The forward of the same small convs (C == 8 padded input channels, K <= 16 filters, 3x3 / 5x5
// stride 1: LeNet-5's two convs) on the MFMA pipe: MFMA A = w (16 rows = filters, one 16-B row of
// 8 channels per lane per tap: the fragments are plain loads, held for the launch), B = a 16-pixel
// tile's input patch, one 16-B gather per lane per 4-tap k-step (a tap in the padding reads
// nothing: zero).  A lane ends with 4 consecutive filters of one pixel: bias (+ ReLU), 8-B store.
template <int KS, int SS, int EPI>
__global__ __launch_bounds__(256) void conv_fwd_c8_mfma_kernel(ConvShape s, const bf16_t* __restrict__ x,
                                                               const bf16_t* __restrict__ w,
                                                               const float* __restrict__ bias, bf16_t* __restrict__ y,
                                                               int tiles) {
  constexpr int RS = SS * SS;
  static_assert(4 * KS >= RS, "k-steps");
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  bf16x8 fa[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int tap = 4 * k + g;
    u16x8 v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (tap < RS && l16 < s.K) v = *reinterpret_cast<const u16x8*>(w + ((size_t)l16 * RS + tap) * 8);
    fa[k] = __builtin_bit_cast(bf16x8, v);
  }
  float bv[4] = {0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI != EPI_NONE) {
#pragma unroll
    for (int v = 0; v < 4; ++v) bv[v] = 4 * g + v < s.K ? bias[4 * g + v] : 0.f;
  }
  const int npix = s.N * s.P * s.Q;   // (the dispatcher checks it fits 31 bits)
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < tiles; t += gridDim.x * 4) {
    const int pix = t * 16 + l16;
    const bool pv = pix < npix;
    const int tt = pv ? pix / s.Q : 0;
    const int q = pv ? pix - tt * s.Q : 0;
    const int n = tt / s.P, p = tt - n * s.P;
    const bf16_t* xn = x + (size_t)n * s.H * s.W * 8;
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int tap = 4 * k + g;
      const int r = tap / SS, sx = tap - r * SS;   // (compile-time divisor)
      const int ih = p - s.pad + r, iw = q - s.pad + sx;
      const bool ok = pv && tap < RS && ih >= 0 && iw >= 0 && ih < s.H && iw < s.W;
      u16x8 b = {0, 0, 0, 0, 0, 0, 0, 0};
      if (ok) b = *reinterpret_cast<const u16x8*>(xn + ((size_t)ih * s.W + iw) * 8);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[k], __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
    }
    if (pv && 4 * g < s.K) {
      u16x4 o;
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        float z = acc[v] + bv[v];
        if constexpr (EPI == EPI_BIAS_RELU) z = fmaxf(z, 0.f);
        o[v] = f2bf(z);
      }
      *reinterpret_cast<u16x4*>(y + (size_t)pix * s.K + 4 * g) = o;
    }
  }
}

constexpr int kDgradC8MaxW = 8192;

// K == 16 (LeNet-5's second conv: 6 -> 16 channels, 5x5) on the MFMA pipe instead:
// dx[pixel][c] = sum_{tap, k} dy[the tap's output pixel][k] w[k][tap][c] with MFMA A = w^T
// (16 rows = channels, 8 of them real, held in registers for the launch: one fragment per
// 32-deep k-step = 2 taps x 16 filters) and B = a 16-pixel tile's dy fragments, one 16-B
// gather per lane per k-step (a tap outside the output reads nothing: zero).  A lane ends with
// 4 consecutive channels of one pixel: 8-B stores, 256 contiguous bytes per tile.  One wave per
// tile.
template <int KS, int SS, bool ST1>   // SS = R = S (5 / 3); ST1: stride 1 (no tap divisibility tests)
__global__ __launch_bounds__(256) void conv_dgrad_c8k16_kernel(ConvShape s, const bf16_t* __restrict__ dy,
                                                               const bf16_t* __restrict__ w, bf16_t* __restrict__ dx,
                                                               int tiles) {
  __shared__ __attribute__((aligned(16))) uint16_t wl[16 * 2 * KS * 8];   // w [16][RS][8] (16-B staged)
  const int lane = threadIdx.x & 63, g = lane >> 4, l16 = lane & 15;
  constexpr int RS = SS * SS;
  static_assert(2 * KS >= RS, "k-steps");
  for (int i = threadIdx.x; i < 16 * RS; i += 256)   // (scattered 2-B global gathers per lane were the cost)
    reinterpret_cast<u16x8*>(wl)[i] = reinterpret_cast<const u16x8*>(w)[i];
  __syncthreads();
  bf16x8 fa[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int tap = 2 * k + (g >> 1);
    u16x8 v;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int kf = (g & 1) * 8 + e;
      v[e] = (l16 < 8 && tap < RS) ? wl[(kf * RS + tap) * 8 + l16] : (uint16_t)0;
    }
    fa[k] = __builtin_bit_cast(bf16x8, v);
  }
  const int npix = s.N * s.H * s.W;   // (the dispatcher checks it fits 31 bits)
  for (int t = blockIdx.x * 4 + (threadIdx.x >> 6); t < tiles; t += gridDim.x * 4) {
  const int pix = t * 16 + l16;
  const bool pv = pix < npix;
  const int tt = pv ? pix / s.W : 0;
  const int wq = pv ? pix - tt * s.W : 0;
  const int n = tt / s.H, h = tt - n * s.H;
  const bf16_t* dyn = dy + (size_t)n * s.P * s.Q * 16 + (g & 1) * 8;
  floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int tap = 2 * k + (g >> 1);
    const int r = tap / SS, sx = tap - r * SS;   // (compile-time divisor)
    const int ph = h + s.pad - r, qw = wq + s.pad - sx;
    int p, q;
    bool ok;
    if constexpr (ST1) {
      p = ph;
      q = qw;
      ok = pv && tap < RS && ph >= 0 && qw >= 0 && p < s.P && q < s.Q;
    } else {
      p = ph / s.stride;
      q = qw / s.stride;
      ok = pv && tap < RS && ph >= 0 && qw >= 0 && ph == p * s.stride && qw == q * s.stride && p < s.P && q < s.Q;
    }
    u16x8 b = {0, 0, 0, 0, 0, 0, 0, 0};
    if (ok) b = *reinterpret_cast<const u16x8*>(dyn + ((size_t)p * s.Q + q) * 16);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[k], __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
  if (g < 2 && pv)
    *reinterpret_cast<u16x4*>(dx + pix * 8 + 4 * g) = u16x4{f2bf(acc[0]), f2bf(acc[1]), f2bf(acc[2]), f2bf(acc[3])};
  }
}
constexpr int kDgradC8Threads = 64;

__global__ __launch_bounds__(kDgradC8Threads) void conv_dgrad_c8_kernel(ConvShape s, const bf16_t* __restrict__ dy,
                                                                        const bf16_t* __restrict__ w,
                                                                        bf16_t* __restrict__ dx) {
  __shared__ __attribute__((aligned(16))) float wl[kDgradC8MaxW];
  const int RS = s.R * s.S, nw = s.K * RS * 8;
  // (16-B weight loads: the 2-B ones left each workgroup's staging a chain of ~50 loads per lane)
  for (int i = threadIdx.x; i < nw / 8; i += kDgradC8Threads) {
    const u16x8 v = reinterpret_cast<const u16x8*>(w)[i];
    reinterpret_cast<floatx4*>(wl)[2 * i] = floatx4{bf2f(v[0]), bf2f(v[1]), bf2f(v[2]), bf2f(v[3])};
    reinterpret_cast<floatx4*>(wl)[2 * i + 1] = floatx4{bf2f(v[4]), bf2f(v[5]), bf2f(v[6]), bf2f(v[7])};
  }
  __syncthreads();
  const int64_t pix = (int64_t)blockIdx.x * kDgradC8Threads + threadIdx.x;
  if (pix >= (int64_t)s.N * s.H * s.W) return;
  const int wq = (int)(pix % s.W);
  const int64_t t = pix / s.W;
  const int h = (int)(t % s.H), n = (int)(t / s.H);
  floatx4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
  for (int r = 0; r < s.R; ++r) {
    const int ph = h + s.pad - r;
    if (ph < 0 || ph % s.stride) continue;
    const int p = ph / s.stride;
    if (p >= s.P) continue;
    for (int sx = 0; sx < s.S; ++sx) {
      const int qw = wq + s.pad - sx;
      if (qw < 0 || qw % s.stride) continue;
      const int q = qw / s.stride;
      if (q >= s.Q) continue;
      const bf16_t* g = dy + (((size_t)n * s.P + p) * s.Q + q) * s.K;
      const float* wr = wl + (r * s.S + sx) * 8;
      for (int k8 = 0; k8 < s.K; k8 += 8) {
        const u16x8 gv = *reinterpret_cast<const u16x8*>(g + k8);
#pragma unroll
        for (int kk = 0; kk < 8; ++kk) {
          const float gk = bf2f(gv[kk]);
          const float* wk = wr + (size_t)(k8 + kk) * RS * 8;
          a0 += gk * *reinterpret_cast<const floatx4*>(wk);
          a1 += gk * *reinterpret_cast<const floatx4*>(wk + 4);
        }
      }
    }
  }
  u16x8 o;
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    o[c] = f2bf(a0[c]);
    o[c + 4] = f2bf(a1[c]);
  }
  *reinterpret_cast<u16x8*>(dx + pix * 8) = o;
}

}  // namespace

namespace {
int g_conv_impl = 0;  // 0: LDS-DMA fast path where it applies, 1: generic kernel only
}  // namespace

void set_conv_impl(int impl) { g_conv_impl = impl; }
int get_conv_impl() { return g_conv_impl; }

hipError_t conv2d_fwd(const ConvShape& s, const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                      int epi, hipStream_t st, float* ws, int* cnt, const BnFin* bn, bool* bn_done,
                      uint16_t* s2d_xs) {
  if (bn_done) *bn_done = false;
  if (s2d_xs != nullptr && g_conv_impl != 0) return hipErrorInvalidValue;
  if (g_conv_impl == 0 && s2d_xs == nullptr && bn == nullptr && s.C == 8 && (s.K == 8 || s.K == 16) &&
      s.stride == 1 && s.R == s.S && (s.R == 5 || s.R == 3) && (epi == EPI_NONE || bias != nullptr) &&
      (epi == EPI_NONE || epi == EPI_BIAS || epi == EPI_BIAS_RELU) && (int64_t)s.N * s.P * s.Q + 16 < (1ll << 31)) {
    // the small-channel convs (LeNet-5) on the MFMA kernel above
    const int64_t npix = (int64_t)s.N * s.P * s.Q;
    if (npix <= 0) return hipSuccess;
    const int tiles = (int)((npix + 15) / 16);
    const unsigned blocks = (unsigned)std::min((tiles + 3) / 4, 1024);
    const bf16_t* x16 = reinterpret_cast<const bf16_t*>(x);
    const bf16_t* w16 = reinterpret_cast<const bf16_t*>(w);
    bf16_t* y16 = reinterpret_cast<bf16_t*>(y);
#define C8F_CASE(KS_, SS_)                                                                                     \
  switch (epi) {                                                                                               \
    case EPI_NONE: conv_fwd_c8_mfma_kernel<KS_, SS_, EPI_NONE><<<blocks, 256, 0, st>>>(s, x16, w16, bias, y16, tiles); break;      \
    case EPI_BIAS: conv_fwd_c8_mfma_kernel<KS_, SS_, EPI_BIAS><<<blocks, 256, 0, st>>>(s, x16, w16, bias, y16, tiles); break;      \
    default: conv_fwd_c8_mfma_kernel<KS_, SS_, EPI_BIAS_RELU><<<blocks, 256, 0, st>>>(s, x16, w16, bias, y16, tiles); break;       \
  }
    if (s.R == 5) {
      C8F_CASE(7, 5)
    } else {
      C8F_CASE(3, 3)
    }
#undef C8F_CASE
    return hipGetLastError();
  }
  if (g_conv_impl == 0) {
    bool used = false;
    const hipError_t e = conv2d_fwd_lds(s, x, w, y, bias, epi, st, ws, cnt, bn, &used, s2d_xs);
    if (e != hipErrorNotSupported) {
      if (bn_done) *bn_done = used && e == hipSuccess;
      return e;
    }
  }
  ConvArgs a{};
  a.s = s;
  a.x = x;
  a.w = w;
  a.out = y;
  a.bias = bias;
  a.M = s.N * s.P * s.Q;
  a.N = s.K;
  a.Kd = s.R * s.S * s.C;
  a.ldc = s.K;
  if (a.M <= 0) return hipSuccess;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles), block(kThreads);
  switch (epi) {
    case EPI_NONE: conv_gemm_kernel<FwdA, FwdB, EPI_NONE, false><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS: conv_gemm_kernel<FwdA, FwdB, EPI_BIAS, false><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_RELU: conv_gemm_kernel<FwdA, FwdB, EPI_BIAS_RELU, false><<<grid, block, 0, st>>>(a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t conv2d_fwd2(const ConvShape& s0, const uint16_t* x, const uint16_t* w0, uint16_t* y0, float* ws0,
                       int* cnt0, const BnFin* bn0, bool* done0, const ConvShape& s1, const uint16_t* w1,
                       uint16_t* y1, float* ws1, int* cnt1, const BnFin* bn1, bool* done1, hipStream_t st) {
  if (g_conv_impl == 0) {
    const hipError_t e = conv2d_fwd2_lds(s0, x, w0, y0, ws0, cnt0, bn0, done0, s1, w1, y1, ws1, cnt1, bn1, done1, st);
    if (e != hipErrorNotSupported) return e;
  }
  const hipError_t e = conv2d_fwd(s0, x, w0, y0, nullptr, EPI_NONE, st, ws0, cnt0, bn0, done0);
  if (e != hipSuccess) return e;
  return conv2d_fwd(s1, x, w1, y1, nullptr, EPI_NONE, st, ws1, cnt1, bn1, done1);
}

hipError_t conv2d_bwd2(const BwdJob& j0, const BwdJob& j1, const uint16_t* x, hipStream_t st) {
  if (g_conv_impl == 0) {
    const hipError_t e = conv2d_bwd2_lds(j0, j1, x, st);
    if (e != hipErrorNotSupported) return e;
  }
  for (const BwdJob* j : {&j0, &j1}) {
    const hipError_t e = conv2d_bwd(j->sd, j->dy, j->w, j->dx, j->ws_d, j->cnt_d, nullptr, nullptr, j->sw, x, j->dw,
                                    j->beta, j->ws_w, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t conv2d_bwd(const ConvShape& sd, const uint16_t* dy, const uint16_t* w, uint16_t* dx, float* ws_d,
                      int* cnt_d, const BnBwdFuse* bnb, bool* bn_done, const ConvShape& sw, const uint16_t* x,
                      float* dw, float beta, float* ws_w, hipStream_t st) {
  if (bn_done) *bn_done = false;
  if (g_conv_impl == 0) {
    const hipError_t e = conv2d_bwd_lds(sd, dy, w, dx, ws_d, cnt_d, bnb, bn_done, sw, x, dw, beta, ws_w, st);
    if (e != hipErrorNotSupported) return e;
  }
  const hipError_t e = conv2d_dgrad(sd, dy, w, dx, st, ws_d, cnt_d, bnb, bn_done);
  if (e != hipSuccess) return e;
  return conv2d_wgrad(sw, dy, x, dw, beta, st, ws_w);
}

hipError_t conv2d_dgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                        float* ws, int* cnt, const BnBwdFuse* bnb, bool* bn_done) {
  if (bn_done) *bn_done = false;
  if (g_conv_impl == 0) {
    const hipError_t e = conv2d_dgrad_lds(s, dy, w, dx, st, ws, cnt, bnb, bn_done);
    if (e != hipErrorNotSupported) return e;
    if (bn_done) *bn_done = false;
  }
  if (g_conv_impl == 0 && s.C == 8 && s.K == 16 && s.stride >= 1 && s.R == s.S && (s.R == 5 || s.R == 3) &&
      (int64_t)s.N * s.H * s.W + 16 < (1ll << 31)) {
    const int64_t pix = (int64_t)s.N * s.H * s.W;
    if (pix <= 0) return hipSuccess;
    const int tiles = (int)((pix + 15) / 16);
    const unsigned blocks = (unsigned)std::min((tiles + 3) / 4, 512);   // (a few tiles per wave: w staged once)
    const bf16_t* dy16 = reinterpret_cast<const bf16_t*>(dy);
    const bf16_t* w16 = reinterpret_cast<const bf16_t*>(w);
    bf16_t* dx16 = reinterpret_cast<bf16_t*>(dx);
    const bool st1 = s.stride == 1;
    if (s.R == 5 && st1) conv_dgrad_c8k16_kernel<13, 5, true><<<blocks, 256, 0, st>>>(s, dy16, w16, dx16, tiles);
    else if (s.R == 5) conv_dgrad_c8k16_kernel<13, 5, false><<<blocks, 256, 0, st>>>(s, dy16, w16, dx16, tiles);
    else if (st1) conv_dgrad_c8k16_kernel<5, 3, true><<<blocks, 256, 0, st>>>(s, dy16, w16, dx16, tiles);
    else conv_dgrad_c8k16_kernel<5, 3, false><<<blocks, 256, 0, st>>>(s, dy16, w16, dx16, tiles);
    return hipGetLastError();
  }
  if (g_conv_impl == 0 && s.C == 8 && s.K % 8 == 0 && s.K * s.R * s.S * 8 <= kDgradC8MaxW && s.stride >= 1) {
    const int64_t pix = (int64_t)s.N * s.H * s.W;
    if (pix <= 0) return hipSuccess;
    conv_dgrad_c8_kernel<<<(unsigned)((pix + kDgradC8Threads - 1) / kDgradC8Threads), kDgradC8Threads, 0, st>>>(
        s, reinterpret_cast<const bf16_t*>(dy), reinterpret_cast<const bf16_t*>(w), reinterpret_cast<bf16_t*>(dx));
    return hipGetLastError();
  }
  ConvArgs a{};
  a.s = s;
  a.dy = dy;
  a.w = w;
  a.out = dx;
  a.M = s.N * s.H * s.W;
  a.N = s.C;
  a.Kd = s.R * s.S * s.K;
  a.ldc = s.C;
  if (a.M <= 0) return hipSuccess;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  conv_gemm_kernel<DgradA, DgradB, EPI_NONE, false><<<dim3(tiles), dim3(kThreads), 0, st>>>(a);
  return hipGetLastError();
}

hipError_t conv2d_wgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* x, float* dw, float beta,
                        hipStream_t st, float* ws, const uint16_t* s2d_xs) {
  if (s2d_xs != nullptr && g_conv_impl != 0) return hipErrorInvalidValue;
  if (g_conv_impl == 0) {
    const hipError_t e = conv2d_wgrad_lds(s, dy, x, dw, beta, st, ws, s2d_xs);
    if (e != hipErrorNotSupported) return e;
  }
  ConvArgs a{};
  a.s = s;
  a.dy = dy;
  a.x = x;
  a.out = dw;
  a.M = s.K;
  a.N = s.R * s.S * s.C;
  a.Kd = s.N * s.P * s.Q;
  a.ldc = a.N;
  a.beta = beta;
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int sk = splitk_for(tiles, a.Kd);
  if (sk > 1) {
    if (beta == 0.f) {
      hipError_t e = zero2d_f32(dw, a.M, a.N, a.ldc, st);
      if (e != hipSuccess) return e;
    } else if (beta != 1.f) {
      return hipErrorInvalidValue;
    }
  }
  conv_gemm_kernel<WgradA, WgradB, EPI_NONE, true><<<dim3(tiles, sk), dim3(kThreads), 0, st>>>(a);
  return hipGetLastError();
}

}  // namespace ldnn
