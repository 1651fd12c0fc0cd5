// Memory-bound helpers: activations, bias-gradient column sums, casts, the
// aggregation "mix" kernel and device-side synthetic data.
//
// All bf16 traffic is vectorised to 16 B per lane (Guideline 13); grids are
// capped at 2048 workgroups and grid-stride the rest (Guideline 11).
//
// mix3_f32 is kernel K18 of SURVEY §2.3: every aggregation formula of the
// reference -- BAR/communication.py:9-10,17-18,25,31 (equal / weighted
// all-reduce), BR/communication.py:30,62 (ring), BDR/communication.py:39-40,77
// (double ring) -- is  out = a*x + b*y1 + c*y2  for suitable (a, b, c), done in
// one pass, in place, with the bf16 compute shadow refreshed in the same pass.
#include <algorithm>

#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t work_items) {
  int64_t g = (work_items + kBlock - 1) / kBlock;
  if (g < 1) g = 1;
  if (g > 2048) g = 2048;
  return (int)g;
}

template <int ACT>
__device__ __forceinline__ float act_f(float x) {
  if constexpr (ACT == ACT_RELU) return fmaxf(x, 0.f);
  return 1.f / (1.f + __expf(-x));
}
template <int ACT>
__device__ __forceinline__ float act_b(float dy, float y) {
  if constexpr (ACT == ACT_RELU) return y > 0.f ? dy : 0.f;
  return dy * y * (1.f - y);
}

template <int ACT>
__global__ void act_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
    u16x8 v = reinterpret_cast<const u16x8*>(x)[i];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(act_f<ACT>(bf2f(v[j])));
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
  for (int64_t i = nv * 8 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = f2bf(act_f<ACT>(bf2f(x[i])));
}

template <int ACT>
__global__ void act_bwd_kernel(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ y,
                               bf16_t* __restrict__ dx, int64_t n) {
  const int64_t nv = n / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
    u16x8 g = reinterpret_cast<const u16x8*>(dy)[i];
    u16x8 v = reinterpret_cast<const u16x8*>(y)[i];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(act_b<ACT>(bf2f(g[j]), bf2f(v[j])));
    reinterpret_cast<u16x8*>(dx)[i] = o;
  }
  for (int64_t i = nv * 8 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    dx[i] = f2bf(act_b<ACT>(bf2f(dy[i]), bf2f(y[i])));
}

// Column sums of a [rows][cols] bf16 matrix (bias gradients), optionally fused with an
// activation backward (BWD: dx = act'(y) * dy, the sums taken from the fp32
// derivative before rounding; dy may alias dx).  A block is `lanes` 8-column groups
// (16-B accesses) x `rl` = 256 / lanes row lanes, lanes = min(cols / 8, 32): narrow
// matrices keep every thread busy (a conv bias of 8 channels was 8 active threads
// per block: 44 us for a 200704 x 8 colsum).  Rows split over gridDim.y, two rows
// in flight per lane.  STORE (a single row block, first write): the block stores its
// sums instead of adding them -- no zeroing launch.
struct CsGeo {
  int lanes, rl, gx, gy, rpb;
};
inline CsGeo cs_geo(int rows, int cols) {
  CsGeo g;
  const int cv = cols / 8;
  g.lanes = cv < 32 ? cv : 32;
  g.rl = 256 / g.lanes;
  g.gx = (cv + g.lanes - 1) / g.lanes;
  int gy = std::max(1, 1024 / g.gx);
  gy = std::min(gy, std::max(1, (rows + 16 * g.rl - 1) / (16 * g.rl)));   // >= 16 rows per row lane
  g.rpb = (rows + gy - 1) / gy;
  g.gy = (rows + g.rpb - 1) / g.rpb;
  return g;
}

// acc / ticket (optional, a caller-kept zeroed scratch of cols floats + one int): the row groups
// add into acc instead of out, and the last workgroup to finish moves acc into out (= or +=) and
// leaves acc and the ticket zero -- one launch where a multi-group sum that overwrites out needed a
// zero-fill launch first (LeNet-5's conv bias gradients: 2 of its 30 kernels)
template <int ACT, bool BWD>
__global__ __launch_bounds__(256) void colsum_geo_kernel(const bf16_t* dy, const bf16_t* __restrict__ y, bf16_t* dx,
                                                         float* __restrict__ out, int rows, int cols, int rpb,
                                                         int lanes, int rl, int store, float* __restrict__ acc,
                                                         int* __restrict__ ticket, int accum_out) {
  __shared__ float part[256 * 8];
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid % lanes, ty = tid / lanes;
  const int c0 = (blockIdx.x * lanes + lane) * 8;
  const int r_begin = blockIdx.y * rpb;
  const int r_end = min(rows, r_begin + rpb);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto row = [&](size_t o) {
    const u16x8 g = *reinterpret_cast<const u16x8*>(dy + o);
    if constexpr (BWD) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(y + o);
      u16x8 d;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float a = act_b<ACT>(bf2f(g[j]), bf2f(v[j]));
        s[j] += a;
        d[j] = f2bf(a);
      }
      *reinterpret_cast<u16x8*>(dx + o) = d;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += bf2f(g[j]);
    }
  };
  if (ty < rl && c0 < cols) {
    int r = r_begin + ty;
    for (; r + rl < r_end; r += 2 * rl) {
      row((size_t)r * cols + c0);
      row((size_t)(r + rl) * cols + c0);
    }
    for (; r < r_end; r += rl) row((size_t)r * cols + c0);
  }
  const int w = lanes * 8;
  if (ty < rl) {
#pragma unroll
    for (int j = 0; j < 8; ++j) part[ty * w + lane * 8 + j] = s[j];
  }
  __syncthreads();
  for (int ch = tid; ch < w; ch += 256) {
    const int c = blockIdx.x * w + ch;
    if (c >= cols) continue;
    float t = 0.f;
    for (int q = 0; q < rl; ++q) t += part[q * w + ch];
    if (acc != nullptr) atomicAdd(acc + c, t);
    else if (store) out[c] = t;
    else atomicAdd(out + c, t);
  }
  if (acc == nullptr) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this thread's adds have completed
  __syncthreads();
  if (tid == 0) {
    const int tk = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = tk == (int)(gridDim.x * gridDim.y) - 1;
    if (s_last) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!s_last) return;
  for (int c = tid; c < cols; c += 256) {
    const float v = atomicExch(acc + c, 0.f);
    out[c] = accum_out ? out[c] + v : v;
  }
}

// Zero a [rows][cols] fp32 block with row stride ld.  A kernel, not
// hipMemset2DAsync: memset nodes captured into hipGraphs are not replayed
// reliably on this stack (found while validating graph-captured split-K wgrads).
__global__ void zero2d_kernel(float* __restrict__ p, int rows, int cols, int ld) {
  const int64_t n = (int64_t)rows * cols;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const int r = (int)(i / cols), c = (int)(i % cols);
    p[(size_t)r * ld + c] = 0.f;
  }
}

// out[c][r] = in[r][c] (bf16, rows and cols multiples of 8): 64 x 64 tiles staged in
// LDS, 16-B loads and stores on both sides.
// Logical NCHW (fp32 or bf16, contiguous) -> dense NHWC bf16 with cp >= C channels,
// the pad channels written as zeros: one thread per (pixel, 8-channel group), the
// C strided reads coalesced across neighbouring pixels, one 16-B store.  Replaces a
// zero fill + permute copy (two ATen launches, ~3x the bytes) at every CNN input.
template <typename T>
__global__ __launch_bounds__(256) void nchw_to_nhwc_kernel(const T* __restrict__ src, bf16_t* __restrict__ dst,
                                                           int64_t total, int C, int HW, int groups,
                                                           const uint2* __restrict__ esrc, uint2* __restrict__ edst,
                                                           int64_t e8) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < e8) edst[i] = esrc[i];   // a batch's labels staged in the same launch (8-B pieces)
  if (i >= total) return;
  const int g = (int)(i % groups);
  const int64_t pix = i / groups;
  const int64_t n = pix / HW;
  const int hw = (int)(pix - n * HW);
  const T* s = src + (size_t)n * C * HW + hw;
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int c = g * 8 + j;
    float v = 0.f;
    if (c < C) {
      if constexpr (sizeof(T) == 4) v = (float)s[(size_t)c * HW];
      else v = bf2f(s[(size_t)c * HW]);
    }
    o[j] = f2bf(v);
  }
  reinterpret_cast<u16x8*>(dst)[i] = o;
}

// The same for the usual CNN input (<= 8 channels -> one 8-channel group, H*W % 4 == 0): a thread
// converts 4 consecutive pixels of one image -- per channel one 16-B (fp32) / 8-B (bf16) load
// instead of four 4 / 2-B ones, four 16-B stores in a row, 32-bit index math (the 64-bit divisions
// of the generic kernel are its VALU cost): the ResNet-18 b256 input staging is 282 MB of traffic.
template <typename T>
__global__ __launch_bounds__(256) void nchw_to_nhwc4_kernel(const T* __restrict__ src, bf16_t* __restrict__ dst,
                                                            int npix4, int C, int HW,
                                                            const uint2* __restrict__ esrc, uint2* __restrict__ edst,
                                                            int64_t e8) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < e8) edst[i] = esrc[i];   // a batch's labels staged in the same launch (8-B pieces)
  if (i >= npix4) return;
  const int pix = i * 4;
  const int n = pix / HW;
  const int hw = pix - n * HW;
  const T* s = src + (size_t)n * C * HW + hw;
  u16x8 o[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    if (c >= C) break;
    if constexpr (sizeof(T) == 4) {
      const floatx4 v = *reinterpret_cast<const floatx4*>(s + (size_t)c * HW);
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k][c] = f2bf(v[k]);
    } else {
      const uint2 v = *reinterpret_cast<const uint2*>(s + (size_t)c * HW);
      o[0][c] = (uint16_t)(v.x & 0xffffu);
      o[1][c] = (uint16_t)(v.x >> 16);
      o[2][c] = (uint16_t)(v.y & 0xffffu);
      o[3][c] = (uint16_t)(v.y >> 16);
    }
  }
  u16x8* d = reinterpret_cast<u16x8*>(dst) + pix;
#pragma unroll
  for (int k = 0; k < 4; ++k) d[k] = o[k];
}

// The staging pass of a graph whose first layer is the 7x7 / 2 stem on its space-to-depth image
// (conv_stem.hip): one thread per s2d pixel (n, i, j) reads the 2x2 input block at rows 2(i-2) + dh,
// columns 2(j-2) + dw of each of the C <= 4 channels (one 8-B / 4-B load per channel and row,
// coalesced across j), writes the block's four NHWC pixels (two 32-B runs) when it lies in the image
// and the 32-B s2d pixel xs[(dh*2 + dw)*4 + c] always (zeros outside the image) -- the conv then
// skips its own pack pass, which re-read the whole NHWC image (ResNet-18 b256: 54 us).
template <typename T>
__global__ __launch_bounds__(256) void nchw_to_nhwc_s2d_kernel(const T* __restrict__ src, bf16_t* __restrict__ dst,
                                                               bf16_t* __restrict__ s2d, int npix, int C, int H, int W,
                                                               int Hs, int Ws, const uint2* __restrict__ esrc,
                                                               uint2* __restrict__ edst, int64_t e8) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < e8) edst[i] = esrc[i];   // a batch's labels staged in the same launch (8-B pieces)
  if (i >= npix) return;
  const int jj = i % Ws, t = i / Ws;
  const int ii = t % Hs, n = t / Hs;
  const int h0 = 2 * (ii - 2), w0 = 2 * (jj - 2);
  const bool in = h0 >= 0 && h0 < H && w0 >= 0 && w0 < W;   // (H, W even: the whole 2x2 block)
  u16x8 px[2][2];   // [dh][dw]: 8-channel NHWC pixels (channels >= C zero)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) px[a][b] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
  if (in) {
    const T* s = src + ((size_t)n * C * H + h0) * W + w0;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      if (c >= C) break;
#pragma unroll
      for (int dh = 0; dh < 2; ++dh) {
        const T* r = s + ((size_t)c * H + dh) * W;
        if constexpr (sizeof(T) == 4) {
          const float2 v = *reinterpret_cast<const float2*>(r);
          px[dh][0][c] = f2bf(v.x);
          px[dh][1][c] = f2bf(v.y);
        } else {
          const uint32_t v = *reinterpret_cast<const uint32_t*>(r);
          px[dh][0][c] = (uint16_t)(v & 0xffffu);
          px[dh][1][c] = (uint16_t)(v >> 16);
        }
      }
    }
#pragma unroll
    for (int dh = 0; dh < 2; ++dh) {
      u16x8* d = reinterpret_cast<u16x8*>(dst) + ((size_t)n * H + h0 + dh) * W + w0;
      d[0] = px[dh][0];
      d[1] = px[dh][1];
    }
  }
  u16x8 o[2];   // s2d channel (dh*2 + dw)*4 + c: o[dh][dw*4 + c]
#pragma unroll
  for (int dh = 0; dh < 2; ++dh)
#pragma unroll
    for (int dw = 0; dw < 2; ++dw)
#pragma unroll
      for (int c = 0; c < 4; ++c) o[dh][dw * 4 + c] = px[dh][dw][c];
  u16x8* xs = reinterpret_cast<u16x8*>(s2d) + (size_t)i * 2;
  xs[0] = o[0];
  xs[1] = o[1];
}

// out[c][r] = in[r][c], 64 x 64 tiles.  The tile goes to LDS as whole 128-B rows (16-B chunks
// XOR-swizzled by row, rows 8 apart shifted by 4 more chunks) and comes back COLUMN-wise through
// ds_read_b64_tr_b16 (per 16-lane group: 4 rows x 16 columns, lane i receives column i):
// wave w owns output rows c0 + 16w .. +15 (lane i of each group one of them), group gq the input
// rows 8gq + 32h .. +7 of pass h, so each lane stores 8 consecutive outputs (16 B) per pass --
// no 2-byte LDS accesses and no bank conflicts (the element-wise tile was 12.4 extra LDS cycles
// per instruction, profiles/r5/pmc_mlp3.txt).  Needs a full 256-thread block (EXEC all ones for
// the transposing read: out-of-range rows / columns are loaded as zeros and not stored).
__device__ __forceinline__ int tr_sw(int row) { return (row & 7) ^ (((row >> 3) & 1) << 2); }

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16_t* __restrict__ in, bf16_t* __restrict__ out,
                                                             int rows, int cols, int ldi, int ldo) {
  typedef __attribute__((address_space(3))) bf16x4 lds_b4;
  __shared__ __attribute__((aligned(16))) char t[64 * 128];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const int p = threadIdx.x + it * 256;
    const int r = p >> 3, ch = p & 7;
    u16x8 v = {};
    if (r0 + r < rows && c0 + ch * 8 < cols) v = *reinterpret_cast<const u16x8*>(in + (size_t)(r0 + r) * ldi + c0 + ch * 8);
    *reinterpret_cast<u16x8*>(t + r * 128 + ((ch ^ tr_sw(r)) << 4)) = v;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int gq = lane >> 4, i = lane & 15, q = i >> 2, pp = i & 3;
  const int ch = 2 * w + (pp >> 1);  // the 16-B chunk of columns 16w + 4pp .. +3
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rb = 32 * h + 8 * gq;  // input rows rb .. rb + 7 -> this lane's 8 outputs
    bf16x4 lo, hi;
    {
      const int r = rb + q;
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4*)(t + r * 128 + ((ch ^ tr_sw(r)) << 4) + (pp & 1) * 8));
    }
    {
      const int r = rb + 4 + q;
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4*)(t + r * 128 + ((ch ^ tr_sw(r)) << 4) + (pp & 1) * 8));
    }
    const int c = c0 + 16 * w + i;
    if (c < cols && r0 + rb < rows) {
      const bf16x8 o = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      *reinterpret_cast<bf16x8*>(out + (size_t)c * ldo + r0 + rb) = o;
    }
  }
}

// split-K slabs ws[s][r][0 .. ldw) -> out[r][0 .. ncols) (row stride ldo) and, when
// extra != nullptr, extra[r] = column ncols (a GEMM whose B operand carries a ones
// column: the bias gradient comes out of the weight-gradient GEMM)
__global__ __launch_bounds__(256) void slab_sum_cols_kernel(const float* __restrict__ ws, int splits, int rows, int ldw,
                                                            float* __restrict__ out, int ldo, int ncols,
                                                            float* __restrict__ extra) {
  const int g4 = (ncols + 4) / 4;  // float4 groups per row, incl. the one holding column ncols
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)rows * g4) return;
  const int r = (int)(i / g4), c = (int)(i % g4) * 4;
  const size_t slab = (size_t)rows * ldw;
  const floatx4* w = reinterpret_cast<const floatx4*>(ws + (size_t)r * ldw + c);
  floatx4 v = w[0];
  for (int sp = 1; sp < splits; ++sp) v += *reinterpret_cast<const floatx4*>(ws + sp * slab + (size_t)r * ldw + c);
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (c + q < ncols) out[(size_t)r * ldo + c + q] = v[q];
    else if (c + q == ncols && extra != nullptr) extra[r] = v[q];
  }
}

__global__ void cast_f32_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, int64_t n) {
  const int64_t nv = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
    const floatx4 v = reinterpret_cast<const floatx4*>(x)[i];
    reinterpret_cast<u16x4*>(y)[i] = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
  }
  for (int64_t i = nv * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) y[i] = f2bf(x[i]);
}

__global__ void cast_bf16_f32_kernel(const bf16_t* __restrict__ x, float* __restrict__ y, int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) y[i] = bf2f(x[i]);
}

template <int NIN>
__global__ void mix_kernel(float* out, const float* x, const float* y1, const float* y2, float a, float b,
                           float c, int64_t n, bf16_t* shadow) {
  const int64_t nv = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
    floatx4 v = a * reinterpret_cast<const floatx4*>(x)[i];
    if constexpr (NIN >= 2) v += b * reinterpret_cast<const floatx4*>(y1)[i];
    if constexpr (NIN >= 3) v += c * reinterpret_cast<const floatx4*>(y2)[i];
    reinterpret_cast<floatx4*>(out)[i] = v;
    if (shadow) reinterpret_cast<u16x4*>(shadow)[i] = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
  }
  for (int64_t i = nv * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = a * x[i];
    if constexpr (NIN >= 2) v += b * y1[i];
    if constexpr (NIN >= 3) v += c * y2[i];
    out[i] = v;
    if (shadow) shadow[i] = f2bf(v);
  }
}

// The same with bf16 neighbour inputs (per-step gossip with a bf16 exchange: the own fp32
// gradient x mixed with the bf16 copies received from the ring neighbours).
template <int NIN>
__global__ void mix_y16_kernel(float* out, const float* x, const uint16_t* y1, const uint16_t* y2, float a, float b,
                               float c, int64_t n, bf16_t* shadow) {
  const int64_t nv = n / 4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nv; i += stride) {
    floatx4 v = a * reinterpret_cast<const floatx4*>(x)[i];
    const u16x4 u1 = reinterpret_cast<const u16x4*>(y1)[i];
    v += b * floatx4{bf2f(u1[0]), bf2f(u1[1]), bf2f(u1[2]), bf2f(u1[3])};
    if constexpr (NIN >= 3) {
      const u16x4 u2 = reinterpret_cast<const u16x4*>(y2)[i];
      v += c * floatx4{bf2f(u2[0]), bf2f(u2[1]), bf2f(u2[2]), bf2f(u2[3])};
    }
    reinterpret_cast<floatx4*>(out)[i] = v;
    if (shadow) reinterpret_cast<u16x4*>(shadow)[i] = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
  }
  for (int64_t i = nv * 4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    float v = a * x[i] + b * bf2f(y1[i]);
    if constexpr (NIN >= 3) v += c * bf2f(y2[i]);
    out[i] = v;
    if (shadow) shadow[i] = f2bf(v);
  }
}

// splitmix64 counter hash -> two uniforms -> Box-Muller normal.
__device__ __forceinline__ uint64_t smix(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void synth_normal_kernel(bf16_t* x, int64_t n, uint64_t seed, float stddev) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t h = smix(seed * 0x100000001B3ull + (uint64_t)i);
    const float u1 = ((h >> 40) + 1) * (1.0f / 16777217.0f);
    const float u2 = ((h & 0xFFFFFF)) * (1.0f / 16777216.0f);
    const float z = sqrtf(-2.f * __logf(u1)) * __cosf(6.2831853f * u2);
    x[i] = f2bf(z * stddev);
  }
}

__global__ void synth_labels_kernel(int64_t* y, int64_t n, int classes, uint64_t seed) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
    y[i] = (int64_t)(smix(seed * 0x9E3779B1ull + (uint64_t)i) % (uint64_t)classes);
}

}  // namespace

hipError_t act_fwd(const uint16_t* x, uint16_t* y, int64_t n, int act, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int g = grid_for((n + 7) / 8);
  if (act == ACT_RELU) act_fwd_kernel<ACT_RELU><<<g, kBlock, 0, s>>>(x, y, n);
  else act_fwd_kernel<ACT_SIGMOID><<<g, kBlock, 0, s>>>(x, y, n);
  return hipGetLastError();
}

hipError_t act_bwd(const uint16_t* dy, const uint16_t* y, uint16_t* dx, int64_t n, int act, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int g = grid_for((n + 7) / 8);
  if (act == ACT_RELU) act_bwd_kernel<ACT_RELU><<<g, kBlock, 0, s>>>(dy, y, dx, n);
  else act_bwd_kernel<ACT_SIGMOID><<<g, kBlock, 0, s>>>(dy, y, dx, n);
  return hipGetLastError();
}

hipError_t nchw_to_nhwc(const void* src, bool src_f32, uint16_t* dst, int N, int C, int HW, int cp, hipStream_t s,
                        const void* extra_src, void* extra_dst, int64_t extra_bytes) {
  if (N <= 0 || HW <= 0) return hipSuccess;
  if (cp % 8 || cp < C || C <= 0) return hipErrorInvalidValue;
  if (extra_bytes % 8 || ((uintptr_t)extra_src & 7) || ((uintptr_t)extra_dst & 7)) return hipErrorInvalidValue;
  const int groups = cp / 8;
  const int64_t total = (int64_t)N * HW * groups;
  const int64_t e8 = extra_bytes / 8;
  const unsigned g = (unsigned)((std::max(total, e8) + 255) / 256);
  const uint2* es = static_cast<const uint2*>(extra_src);
  uint2* ed = static_cast<uint2*>(extra_dst);
  if (groups == 1 && HW % 4 == 0 && (int64_t)N * HW < (int64_t)1 << 30 && ((uintptr_t)src & 15) == 0) {
    const int npix4 = N * HW / 4;
    const unsigned g4 = (unsigned)((std::max((int64_t)npix4, e8) + 255) / 256);
    if (src_f32)
      nchw_to_nhwc4_kernel<float><<<g4, 256, 0, s>>>(static_cast<const float*>(src), dst, npix4, C, HW, es, ed, e8);
    else
      nchw_to_nhwc4_kernel<bf16_t><<<g4, 256, 0, s>>>(static_cast<const bf16_t*>(src), dst, npix4, C, HW, es, ed, e8);
    return hipGetLastError();
  }
  if (src_f32)
    nchw_to_nhwc_kernel<float><<<g, 256, 0, s>>>(static_cast<const float*>(src), dst, total, C, HW, groups, es, ed, e8);
  else
    nchw_to_nhwc_kernel<bf16_t><<<g, 256, 0, s>>>(static_cast<const bf16_t*>(src), dst, total, C, HW, groups, es, ed, e8);
  return hipGetLastError();
}

hipError_t nchw_to_nhwc_s2d(const void* src, bool src_f32, uint16_t* dst, uint16_t* s2d, int N, int C, int H, int W,
                            hipStream_t s, const void* extra_src, void* extra_dst, int64_t extra_bytes) {
  if (N <= 0) return hipSuccess;
  if (C <= 0 || C > 4 || H % 2 || W % 2 || H <= 0 || W <= 0) return hipErrorInvalidValue;
  if (extra_bytes % 8 || ((uintptr_t)extra_src & 7) || ((uintptr_t)extra_dst & 7)) return hipErrorInvalidValue;
  const int Hs = H / 2 + 3, Ws = W / 2 + 3;
  if ((int64_t)N * Hs * Ws >= (int64_t)1 << 30 || (int64_t)N * C * H * W >= (int64_t)1 << 40) return hipErrorInvalidValue;
  const int npix = N * Hs * Ws;
  const int64_t e8 = extra_bytes / 8;
  const unsigned g = (unsigned)((std::max((int64_t)npix, e8) + 255) / 256);
  const uint2* es = static_cast<const uint2*>(extra_src);
  uint2* ed = static_cast<uint2*>(extra_dst);
  bf16_t* d = reinterpret_cast<bf16_t*>(dst);
  bf16_t* x2 = reinterpret_cast<bf16_t*>(s2d);
  if (src_f32)
    nchw_to_nhwc_s2d_kernel<float><<<g, 256, 0, s>>>(static_cast<const float*>(src), d, x2, npix, C, H, W, Hs, Ws, es,
                                                      ed, e8);
  else
    nchw_to_nhwc_s2d_kernel<bf16_t><<<g, 256, 0, s>>>(static_cast<const bf16_t*>(src), d, x2, npix, C, H, W, Hs, Ws,
                                                       es, ed, e8);
  return hipGetLastError();
}

hipError_t transpose_bf16(const uint16_t* in, uint16_t* out, int rows, int cols, int ldi, int ldo, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (rows % 8 || cols % 8 || ldi % 8 || ldo % 8) return hipErrorInvalidValue;
  transpose_bf16_kernel<<<dim3((cols + 63) / 64, (rows + 63) / 64), 256, 0, s>>>(in, out, rows, cols, ldi, ldo);
  return hipGetLastError();
}

hipError_t slab_sum_cols(const float* ws, int splits, int rows, int ldw, float* out, int ldo, int ncols, float* extra,
                         hipStream_t s) {
  if (rows <= 0 || ncols <= 0) return hipSuccess;
  if (ldw % 4 || ncols + (extra ? 1 : 0) > ldw || ((ncols + 4) / 4) * 4 > ldw) return hipErrorInvalidValue;
  const int64_t n = (int64_t)rows * ((ncols + 4) / 4);
  slab_sum_cols_kernel<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(ws, splits, rows, ldw, out, ldo, ncols, extra);
  return hipGetLastError();
}

hipError_t zero2d_f32(float* p, int rows, int cols, int ld, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  zero2d_kernel<<<grid_for((int64_t)rows * cols), kBlock, 0, s>>>(p, rows, cols, ld);
  return hipGetLastError();
}

hipError_t colsum_bf16(const uint16_t* x, float* out, int rows, int cols, bool accumulate, hipStream_t s, float* ws) {
  if (cols <= 0) return hipSuccess;
  if (cols % 8) return hipErrorInvalidValue;
  const CsGeo g = cs_geo(std::max(rows, 1), cols);
  const bool store = !accumulate && g.gy == 1;
  const bool self = ws != nullptr && !accumulate && !store;   // (one launch: the ticketed scratch)
  if (!accumulate && !store && !self) {
    hipError_t e = zero2d_f32(out, 1, cols, cols, s);
    if (e != hipSuccess) return e;
  }
  colsum_geo_kernel<ACT_RELU, false><<<dim3(g.gx, g.gy), kBlock, 0, s>>>(
      x, nullptr, nullptr, out, rows, cols, g.rpb, g.lanes, g.rl, store ? 1 : 0, self ? ws : nullptr,
      self ? reinterpret_cast<int*>(ws + cols) : nullptr, 0);
  return hipGetLastError();
}

hipError_t act_bwd_colsum(const uint16_t* dy, const uint16_t* y, uint16_t* dx, float* out, int rows, int cols,
                          int act, bool accumulate, hipStream_t s, float* ws) {
  if (cols <= 0) return hipSuccess;
  if (cols % 8) return hipErrorInvalidValue;
  const CsGeo g = cs_geo(std::max(rows, 1), cols);
  const bool store = !accumulate && g.gy == 1;
  const bool self = ws != nullptr && !accumulate && !store;
  if (!accumulate && !store && !self) {
    hipError_t e = zero2d_f32(out, 1, cols, cols, s);
    if (e != hipSuccess) return e;
  }
  const dim3 grid(g.gx, g.gy);
  float* acc = self ? ws : nullptr;
  int* tk = self ? reinterpret_cast<int*>(ws + cols) : nullptr;
  if (act == ACT_RELU)
    colsum_geo_kernel<ACT_RELU, true><<<grid, kBlock, 0, s>>>(dy, y, dx, out, rows, cols, g.rpb, g.lanes, g.rl,
                                                              store ? 1 : 0, acc, tk, 0);
  else
    colsum_geo_kernel<ACT_SIGMOID, true><<<grid, kBlock, 0, s>>>(dy, y, dx, out, rows, cols, g.rpb, g.lanes, g.rl,
                                                                 store ? 1 : 0, acc, tk, 0);
  return hipGetLastError();
}

hipError_t cast_f32_bf16(const float* x, uint16_t* y, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  cast_f32_bf16_kernel<<<grid_for((n + 3) / 4), kBlock, 0, s>>>(x, y, n);
  return hipGetLastError();
}

hipError_t cast_bf16_f32(const uint16_t* x, float* y, int64_t n, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  cast_bf16_f32_kernel<<<grid_for(n), kBlock, 0, s>>>(x, y, n);
  return hipGetLastError();
}

hipError_t mix3_f32(float* out, const float* x, const float* y1, const float* y2, float a, float b, float c,
                    int64_t n, uint16_t* shadow, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  const int g = grid_for((n + 3) / 4);
  if (y2) mix_kernel<3><<<g, kBlock, 0, s>>>(out, x, y1, y2, a, b, c, n, shadow);
  else if (y1) mix_kernel<2><<<g, kBlock, 0, s>>>(out, x, y1, y2, a, b, c, n, shadow);
  else mix_kernel<1><<<g, kBlock, 0, s>>>(out, x, y1, y2, a, b, c, n, shadow);
  return hipGetLastError();
}

hipError_t mix3_y16(float* out, const float* x, const uint16_t* y1, const uint16_t* y2, float a, float b, float c,
                    int64_t n, uint16_t* shadow, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (!y1) return hipErrorInvalidValue;
  const int g = grid_for((n + 3) / 4);
  if (y2) mix_y16_kernel<3><<<g, kBlock, 0, s>>>(out, x, y1, y2, a, b, c, n, shadow);
  else mix_y16_kernel<2><<<g, kBlock, 0, s>>>(out, x, y1, y2, a, b, c, n, shadow);
  return hipGetLastError();
}

hipError_t scale_f32(float* x, float scale, int64_t n, uint16_t* shadow, hipStream_t s) {
  return mix3_f32(x, x, nullptr, nullptr, scale, 0.f, 0.f, n, shadow, s);
}

hipError_t synth_normal_bf16(uint16_t* x, int64_t n, uint64_t seed, float stddev, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  synth_normal_kernel<<<grid_for(n), kBlock, 0, s>>>(x, n, seed, stddev);
  return hipGetLastError();
}

hipError_t synth_labels(int64_t* y, int64_t n, int classes, uint64_t seed, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  synth_labels_kernel<<<grid_for(n), kBlock, 0, s>>>(y, n, classes, seed);
  return hipGetLastError();
}

// Communication stand-in for overlap probes (parallel/overlap_probe.py): a copy of a
// gradient bucket on a FEW workgroups, repeated `reps` times -- the footprint of an
// RCCL ring all-reduce (a handful of channels, each one workgroup, link-paced),
// not of a chip-wide HBM copy that would take every CU from the backward.
__global__ __launch_bounds__(kBlock) void standin_copy_kernel(const floatx4* __restrict__ src,
                                                              floatx4* __restrict__ dst, int64_t n4, int reps) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int r = 0; r < reps; ++r) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) dst[i] = src[i];
    __syncthreads();
  }
}

hipError_t standin_copy(const float* src, float* dst, int64_t n, int blocks, int reps, hipStream_t s) {
  if (n <= 0 || reps <= 0) return hipSuccess;
  if (n % 4 != 0 || blocks < 1) return hipErrorInvalidValue;
  standin_copy_kernel<<<blocks, kBlock, 0, s>>>(reinterpret_cast<const floatx4*>(src), reinterpret_cast<floatx4*>(dst),
                                                n / 4, reps);
  return hipGetLastError();
}

}  // namespace ldnn
