// BatchNorm (train / eval), fused BN + residual-add + ReLU, and pooling on NHWC
// bf16 activations (BAR/model.py BatchNorm2d, the
// `out += shortcut(x)` / F.relu of ResBlock.forward, AdaptiveAvgPool2d, and the
// BASELINE LeNet / ResNet-18 pools).
//
// With channels innermost, every per-channel reduction is a column sum over an
// [M = N*H*W][C] matrix (geometry at bn_reduce_kernel).  Statistics are fp32
// throughout; the normalise / affine / residual / ReLU pass and the backward
// dx = A g + B x + D pass are single vectorised sweeps in which every thread
// owns a fixed group of 8 channels.  Launches per BN: forward 2 (reduce with
// the finalize fused into its last block, apply), backward 2 (reduce + fused
// coefficients / dgamma / dbeta, apply).  Backward coefficients:
// dx = A g + B x + D, A = gamma*invstd, B = -gamma*invstd^2 * sum(g xhat)/M,
// D = -gamma*invstd*sum(g)/M - B*mean.
#include <algorithm>
#include <cstdlib>

#include "ldnn_common.h"
#include "ldnn_fastdiv.h"
#include "ldnn_kernels.h"
#include "ldnn_bn_fin.h"

namespace ldnn {

using convlds::FastDiv;   // (ldnn_fastdiv.h: multiply-shift division by a launch constant)
using convlds::fdiv;
using convlds::make_fastdiv;

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

// ---- per-channel column reductions over [M][C] ------------------------------
// Geometry: a 256-thread block covers up to 2048 channels as `lanes` 16-B column
// vectors x `rl` row lanes (lanes = min(C/8, 256), rl = 256 / lanes), so every
// thread keeps ONE fixed group of 8 channels -- all lanes busy at C = 64, the
// per-channel constants loaded once -- and a wave reads whole contiguous row
// runs.  Rows split over gridDim.y; the row loop is unrolled 4 deep so each
// thread has 4 independent 16-B loads per tensor in flight.  Block partials are
// reduced in LDS and added with one fp32 atomic per channel per block into an
// accumulator that the finalize kernel consumes and clears (no zeroing launch).
//   forward:  acc[c] += sum x,          acc[C + c] += sum x^2
//   backward: acc[c] += sum g,          acc[C + c] += sum g * xhat,  g = dy * relu'(y)
struct RedGeo {
  int lanes, rl, gx, gy, rpb;
};

// reduce geometry: total blocks and rows per row lane of the reduce kernels; 512 x 8 measured
// best with 8 accumulator copies (profiles/cnn_bn_reduce_r2.jsonl)
constexpr int kBnRedBlocks = 512, kBnRedRows = 8;
// rows per row lane of the apply passes: 1 = the most blocks, one row per thread -- measured on
// MI355X (profiles/r3/bn_apply_rows_ab_r3.jsonl, alternated) EnhancedCNN b64 2.145 -> 2.076 ms vs 8
// rows, ResNet-18 b64 / b256 unchanged
constexpr int kBnApplyRows = 1;

// accumulator copies the reduce blocks spread over (copies only pay when many blocks contend for
// the same addresses: below 64 blocks one copy)
int bn_ncop(bool, int nblk) { return nblk < 64 ? 1 : kBnCopies; }

RedGeo red_geo(int M, int C, bool reduce = false) {
  RedGeo g;
  const int cv = C / 8;
  g.lanes = cv < 256 ? cv : 256;
  g.rl = 256 / g.lanes;
  g.gx = (cv + 255) / 256;
  int gy = std::max(1, (reduce ? kBnRedBlocks : 1024) / g.gx);   // ~4 blocks per CU in total
  const int min_rows = (reduce ? kBnRedRows : kBnApplyRows) * g.rl;  // >= 8 rows per row lane
  gy = std::min(gy, std::max(1, (M + min_rows - 1) / min_rows));
  g.rpb = (M + gy - 1) / gy;
  g.gy = (M + g.rpb - 1) / g.rpb;
  return g;
}

// RELU: g = dy * relu'(y); MASK: relu'(y) from the forward's bit mask (mask + o / 8)
// dy2 (nullable, wave-uniform): a second gradient of the same output, added to dy
template <bool BWD, bool RELU, bool MASK = false>
__device__ __forceinline__ void red_row(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                        const bf16_t* __restrict__ y, size_t o, const float (&mu)[8],
                                        const float (&is)[8], float (&s0)[8], float (&s1)[8],
                                        const uint8_t* __restrict__ mask = nullptr,
                                        const bf16_t* __restrict__ dy2 = nullptr, float w = 1.f) {
  const u16x8 xv = *reinterpret_cast<const u16x8*>(x + o);
  if constexpr (BWD) {
    const u16x8 gv = *reinterpret_cast<const u16x8*>(dy + o);
    u16x8 g2v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (dy2) g2v = *reinterpret_cast<const u16x8*>(dy2 + o);
    u16x8 yv;
    uint32_t mb = 0;
    if constexpr (RELU && MASK) mb = mask[o >> 3];
    else if constexpr (RELU) yv = *reinterpret_cast<const u16x8*>(y + o);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = (bf2f(gv[j]) + bf2f(g2v[j])) * w;
      if constexpr (RELU && MASK) g = ((mb >> j) & 1u) ? g : 0.f;
      else if constexpr (RELU) g = bf2f(yv[j]) > 0.f ? g : 0.f;
      s0[j] += g;
      s1[j] += g * (bf2f(xv[j]) - mu[j]) * is[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = bf2f(xv[j]) * w;
      s0[j] += v;
      s1[j] += v * v;
    }
  }
}

template <bool BWD, bool RELU, bool MASK = false>
__global__ __launch_bounds__(256) void bn_reduce_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                        const bf16_t* __restrict__ y, const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, float* __restrict__ acc,
                                                        int M, int C, int rpb, int lanes, int rl, BnFin fin,
                                                        const uint8_t* __restrict__ mask, int ncop,
                                                        const bf16_t* __restrict__ dy2 = nullptr) {
  // partials channel-major: element j of thread tid at red[k][j * (256 + lanes) + tid] --
  // conflict-free stores (consecutive threads, consecutive words) and, with the
  // (256 + lanes) stride, conflict-free per-channel reads for every lanes value
  // (the thread-major [tid][8] image was an 8-way bank conflict on every store)
  __shared__ float red[2][8 * 512];
  const int tid = threadIdx.x, lane = tid % lanes, rlane = tid / lanes;
  const int cv0 = blockIdx.x * 256 + lane;
  const int c0 = cv0 * 8;
  const bool active = rlane < rl && c0 < C;
  float s0[8], s1[8], mu[8], is[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s0[j] = 0.f;
    s1[j] = 0.f;
    mu[j] = 0.f;
    is[j] = 0.f;
  }
  if (active) {
    if constexpr (BWD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mu[j] = mean[c0 + j];
        is[j] = invstd[c0 + j];
      }
    }
    const int r_end = min(M, (int)(blockIdx.y + 1) * rpb);
    int r = blockIdx.y * rpb + rlane;
    for (; r + 3 * rl < r_end; r += 4 * rl) {
#pragma unroll
      for (int u = 0; u < 4; ++u)
        red_row<BWD, RELU, MASK>(x, dy, y, (size_t)(r + u * rl) * C + c0, mu, is, s0, s1, mask, dy2);
    }
    for (; r < r_end; r += rl) red_row<BWD, RELU, MASK>(x, dy, y, (size_t)r * C + c0, mu, is, s0, s1, mask, dy2);
  }
  const int row = lanes * 8, js = 256 + lanes;
  if (rlane < rl) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][j * js + tid] = s0[j];
      red[1][j * js + tid] = s1[j];
    }
  }
  __syncthreads();
  for (int idx = tid; idx < row; idx += 256) {
    const int j = idx / lanes, ln = idx - j * lanes;   // channel ln * 8 + j of this block
    float t0 = 0.f, t1 = 0.f;
    for (int q = 0; q < rl; ++q) {
      t0 += red[0][j * js + q * lanes + ln];
      t1 += red[1][j * js + q * lanes + ln];
    }
    const int c = blockIdx.x * 2048 + ln * 8 + j;
    float* accc = acc + (size_t)((blockIdx.x + gridDim.x * blockIdx.y) % ncop) * 2 * C;
    if (c < C) {
      bn_acc_add(accc + c, t0);
      bn_acc_add(accc + C + c, t1);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics have completed
  bn_finalize_last<BWD, kBnCopies>(fin, M, C, gridDim.x * gridDim.y, &red[0][0], 2 * 8 * 512, ncop);
}

// Small-M statistics (the 4x4 / 2x2 stages of EnhancedCNN at batch 64: M = 1024 / 256 rows):
// the reduce above is a chain of dependent round trips there -- block partials, fp32 atomics,
// a ticket, then the last block's exchange-and-finalize -- ~11-15 us for a 0.5-2 MB tensor
// (profiles/r5/pmc_enhanced_cnn_b64_mem.txt).  Here ONE workgroup per 64-channel group reads
// every row of its channels (8 row-parallel loads in flight per thread) and finalizes them
// itself: no accumulator, no atomics, no ticket.
//
// Mid-size M (EnhancedCNN 8x8 / 16x16, ResNet-18 7x7 / 14x14 at b64): the same workgroups split
// the rows too (grid.y = row groups, `rpb` rows each).  Each publishes its 64 channels' partial
// sums to `part` ([grid.y][2][C]); the LAST of a column's grid.y workgroups (per-column ticket)
// sums them and finalizes those 64 channels -- a short chain per column, all columns in parallel,
// instead of the big reduce's fp32 atomics + one block exchanging every channel's copies.
template <bool BWD, bool RELU, bool MASK = false>
__global__ __launch_bounds__(256) void bn_reduce_small_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                                              const bf16_t* __restrict__ y, const float* __restrict__ mean,
                                                              const float* __restrict__ invstd, int M, int C, BnFin fin,
                                                              const uint8_t* __restrict__ mask,
                                                              const bf16_t* __restrict__ dy2, float* __restrict__ part,
                                                              int* __restrict__ tickets, int rpb) {
  constexpr int kLanes = 8, kRl = 32, kJs = 256 + kLanes;
  __shared__ float red[2][8 * kJs];
  const int tid = threadIdx.x, lane = tid % kLanes, rlane = tid / kLanes;
  const int c0 = blockIdx.x * 64 + lane * 8;
  const bool active = c0 < C;
  float s0[8], s1[8], mu[8], is[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s0[j] = 0.f;
    s1[j] = 0.f;
    mu[j] = 0.f;
    is[j] = 0.f;
  }
  if (active) {
    if constexpr (BWD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mu[j] = mean[c0 + j];
        is[j] = invstd[c0 + j];
      }
    }
    // batches of 8 rows per lane, all loads in flight together; a short batch re-reads the
    // group's last row with weight 0 instead of a one-row-per-round-trip tail loop
    const int r_end = min(M, (int)(blockIdx.y + 1) * rpb);
    for (int r = blockIdx.y * rpb + rlane; r < r_end; r += 8 * kRl) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int rr = r + u * kRl;
        red_row<BWD, RELU, MASK>(x, dy, y, (size_t)min(rr, r_end - 1) * C + c0, mu, is, s0, s1, mask, dy2,
                                 rr < r_end ? 1.f : 0.f);
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][j * kJs + tid] = s0[j];
    red[1][j * kJs + tid] = s1[j];
  }
  __syncthreads();
  if (tid < 64) {
    const int j = tid / kLanes, ln = tid - j * kLanes;   // channel ln * 8 + j of this group
    float t0 = 0.f, t1 = 0.f;
#pragma unroll 8
    for (int q = 0; q < kRl; ++q) {
      t0 += red[0][j * kJs + q * kLanes + ln];
      t1 += red[1][j * kJs + q * kLanes + ln];
    }
    const int c = blockIdx.x * 64 + ln * 8 + j;
    if (gridDim.y == 1) {
      if (c < C) bn_finalize_channel<BWD>(fin, M, C, c, t0, t1, 1.f / (float)M);
    } else if (c < C) {
      grp_store(part + (size_t)blockIdx.y * 2 * C + c, t0);
      grp_store(part + ((size_t)blockIdx.y * 2 + 1) * C + c, t1);
    }
  }
  if (!BWD && blockIdx.x == 0 && blockIdx.y == 0 && tid == 0 && fin.num_batches) fin.num_batches[0] += 1;
  if (gridDim.y == 1) return;
  __shared__ int last;
  if (!grp_ticket(tickets + blockIdx.x, gridDim.y, last)) return;
  float* tot = &red[0][0];
  const int cc = blockIdx.x * 64 + (tid & 63);
  grp_sum(part, C, cc, 0, gridDim.y, tot);
  grp_sum(part, C, cc, 1, gridDim.y, tot);
  __syncthreads();
  if (tid < 64 && cc < C) {
    const float S0 = tot[tid] + tot[64 + tid] + tot[128 + tid] + tot[192 + tid];
    const float S1 = tot[256 + tid] + tot[320 + tid] + tot[384 + tid] + tot[448 + tid];
    bn_finalize_channel<BWD>(fin, M, C, cc, S0, S1, 1.f / (float)M);
  }
}

__global__ void bn_eval_coeff_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                     const float* __restrict__ rm, const float* __restrict__ rv,
                                     float* __restrict__ scale, float* __restrict__ shift, int C, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - rm[c] * g * is;
}

__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
  const floatx4 a = *reinterpret_cast<const floatx4*>(p), b = *reinterpret_cast<const floatx4*>(p + 4);
  v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
  v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
}

// y = relu?( x * scale[c] + shift[c] (+ res) ) -- same fixed-channel geometry
// RA: the residual is itself a BatchNorm's INPUT (the pre-BN shortcut conv output):
// y = relu?( x * scale + shift + res * scale2 + shift2 ) -- the shortcut BN's output is never stored
template <bool RES, bool RELU, bool MASK = false, bool RA = false>
__global__ __launch_bounds__(256) void bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                                       const float* __restrict__ scale,
                                                       const float* __restrict__ shift, bf16_t* __restrict__ y,
                                                       int M, int C, int rpb, int lanes, int rl,
                                                       uint8_t* __restrict__ mask = nullptr,
                                                       const float* __restrict__ scale2 = nullptr,
                                                       const float* __restrict__ shift2 = nullptr) {
  const int tid = threadIdx.x, lane = tid % lanes, rlane = tid / lanes;
  const int c0 = (blockIdx.x * 256 + lane) * 8;
  if (rlane >= rl || c0 >= C) return;
  float sc[8], sh[8], sc2[8], sh2[8];
  load8(scale + c0, sc);
  load8(shift + c0, sh);
  if constexpr (RA) {
    load8(scale2 + c0, sc2);
    load8(shift2 + c0, sh2);
#pragma unroll
    for (int j = 0; j < 8; ++j) sh[j] += sh2[j];
  }
  const int r_end = min(M, (int)(blockIdx.y + 1) * rpb);
#pragma unroll 4
  for (int r = blockIdx.y * rpb + rlane; r < r_end; r += rl) {
    const size_t o = (size_t)r * C + c0;
    const u16x8 xv = *reinterpret_cast<const u16x8*>(x + o);
    u16x8 rv;
    if constexpr (RES) rv = *reinterpret_cast<const u16x8*>(res + o);
    u16x8 out;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = bf2f(xv[j]) * sc[j] + sh[j];
      if constexpr (RA) v += bf2f(rv[j]) * sc2[j];
      else if constexpr (RES) v += bf2f(rv[j]);
      if constexpr (RELU) v = fmaxf(v, 0.f);
      out[j] = f2bf(v);
    }
    *reinterpret_cast<u16x8*>(y + o) = out;
    if constexpr (RELU && MASK) {
      uint32_t mb = 0;
#pragma unroll
      for (int j = 0; j < 8; ++j) mb |= (bf2f(out[j]) > 0.f ? 1u : 0u) << j;
      mask[o >> 3] = (uint8_t)mb;
    }
  }
}

// dx = A g + B x + D, g = dy * relu'(y); dres = g (the residual branch's gradient)
template <bool RELU, bool MASK = false>
__global__ __launch_bounds__(256) void bn_bwd_apply_kernel(const bf16_t* __restrict__ x,
                                                           const bf16_t* __restrict__ dy,
                                                           const bf16_t* __restrict__ y,
                                                           const float* __restrict__ coef, bf16_t* __restrict__ dx,
                                                           bf16_t* __restrict__ dres, int M, int C, int rpb,
                                                           int lanes, int rl, const uint8_t* __restrict__ mask = nullptr,
                                                           const bf16_t* __restrict__ dy2 = nullptr) {
  const int tid = threadIdx.x, lane = tid % lanes, rlane = tid / lanes;
  const int c0 = (blockIdx.x * 256 + lane) * 8;
  if (rlane >= rl || c0 >= C) return;
  float A[8], B[8], D[8];
  load8(coef + c0, A);
  load8(coef + C + c0, B);
  load8(coef + 2 * C + c0, D);
  const int r_end = min(M, (int)(blockIdx.y + 1) * rpb);
#pragma unroll 4
  for (int r = blockIdx.y * rpb + rlane; r < r_end; r += rl) {
    const size_t o = (size_t)r * C + c0;
    const u16x8 xv = *reinterpret_cast<const u16x8*>(x + o);
    const u16x8 gv = *reinterpret_cast<const u16x8*>(dy + o);
    u16x8 g2v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (dy2) g2v = *reinterpret_cast<const u16x8*>(dy2 + o);
    u16x8 yv;
    uint32_t mb = 0;
    if constexpr (RELU && MASK) mb = mask[o >> 3];
    else if constexpr (RELU) yv = *reinterpret_cast<const u16x8*>(y + o);
    u16x8 out, og;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = bf2f(gv[j]) + bf2f(g2v[j]);
      if constexpr (RELU && MASK) g = ((mb >> j) & 1u) ? g : 0.f;
      else if constexpr (RELU) g = bf2f(yv[j]) > 0.f ? g : 0.f;
      out[j] = f2bf(A[j] * g + B[j] * bf2f(xv[j]) + D[j]);
      og[j] = f2bf(g);
    }
    *reinterpret_cast<u16x8*>(dx + o) = out;
    if (dres) *reinterpret_cast<u16x8*>(dres + o) = og;
  }
}

// ---- residual block tail with a BN on both branches: y = relu(bn1(x) + bn2(r)) ------
// Both BNs see the same post-ReLU gradient g = dy (+ dy2) * relu'(y), so one pass
// accumulates sum g (shared), sum g * xhat and sum g * rhat, and its last block
// finalizes both BNs' coefficients; one apply pass writes dx and dr.  (The separate
// path: bn1 reduce + apply writing dx AND the residual gradient g, then the shortcut BN's
// reduce + apply reading g back.)
template <bool MASK>
__global__ __launch_bounds__(256) void bn_reduce_dual_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ r,
                                                             const bf16_t* __restrict__ dy,
                                                             const bf16_t* __restrict__ dy2,
                                                             const bf16_t* __restrict__ y,
                                                             const uint8_t* __restrict__ mask, int M, int C, int rpb,
                                                             int lanes, int rl, BnFin fin1, BnFin fin2, int ncop) {
  __shared__ float red[3][8 * 512];   // channel-major partials, see bn_reduce_kernel
  const int tid = threadIdx.x, lane = tid % lanes, rlane = tid / lanes;
  const int c0 = (blockIdx.x * 256 + lane) * 8;
  const bool active = rlane < rl && c0 < C;
  float s0[8], s1[8], s2[8], mu1[8], is1[8], mu2[8], is2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s0[j] = s1[j] = s2[j] = 0.f;
    mu1[j] = is1[j] = mu2[j] = is2[j] = 0.f;
  }
  if (active) {
    load8(fin1.save_mean + c0, mu1);
    load8(fin1.save_invstd + c0, is1);
    load8(fin2.save_mean + c0, mu2);
    load8(fin2.save_invstd + c0, is2);
    const int r_end = min(M, (int)(blockIdx.y + 1) * rpb);
#pragma unroll 2
    for (int row = blockIdx.y * rpb + rlane; row < r_end; row += rl) {
      const size_t o = (size_t)row * C + c0;
      const u16x8 xv = *reinterpret_cast<const u16x8*>(x + o);
      const u16x8 rv = *reinterpret_cast<const u16x8*>(r + o);
      const u16x8 gv = *reinterpret_cast<const u16x8*>(dy + o);
      u16x8 g2v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (dy2) g2v = *reinterpret_cast<const u16x8*>(dy2 + o);
      u16x8 yv;
      uint32_t mb = 0;
      if constexpr (MASK) mb = mask[o >> 3];
      else yv = *reinterpret_cast<const u16x8*>(y + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float g = bf2f(gv[j]) + bf2f(g2v[j]);
        if constexpr (MASK) g = ((mb >> j) & 1u) ? g : 0.f;
        else g = bf2f(yv[j]) > 0.f ? g : 0.f;
        s0[j] += g;
        s1[j] += g * (bf2f(xv[j]) - mu1[j]) * is1[j];
        s2[j] += g * (bf2f(rv[j]) - mu2[j]) * is2[j];
      }
    }
  }
  const int wrow = lanes * 8, js = 256 + lanes;
  if (rlane < rl) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      red[0][j * js + tid] = s0[j];
      red[1][j * js + tid] = s1[j];
      red[2][j * js + tid] = s2[j];
    }
  }
  __syncthreads();
  const int cp = (blockIdx.x + gridDim.x * blockIdx.y) % ncop;
  float* acc1 = fin1.acc + (size_t)cp * 2 * C;
  float* acc2 = fin2.acc + (size_t)cp * 2 * C;
  for (int idx = tid; idx < wrow; idx += 256) {
    const int j = idx / lanes, ln = idx - j * lanes;
    float t0 = 0.f, t1 = 0.f, t2 = 0.f;
    for (int q = 0; q < rl; ++q) {
      t0 += red[0][j * js + q * lanes + ln];
      t1 += red[1][j * js + q * lanes + ln];
      t2 += red[2][j * js + q * lanes + ln];
    }
    const int c = blockIdx.x * 2048 + ln * 8 + j;
    if (c < C) {
      bn_acc_add(acc1 + c, t0);
      bn_acc_add(acc1 + C + c, t1);
      bn_acc_add(acc2 + c, t0);
      bn_acc_add(acc2 + C + c, t2);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics have completed
  const int nblk = gridDim.x * gridDim.y;
  bn_finalize_last<true, kBnCopies>(fin1, M, C, nblk, &red[0][0], 3 * 8 * 512, ncop);
  __syncthreads();
  bn_finalize_last<true, kBnCopies>(fin2, M, C, nblk, &red[0][0], 3 * 8 * 512, ncop);
}

// The same statistics for small M (see bn_reduce_small_kernel): one workgroup per 64-channel
// group reads all rows and finalizes both BNs' coefficients itself.
template <bool MASK>
__global__ __launch_bounds__(256) void bn_reduce_dual_small_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ r, const bf16_t* __restrict__ dy,
    const bf16_t* __restrict__ dy2, const bf16_t* __restrict__ y, const uint8_t* __restrict__ mask, int M, int C,
    BnFin fin1, BnFin fin2, float* __restrict__ part1, float* __restrict__ part2, int* __restrict__ tickets, int rpb) {
  constexpr int kLanes = 8, kRl = 32, kJs = 256 + kLanes;
  __shared__ float red[3][8 * kJs];
  const int tid = threadIdx.x, lane = tid % kLanes, rlane = tid / kLanes;
  const int c0 = blockIdx.x * 64 + lane * 8;
  float s0[8], s1[8], s2[8], mu1[8], is1[8], mu2[8], is2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s0[j] = s1[j] = s2[j] = 0.f;
    mu1[j] = is1[j] = mu2[j] = is2[j] = 0.f;
  }
  if (c0 < C) {
    load8(fin1.save_mean + c0, mu1);
    load8(fin1.save_invstd + c0, is1);
    load8(fin2.save_mean + c0, mu2);
    load8(fin2.save_invstd + c0, is2);
    const int r_end = min(M, (int)(blockIdx.y + 1) * rpb);
    for (int r0 = blockIdx.y * rpb + rlane; r0 < r_end; r0 += 4 * kRl)   // batches of 4 rows (see above)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float w = r0 + u * kRl < r_end ? 1.f : 0.f;
      const size_t o = (size_t)min(r0 + u * kRl, r_end - 1) * C + c0;
      const u16x8 xv = *reinterpret_cast<const u16x8*>(x + o);
      const u16x8 rv = *reinterpret_cast<const u16x8*>(r + o);
      const u16x8 gv = *reinterpret_cast<const u16x8*>(dy + o);
      u16x8 g2v = {0, 0, 0, 0, 0, 0, 0, 0};
      if (dy2) g2v = *reinterpret_cast<const u16x8*>(dy2 + o);
      u16x8 yv;
      uint32_t mb = 0;
      if constexpr (MASK) mb = mask[o >> 3];
      else yv = *reinterpret_cast<const u16x8*>(y + o);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float g = (bf2f(gv[j]) + bf2f(g2v[j])) * w;
        if constexpr (MASK) g = ((mb >> j) & 1u) ? g : 0.f;
        else g = bf2f(yv[j]) > 0.f ? g : 0.f;
        s0[j] += g;
        s1[j] += g * (bf2f(xv[j]) - mu1[j]) * is1[j];
        s2[j] += g * (bf2f(rv[j]) - mu2[j]) * is2[j];
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][j * kJs + tid] = s0[j];
    red[1][j * kJs + tid] = s1[j];
    red[2][j * kJs + tid] = s2[j];
  }
  __syncthreads();
  if (tid < 64) {
    const int j = tid / kLanes, ln = tid - j * kLanes;
    float t0 = 0.f, t1 = 0.f, t2 = 0.f;
#pragma unroll 8
    for (int q = 0; q < kRl; ++q) {
      t0 += red[0][j * kJs + q * kLanes + ln];
      t1 += red[1][j * kJs + q * kLanes + ln];
      t2 += red[2][j * kJs + q * kLanes + ln];
    }
    const int c = blockIdx.x * 64 + ln * 8 + j;
    if (gridDim.y == 1) {
      if (c < C) {
        bn_finalize_channel<true>(fin1, M, C, c, t0, t1, 1.f / (float)M);
        bn_finalize_channel<true>(fin2, M, C, c, t0, t2, 1.f / (float)M);
      }
    } else if (c < C) {
      grp_store(part1 + (size_t)blockIdx.y * 2 * C + c, t0);
      grp_store(part1 + ((size_t)blockIdx.y * 2 + 1) * C + c, t1);
      grp_store(part2 + ((size_t)blockIdx.y * 2 + 1) * C + c, t2);
    }
  }
  if (gridDim.y == 1) return;
  __shared__ int last;
  if (!grp_ticket(tickets + blockIdx.x, gridDim.y, last)) return;
  float* tot = &red[0][0];
  const int cc = blockIdx.x * 64 + (tid & 63);
  grp_sum(part1, C, cc, 0, gridDim.y, tot);
  grp_sum(part1, C, cc, 1, gridDim.y, tot);
  grp_sum(part2, C, cc, 1, gridDim.y, tot + 512);
  __syncthreads();
  if (tid < 64 && cc < C) {
    const float S0 = tot[tid] + tot[64 + tid] + tot[128 + tid] + tot[192 + tid];
    const float S1 = tot[256 + tid] + tot[320 + tid] + tot[384 + tid] + tot[448 + tid];
    const float S2 = tot[768 + tid] + tot[832 + tid] + tot[896 + tid] + tot[960 + tid];
    bn_finalize_channel<true>(fin1, M, C, cc, S0, S1, 1.f / (float)M);
    bn_finalize_channel<true>(fin2, M, C, cc, S0, S2, 1.f / (float)M);
  }
}

// dx = A1 g + B1 x + D1, dr = A2 g + B2 r + D2
template <bool MASK>
__global__ __launch_bounds__(256) void bn_bwd_apply_dual_kernel(const bf16_t* __restrict__ x,
                                                                const bf16_t* __restrict__ r,
                                                                const bf16_t* __restrict__ dy,
                                                                const bf16_t* __restrict__ dy2,
                                                                const bf16_t* __restrict__ y,
                                                                const uint8_t* __restrict__ mask,
                                                                const float* __restrict__ coef1,
                                                                const float* __restrict__ coef2, bf16_t* __restrict__ dx,
                                                                bf16_t* __restrict__ dr, int M, int C, int rpb,
                                                                int lanes, int rl) {
  const int tid = threadIdx.x, lane = tid % lanes, rlane = tid / lanes;
  const int c0 = (blockIdx.x * 256 + lane) * 8;
  if (rlane >= rl || c0 >= C) return;
  float A1[8], B1[8], D1[8], A2[8], B2[8], D2[8];
  load8(coef1 + c0, A1);
  load8(coef1 + C + c0, B1);
  load8(coef1 + 2 * C + c0, D1);
  load8(coef2 + c0, A2);
  load8(coef2 + C + c0, B2);
  load8(coef2 + 2 * C + c0, D2);
  const int r_end = min(M, (int)(blockIdx.y + 1) * rpb);
#pragma unroll 2
  for (int row = blockIdx.y * rpb + rlane; row < r_end; row += rl) {
    const size_t o = (size_t)row * C + c0;
    const u16x8 xv = *reinterpret_cast<const u16x8*>(x + o);
    const u16x8 rv = *reinterpret_cast<const u16x8*>(r + o);
    const u16x8 gv = *reinterpret_cast<const u16x8*>(dy + o);
    u16x8 g2v = {0, 0, 0, 0, 0, 0, 0, 0};
    if (dy2) g2v = *reinterpret_cast<const u16x8*>(dy2 + o);
    u16x8 yv;
    uint32_t mb = 0;
    if constexpr (MASK) mb = mask[o >> 3];
    else yv = *reinterpret_cast<const u16x8*>(y + o);
    u16x8 ox, orr;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = bf2f(gv[j]) + bf2f(g2v[j]);
      if constexpr (MASK) g = ((mb >> j) & 1u) ? g : 0.f;
      else g = bf2f(yv[j]) > 0.f ? g : 0.f;
      ox[j] = f2bf(A1[j] * g + B1[j] * bf2f(xv[j]) + D1[j]);
      orr[j] = f2bf(A2[j] * g + B2[j] * bf2f(rv[j]) + D2[j]);
    }
    *reinterpret_cast<u16x8*>(dx + o) = ox;
    *reinterpret_cast<u16x8*>(dr + o) = orr;
  }
}

// ---- pooling (NHWC): one thread per 8 channels of one output pixel ----------
// Grid: blockIdx.y = one output row (n, p) [bwd: one input row (n, h)], threads over
// (column, 8-channel group) of that row -- one division per element instead of
// three.  KS > 0: a compile-time KS x KS window with stride ST (the ResNet stem's
// 3x3/2 max-pool: every tap's load issued up front, predicated); KS = 0: runtime
// window.  The 8 per-channel argmax bytes move as one 8-B load / store.
template <bool MAX, int KS, int ST>
__global__ __launch_bounds__(256) void pool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                       uint8_t* __restrict__ arg, int N, int H, int W, int C, int P,
                                                       int Q, int R_, int S_, int st_, int pad, int cl) {
  const int R = KS ? KS : R_, S = KS ? KS : S_, st = KS ? ST : st_;
  const int cv = C / 8;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= Q * cv) return;
  const int c8 = j % cv, q = j / cv;
  for (int row = blockIdx.y; row < N * P; row += gridDim.y) {
  const int n = row / P, p = row - n * P;
  const size_t img = (size_t)n * H;
  float best[8];
  int bidx[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    best[t] = MAX ? -INFINITY : 0.f;
    bidx[t] = 0;
  }
#pragma unroll
  for (int r = 0; r < (KS ? KS : 1); ++r) {
    for (int rr = (KS ? r : 0); rr < (KS ? r + 1 : R); ++rr) {
      const int h = p * st - pad + rr;
      const bool hok = h >= 0 && h < H;
#pragma unroll
      for (int s0 = 0; s0 < (KS ? KS : 1); ++s0) {
        for (int ss = (KS ? s0 : 0); ss < (KS ? s0 + 1 : S); ++ss) {
          const int w = q * st - pad + ss;
          if (!hok || w < 0 || w >= W) continue;
          const u16x8 v = *reinterpret_cast<const u16x8*>(x + ((img + h) * W + w) * C + c8 * 8);
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const float f = bf2f(v[t]);
            if (MAX) {
              if (f > best[t]) { best[t] = f; bidx[t] = rr * S + ss; }
            } else {
              best[t] += f;
            }
          }
        }
      }
    }
  }
  u16x8 o;
  const float inv = MAX ? 1.f : 1.f / (float)(R * S);  // count_include_pad=True (torch default)
#pragma unroll
  for (int t = 0; t < 8; ++t) o[t] = f2bf(best[t] * inv);
  const size_t oi = ((size_t)row * Q + q) * cv + c8;
  if (cl) {  // NCHW output of the cl logical channels (a flatten consumer reads it as is)
#pragma unroll
    for (int t = 0; t < 8; ++t)
      if (c8 * 8 + t < cl) y[(((size_t)n * cl + c8 * 8 + t) * P + p) * Q + q] = o[t];
  } else {
    reinterpret_cast<u16x8*>(y)[oi] = o;
  }
  if (MAX) {
    uint2 a;
    a.x = (uint32_t)bidx[0] | ((uint32_t)bidx[1] << 8) | ((uint32_t)bidx[2] << 16) | ((uint32_t)bidx[3] << 24);
    a.y = (uint32_t)bidx[4] | ((uint32_t)bidx[5] << 8) | ((uint32_t)bidx[6] << 16) | ((uint32_t)bidx[7] << 24);
    reinterpret_cast<uint2*>(arg)[oi] = a;
  }
  }  // rows
}

// gather form (no atomics): each input pixel sums the outputs whose window holds it
// (KS > 0: at most ceil(KS / ST)^2 candidate outputs, unrolled)
template <bool MAX, int KS, int ST>
__global__ __launch_bounds__(256) void pool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                                       bf16_t* __restrict__ dx, int N, int H, int W, int C, int P,
                                                       int Q, int R_, int S_, int st_, int pad,
                                                       const bf16_t* __restrict__ dy2, int cl) {
  const int R = KS ? KS : R_, S = KS ? KS : S_, st = KS ? ST : st_;
  constexpr int kSpan = KS ? (KS + ST - 1) / ST : 1;
  const int cv = C / 8;
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= W * cv) return;
  const int c8 = j % cv, w = j / cv;
  for (int row = blockIdx.y; row < N * H; row += gridDim.y) {
  const int n = row / H, h = row - n * H;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  // outputs p with p*st - pad <= h <= p*st - pad + R - 1
  const int p_lo = max(0, (h + pad - R + st) / st), p_hi = min(P - 1, (h + pad) / st);
  const int q_lo = max(0, (w + pad - S + st) / st), q_hi = min(Q - 1, (w + pad) / st);
#pragma unroll
  for (int i = 0; i < kSpan; ++i) {
    for (int p = (KS ? p_lo + i : p_lo); p <= (KS ? min(p_lo + i, p_hi) : p_hi); ++p) {
      const int r = h - (p * st - pad);
      if (r < 0 || r >= R) continue;
#pragma unroll
      for (int k = 0; k < kSpan; ++k) {
        for (int q = (KS ? q_lo + k : q_lo); q <= (KS ? min(q_lo + k, q_hi) : q_hi); ++q) {
          const int s = w - (q * st - pad);
          if (s < 0 || s >= S) continue;
          const size_t o = (((size_t)n * P + p) * Q + q) * cv + c8;
          u16x8 g;
          if (cl) {  // NCHW gradient of the cl logical channels (zero for the pad channels)
#pragma unroll
            for (int t = 0; t < 8; ++t)
              g[t] = c8 * 8 + t < cl ? dy[(((size_t)n * cl + c8 * 8 + t) * P + p) * Q + q] : (uint16_t)0;
          } else {
            g = reinterpret_cast<const u16x8*>(dy)[o];
          }
          u16x8 g2 = {0, 0, 0, 0, 0, 0, 0, 0};  // a second gradient of the same output (a residual
          if (dy2) g2 = reinterpret_cast<const u16x8*>(dy2)[o];  // block's input), summed here
          if (MAX) {
            const uint2 a = reinterpret_cast<const uint2*>(arg)[o];
            const uint32_t want = (uint32_t)(r * S + s);
#pragma unroll
            for (int t = 0; t < 8; ++t)
              if ((((t < 4 ? a.x : a.y) >> (8 * (t & 3))) & 0xffu) == want) acc[t] += bf2f(g[t]) + bf2f(g2[t]);
          } else {
#pragma unroll
            for (int t = 0; t < 8; ++t) acc[t] += bf2f(g[t]) + bf2f(g2[t]);
          }
        }
      }
    }
  }
  u16x8 out;
  const float inv = MAX ? 1.f : 1.f / (float)(R * S);
#pragma unroll
  for (int t = 0; t < 8; ++t) out[t] = f2bf(acc[t] * inv);
  reinterpret_cast<u16x8*>(dx)[((size_t)row * W + w) * cv + c8] = out;
  }  // rows
}

// ---- BatchNorm + ReLU + 3x3/2 max-pool in one pass (the ResNet stem) ----------
// The BN output is never stored: the forward applies scale / shift + ReLU to every
// tap of the window on the fly (same bf16 rounding as bn_apply_kernel, so the same
// maxima and argmax as the unfused BN -> pool pair) and writes only the pooled
// output + argmax.  relu'(bn(x)) at a window's argmax is (pooled max > 0), so the
// argmax byte doubles as the ReLU mask: kNoGrad when the max was clamped to 0.  The
// backward gathers the pool gradient of each input pixel from its candidate windows
// and feeds it straight into the BN statistics (reduce) and into dx = A g + B x + D
// (apply): the 4x larger pre-pool gradient is never written or re-read.  Traffic at the ResNet-18 stem, b64: forward 142 MB instead of
// 206 (apply) + 135 (pool); backward 387 MB instead of 135 + 206 + 309.
constexpr uint32_t kNoGrad = 0xffu;

// Branch-free address arithmetic throughout (out-of-range window taps / candidates are
// loaded from a clamped address and masked), so every load of a thread is independent
// and in flight together.  PAD (0 or 1) is compile-time: the tap of a window that holds
// a given input pixel is then a constant.
//
// The backward works on 2x2 input blocks (2a..2a+1) x (2b..2b+1): with a 3x3 / 2 window
// every pixel of the block lies in windows {a-1+PAD, a+PAD} x {b-1+PAD, b+PAD} (row 2a+di
// at tap di + 2 - PAD - 2i of window a-1+PAD+i), so a thread loads those 4 windows' argmax
// and gradient once and produces 4 pixels (1 window load per pixel instead of 2.25).
template <int PAD>
__device__ __forceinline__ void block_grads(const bf16_t* __restrict__ dy, const bf16_t* __restrict__ dy2,
                                            const uint8_t* __restrict__ arg, int n, int a, int b, int c8, int cv,
                                            int P, int Q, float (&g)[2][2][8]) {
  uint2 am[2][2];
  u16x8 gv[2][2], g2[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int p = a - 1 + PAD + i, q = b - 1 + PAD + k;
      const bool ok = p >= 0 && p < P && q >= 0 && q < Q;
      const int pc = min(max(p, 0), P - 1), qc = min(max(q, 0), Q - 1);
      const size_t o = (((size_t)n * P + pc) * Q + qc) * cv + c8;
      am[i][k] = reinterpret_cast<const uint2*>(arg)[o];
      gv[i][k] = reinterpret_cast<const u16x8*>(dy)[o];
      g2[i][k] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      if (dy2) g2[i][k] = reinterpret_cast<const u16x8*>(dy2)[o];
      if (!ok) am[i][k] = uint2{0xffffffffu, 0xffffffffu};   // kNoGrad bytes never match a tap
    }
#pragma unroll
  for (int di = 0; di < 2; ++di)
#pragma unroll
    for (int dj = 0; dj < 2; ++dj) {
#pragma unroll
      for (int t = 0; t < 8; ++t) g[di][dj][t] = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = di + 2 - PAD - 2 * i;
        if (r < 0 || r > 2) continue;   // compile-time
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int sc = dj + 2 - PAD - 2 * k;
          if (sc < 0 || sc > 2) continue;
          const uint32_t want = (uint32_t)(r * 3 + sc);
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const uint32_t bt = ((t < 4 ? am[i][k].x : am[i][k].y) >> (8 * (t & 3))) & 0xffu;
            g[di][dj][t] += bt == want ? bf2f(gv[i][k][t]) + bf2f(g2[i][k][t]) : 0.f;
          }
        }
      }
    }
}

// forward: one thread per (output pixel, 8-channel group), flat over the whole output (every lane
// busy: one workgroup pair per output row left 64 of 512 threads idle at Q = 56); cv divides 256
// (bnpool_ok), so a thread's channel group stays fixed across its grid-stride steps
template <int PAD>
__global__ __launch_bounds__(256) void bn_maxpool_fwd_kernel(const bf16_t* __restrict__ x,
                                                             const float* __restrict__ scale,
                                                             const float* __restrict__ shift, bf16_t* __restrict__ y,
                                                             uint8_t* __restrict__ arg, bf16_t* __restrict__ xam,
                                                             int N, int H, int W, int C, int P, int Q, FastDiv fq,
                                                             FastDiv fp) {
  const int cv = C / 8, lcv = __builtin_ctz(cv);
  const int c8 = threadIdx.x & (cv - 1);
  float sc[8], sh[8];
  load8(scale + c8 * 8, sc);
  load8(shift + c8 * 8, sh);
  const int total = N * P * Q * cv;
  for (int j = blockIdx.x * 256 + threadIdx.x; j < total; j += gridDim.x * 256) {
    const int tq = j >> lcv;
    const int row = fdiv(tq, fq), q = tq - row * Q;
    const int n = fdiv(row, fp), p = row - n * P;
    u16x8 v[3][3];
    bool ok[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        const int h = p * 2 - PAD + r, w = q * 2 - PAD + s;
        ok[r][s] = h >= 0 && h < H && w >= 0 && w < W;
        const int hc = min(max(h, 0), H - 1), wc = min(max(w, 0), W - 1);
        v[r][s] = *reinterpret_cast<const u16x8*>(x + (((size_t)n * H + hc) * W + wc) * C + c8 * 8);
      }
    float best[8];
    uint32_t bidx[8];
    u16x8 bx;   // the BN input at the argmax (xam: the backward statistics read it instead of x)
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      best[t] = -INFINITY;
      bidx[t] = 0;
      bx[t] = 0;
    }
#pragma unroll
    for (int r = 0; r < 3; ++r)
#pragma unroll
      for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          // the unfused BN apply's bf16 output, then the pool's first-max scan
          const float f = bf2f(f2bf(fmaxf(bf2f(v[r][s][t]) * sc[t] + sh[t], 0.f)));
          if (ok[r][s] && f > best[t]) {
            best[t] = f;
            bidx[t] = (uint32_t)(r * 3 + s);
            bx[t] = v[r][s][t];
          }
        }
    u16x8 o;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      o[t] = f2bf(best[t]);
      if (!(best[t] > 0.f)) bidx[t] = kNoGrad;   // relu'(bn) = 0 at the argmax: no gradient
    }
    const size_t oi = ((size_t)row * Q + q) * cv + c8;
    reinterpret_cast<u16x8*>(y)[oi] = o;
    if (xam) reinterpret_cast<u16x8*>(xam)[oi] = bx;
    uint2 am;
    am.x = bidx[0] | (bidx[1] << 8) | (bidx[2] << 16) | (bidx[3] << 24);
    am.y = bidx[4] | (bidx[5] << 8) | (bidx[6] << 16) | (bidx[7] << 24);
    reinterpret_cast<uint2*>(arg)[oi] = am;
  }
}

// backward statistics: acc += (sum g, sum g xhat) per channel; one thread per (2x2 input
// block column, 8-channel group) -- the channel group is fixed per thread (256 % cv == 0)
template <int PAD>
__global__ __launch_bounds__(256) void bn_maxpool_bwd_reduce_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, const bf16_t* __restrict__ dy2,
    const uint8_t* __restrict__ arg, const float* __restrict__ mean, const float* __restrict__ invstd,
    float* __restrict__ acc, int N, int H, int W, int C, int P, int Q, BnFin fin, int ncop) {
  // channel-major partials: element t of thread tid at red[k][t * 264 + tid] (consecutive
  // threads store consecutive words; the 264 = 8 mod 64 stride keeps the reads conflict-free)
  constexpr int kS = 264;
  __shared__ float red[2][8 * kS];
  const int cv = C / 8;
  const int tid = threadIdx.x;
  const int j = blockIdx.x * blockDim.x + tid;
  const int c8 = tid % cv, b = j / cv;
  const int Hb = (H + 1) / 2, Wb = (W + 1) / 2;
  float s0[8], s1[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    s0[t] = 0.f;
    s1[t] = 0.f;
  }
  if (b < Wb) {
    float mu[8], is[8];
    load8(mean + c8 * 8, mu);
    load8(invstd + c8 * 8, is);
    for (int rb = blockIdx.y; rb < N * Hb; rb += gridDim.y) {
      const int n = rb / Hb, a = rb - n * Hb;
      u16x8 xv[2][2];
      bool in[2][2];
#pragma unroll
      for (int di = 0; di < 2; ++di)
#pragma unroll
        for (int dj = 0; dj < 2; ++dj) {
          const int h = 2 * a + di, w = 2 * b + dj;
          in[di][dj] = h < H && w < W;
          xv[di][dj] = *reinterpret_cast<const u16x8*>(
              x + (((size_t)n * H + min(h, H - 1)) * W + min(w, W - 1)) * C + c8 * 8);
        }
      float g[2][2][8];
      block_grads<PAD>(dy, dy2, arg, n, a, b, c8, cv, P, Q, g);
#pragma unroll
      for (int di = 0; di < 2; ++di)
#pragma unroll
        for (int dj = 0; dj < 2; ++dj)
#pragma unroll
          for (int t = 0; t < 8; ++t) {
            const float gg = in[di][dj] ? g[di][dj][t] : 0.f;
            s0[t] += gg;
            s1[t] += gg * (bf2f(xv[di][dj][t]) - mu[t]) * is[t];
          }
    }
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    red[0][t * kS + tid] = s0[t];
    red[1][t * kS + tid] = s1[t];
  }
  __syncthreads();
  float* accc = acc + (size_t)((blockIdx.x + gridDim.x * blockIdx.y) % ncop) * 2 * C;
  for (int ch = tid; ch < C; ch += 256) {   // ch = c8 * 8 + t; threads c8, c8 + cv, ... hold it
    const int g8 = ch >> 3, t = ch & 7;
    float t0 = 0.f, t1 = 0.f;
    for (int k = g8; k < 256; k += cv) {
      t0 += red[0][t * kS + k];
      t1 += red[1][t * kS + k];
    }
    bn_acc_add(accc + ch, t0);
    bn_acc_add(accc + C + ch, t1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics have completed
  bn_finalize_last<true, kBnCopies>(fin, N * H * W, C, gridDim.x * gridDim.y, &red[0][0], 2 * 8 * kS, ncop);
}

// backward statistics from the pooled side: every input gradient of the pool is a sum of
// window gradients routed to that window's argmax, so sum_in g xhat = sum_windows dy xhat(x at
// the argmax) -- the forward's xam -- and sum_in g = sum of the routed dy.  Reads dy (+ dy2),
// the argmax bytes and xam (the pooled size, ~1/4 of the input each) instead of the whole BN
// input.  One thread per (pooled position, 8-channel group), grid-stride over positions.
__global__ __launch_bounds__(256) void bn_maxpool_bwd_reduce_am_kernel(
    const bf16_t* __restrict__ xam, const bf16_t* __restrict__ dy, const bf16_t* __restrict__ dy2,
    const uint8_t* __restrict__ arg, const float* __restrict__ mean, const float* __restrict__ invstd,
    float* __restrict__ acc, int npos, int M, int C, BnFin fin, int ncop) {
  constexpr int kS = 264;   // (layout as bn_maxpool_bwd_reduce_kernel)
  __shared__ float red[2][8 * kS];
  const int cv = C / 8;
  const int tid = threadIdx.x;
  const int c8 = tid % cv;   // fixed per thread: 256 % cv == 0 and the stride below is a multiple of cv
  float s0[8], s1[8], mu[8], is[8];
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    s0[t] = 0.f;
    s1[t] = 0.f;
  }
  load8(mean + c8 * 8, mu);
  load8(invstd + c8 * 8, is);
  const int64_t total = (int64_t)npos * cv, stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + tid; i < total; i += stride) {
    const uint2 am = reinterpret_cast<const uint2*>(arg)[i];
    const u16x8 gv = reinterpret_cast<const u16x8*>(dy)[i];
    const u16x8 xv = reinterpret_cast<const u16x8*>(xam)[i];
    u16x8 g2 = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
    if (dy2) g2 = reinterpret_cast<const u16x8*>(dy2)[i];
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const uint32_t bt = ((t < 4 ? am.x : am.y) >> (8 * (t & 3))) & 0xffu;
      const float gg = bt != kNoGrad ? bf2f(gv[t]) + bf2f(g2[t]) : 0.f;
      s0[t] += gg;
      s1[t] += gg * (bf2f(xv[t]) - mu[t]) * is[t];
    }
  }
#pragma unroll
  for (int t = 0; t < 8; ++t) {
    red[0][t * kS + tid] = s0[t];
    red[1][t * kS + tid] = s1[t];
  }
  __syncthreads();
  float* accc = acc + (size_t)(blockIdx.x % ncop) * 2 * C;
  for (int ch = tid; ch < C; ch += 256) {
    const int g8 = ch >> 3, t = ch & 7;
    float t0 = 0.f, t1 = 0.f;
    for (int k = g8; k < 256; k += cv) {
      t0 += red[0][t * kS + k];
      t1 += red[1][t * kS + k];
    }
    bn_acc_add(accc + ch, t0);
    bn_acc_add(accc + C + ch, t1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics have completed
  bn_finalize_last<true, kBnCopies>(fin, M, C, gridDim.x, &red[0][0], 2 * 8 * kS, ncop);
}

// backward apply: dx = A g + B x + D, one thread per (2x2 input block, 8-channel group), flat over
// the whole input like the forward (fb: division by the block columns, fh: by the block rows)
template <int PAD>
__global__ __launch_bounds__(256) void bn_maxpool_bwd_apply_kernel(
    const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy, const bf16_t* __restrict__ dy2,
    const uint8_t* __restrict__ arg, const float* __restrict__ coef, bf16_t* __restrict__ dx, int N, int H, int W,
    int C, int P, int Q, FastDiv fb, FastDiv fh) {
  const int cv = C / 8, lcv = __builtin_ctz(cv);
  const int c8 = threadIdx.x & (cv - 1);
  const int Hb = (H + 1) / 2, Wb = (W + 1) / 2;
  float A[8], B[8], D[8];
  load8(coef + c8 * 8, A);
  load8(coef + C + c8 * 8, B);
  load8(coef + 2 * C + c8 * 8, D);
  const int total = N * Hb * Wb * cv;
  for (int j = blockIdx.x * 256 + threadIdx.x; j < total; j += gridDim.x * 256) {
    const int tb = j >> lcv;
    const int rb = fdiv(tb, fb), b = tb - rb * Wb;
    const int n = fdiv(rb, fh), a = rb - n * Hb;
    u16x8 xv[2][2];
#pragma unroll
    for (int di = 0; di < 2; ++di)
#pragma unroll
      for (int dj = 0; dj < 2; ++dj)
        xv[di][dj] = *reinterpret_cast<const u16x8*>(
            x + (((size_t)n * H + min(2 * a + di, H - 1)) * W + min(2 * b + dj, W - 1)) * C + c8 * 8);
    float g[2][2][8];
    block_grads<PAD>(dy, dy2, arg, n, a, b, c8, cv, P, Q, g);
#pragma unroll
    for (int di = 0; di < 2; ++di)
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        const int h = 2 * a + di, w = 2 * b + dj;
        if (h >= H || w >= W) continue;
        u16x8 out;
#pragma unroll
        for (int t = 0; t < 8; ++t) out[t] = f2bf(A[t] * g[di][dj][t] + B[t] * bf2f(xv[di][dj][t]) + D[t]);
        *reinterpret_cast<u16x8*>(dx + (((size_t)n * H + h) * W + w) * C + c8 * 8) = out;
      }
  }
}

// global average pool [N][HW][C] -> [N][C] (fp32 accumulate), and its backward
__global__ void gap_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N, int HW, int C) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % cv), n = (int)(i / cv);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < HW; ++k) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(x + ((size_t)n * HW + k) * C + c8 * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j] / (float)HW);
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
}

// Split-HW global average pool: one block per (image, L-lane channel chunk); the
// block's 256 threads split the H*W positions over G = 256 / L row groups (each
// group reads L x 16 B contiguous) and the partial sums meet in LDS.  The one-
// thread-per-channel-octet kernel above walks all H*W positions serially: with
// ResNet-18's 64 x 7 x 7 x 512 input that is 16 workgroups doing 49 dependent
// loads each (16.8 us per step, profiles/r3s2/resnet18_b64_step_timeline.txt).
__global__ __launch_bounds__(256) void gap_fwd_split_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y,
                                                            int HW, int C, int L) {
  __shared__ float part[8][256];
  const int cv = C / 8, chunks = cv / L;
  const int n = blockIdx.x / chunks, ch = blockIdx.x - n * chunks;
  const int l = threadIdx.x % L, g = threadIdx.x / L, G = blockDim.x / L;
  const int c8 = ch * L + l;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const bf16_t* base = x + (size_t)n * HW * C + c8 * 8;
  for (int k = g; k < HW; k += G) {
    const u16x8 v = *reinterpret_cast<const u16x8*>(base + (size_t)k * C);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) part[j][threadIdx.x] = acc[j];
  __syncthreads();
  if (g != 0) return;
  u16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float t = 0.f;
    for (int q = 0; q < G; ++q) t += part[j][q * L + l];
    o[j] = f2bf(t / (float)HW);
  }
  reinterpret_cast<u16x8*>(y)[(size_t)n * cv + c8] = o;
}

__global__ void gap_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int N, int HW, int C) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * HW * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % cv);
    const int n = (int)(i / cv / HW);
    const u16x8 g = reinterpret_cast<const u16x8*>(dy)[(size_t)n * cv + c8];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(g[j]) / (float)HW);
    reinterpret_cast<u16x8*>(dx)[i] = o;
  }
}

}  // namespace

// Workspace (fp32, zeroed once, kept by the caller -- e.g. per BatchNorm module):
//   [0, C) scale | [C, 2C) shift | [6C, 9C) backward coefficients A, B, D |
//   [10C] forward ticket | [10C + 16] backward ticket |
//   [10C + 32, 26C + 32) kBnCopies x [2C] forward accumulators, shared by the BN
//   reduce and the conv-epilogue statistics path (one BN's statistics come from
//   exactly one of the two) |
//   [26C + 32, 42C + 32) kBnCopies x [2C] backward accumulators |
//   [42C + 32, ...) kGrpMax x [2C] row-group partials of the mid-M reduce (bn_reduce_small_kernel),
//   then its ceil(C / 64) per-column tickets.
// Accumulators and tickets are left zero by the finalizing block.
int bn_workspace_floats(int C) { return 42 * C + 32 + kGrpMax * 2 * C + ((C + 63) / 64 + 3) / 4 * 4; }

namespace {
float* grp_part(const BnArgs& a) { return a.ws + 42 * a.C + 32; }
int* grp_tickets(const BnArgs& a) { return reinterpret_cast<int*>(a.ws + 42 * a.C + 32 + kGrpMax * 2 * a.C); }
}  // namespace

BnFin bn_forward_fin(const BnArgs& a) {
  const int C = a.C;
  BnFin f{};
  f.acc = a.ws + 10 * C + 32;
  f.ticket = reinterpret_cast<int*>(a.ws + 10 * C);
  f.gamma = a.gamma;
  f.beta = a.beta;
  f.running_mean = a.running_mean;
  f.running_var = a.running_var;
  f.save_mean = a.save_mean;
  f.save_invstd = a.save_invstd;
  f.coef = a.ws;
  f.num_batches = a.num_batches;
  f.eps = a.eps;
  f.momentum = a.momentum;
  f.part = grp_part(a);
  f.tickets = grp_tickets(a);
  return f;
}

BnFin bn_forward_fin_conv(const BnArgs& a) { return bn_forward_fin(a); }

hipError_t bn_forward_apply(const BnArgs& a, hipStream_t s) {
  const int M = a.M, C = a.C;
  if (C % 8) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  const RedGeo g = red_geo(M, C);
  const dim3 grid(g.gx, g.gy);
  const float* sc = a.ws;
  const float* sh = a.ws + C;
#define BN_APPLY_CASE(RES, RELU, MASK)                                                                  \
  bn_apply_kernel<RES, RELU, MASK><<<grid, 256, 0, s>>>(a.x, a.residual, sc, sh, a.y, M, C, g.rpb, g.lanes, g.rl, \
                                                        a.mask)
  const bool mk = a.relu && a.mask != nullptr;
  if (a.residual) {
    if (mk) BN_APPLY_CASE(true, true, true);
    else if (a.relu) BN_APPLY_CASE(true, true, false);
    else BN_APPLY_CASE(true, false, false);
  } else {
    if (mk) BN_APPLY_CASE(false, true, true);
    else if (a.relu) BN_APPLY_CASE(false, true, false);
    else BN_APPLY_CASE(false, false, false);
  }
#undef BN_APPLY_CASE
  return hipGetLastError();
}

// the small-M reduce (bn_reduce_small_kernel, one workgroup per 64 channels) below this many
// rows (round 5: EnhancedCNN b64 2.09 -> 1.98 ms)
constexpr int kBnSmallRows = 2048;
int bn_small_rows() { return kBnSmallRows; }
// the same kernel with row groups up to 65536 rows, aiming at 512 workgroups with >= 256 rows
// each (round 5: 1.96 -> 1.94 ms, profiles/r5/bn_grouped_reduce_ab.jsonl)
struct Grp {
  int ny, rpb;
  bool on;
};
Grp grp_geo(int M, int C) {
  constexpr int rows = 65536, target = 512, min_rows = 256;
  if (M > rows && M > bn_small_rows()) return {0, 0, false};
  if (M > rows) return {1, M, true};
  const int G = (C + 63) / 64;
  int ny = (target + G - 1) / G;
  ny = std::min(ny, std::max(1, M / min_rows));
  ny = std::max(1, std::min(ny, kGrpMax));
  const int rpb = (M + ny - 1) / ny;
  return {(M + rpb - 1) / rpb, rpb, true};
}

// the statistics half of the forward: batch statistics (training) or the running ones (eval)
// -> scale / shift in a.ws
static void bn_forward_stats(const BnArgs& a, hipStream_t s) {
  const int M = a.M, C = a.C;
  const RedGeo g = red_geo(M, C, true);
  const dim3 grid(g.gx, g.gy);
  const Grp gg = grp_geo(M, C);
  if (a.training && gg.on) {
    const dim3 gs((C + 63) / 64, gg.ny);
    bn_reduce_small_kernel<false, false><<<gs, 256, 0, s>>>(a.x, nullptr, nullptr, nullptr, nullptr, M, C,
                                                            bn_forward_fin(a), nullptr, nullptr, grp_part(a),
                                                            grp_tickets(a), gg.rpb);
    return;
  }
  if (a.training) {
    const BnFin f = bn_forward_fin(a);
    bn_reduce_kernel<false, false><<<grid, 256, 0, s>>>(a.x, nullptr, nullptr, nullptr, nullptr, f.acc, M, C, g.rpb,
                                                        g.lanes, g.rl, f, nullptr, bn_ncop(false, g.gx * g.gy));
  } else {
    bn_eval_coeff_kernel<<<(C + 255) / 256, 256, 0, s>>>(a.gamma, a.beta, a.running_mean, a.running_var, a.ws,
                                                         a.ws + C, C, a.eps);
  }
}

hipError_t bn_forward(const BnArgs& a, hipStream_t s) {
  const int M = a.M, C = a.C;
  if (C % 8) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  bn_forward_stats(a, s);
  return bn_forward_apply(a, s);
}

// BN + ReLU + 3x3/2 max-pool (kernels above); 2048 workgroups in the backward statistics pass
namespace {
int bnpool_blocks() { return 2048; }
bool bnpool_ok(const BnArgs& a, int N, int H, int W, int P, int Q, int pad) {
  const int cv = a.C / 8;
  return a.C % 8 == 0 && cv <= 256 && 256 % cv == 0 && N > 0 && pad >= 0 && pad <= 1 &&
         P == (H + 2 * pad - 3) / 2 + 1 && Q == (W + 2 * pad - 3) / 2 + 1 && (int64_t)N * H * W == a.M &&
         (int64_t)N * H * W * cv < (1ll << 31);   // (flat item indices of the kernels above are 32-bit)
}
}  // namespace

hipError_t bn_maxpool_forward(const BnArgs& a, int N, int H, int W, int P, int Q, int pad, uint16_t* y,
                              uint8_t* arg, bool stats_ready, hipStream_t s, uint16_t* xam) {
  if (!bnpool_ok(a, N, H, W, P, Q, pad) || !a.relu || !y || !arg) return hipErrorInvalidValue;
  if (!stats_ready) bn_forward_stats(a, s);
  const int cv = a.C / 8;
  const unsigned g = (unsigned)(((int64_t)N * P * Q * cv + kBlock - 1) / kBlock);   // one thread per output item
  const FastDiv fq = make_fastdiv(Q), fp = make_fastdiv(P);
  if (pad)
    bn_maxpool_fwd_kernel<1><<<g, kBlock, 0, s>>>(a.x, a.ws, a.ws + a.C, y, arg, xam, N, H, W, a.C, P, Q, fq, fp);
  else
    bn_maxpool_fwd_kernel<0><<<g, kBlock, 0, s>>>(a.x, a.ws, a.ws + a.C, y, arg, xam, N, H, W, a.C, P, Q, fq, fp);
  return hipGetLastError();
}

hipError_t bn_maxpool_backward(const BnArgs& a, int N, int H, int W, int P, int Q, int pad, const uint16_t* dy,
                               const uint8_t* arg, uint16_t* dx, float* dgamma, float* dbeta, hipStream_t s,
                               bool grad_assign, const uint16_t* xam) {
  if (!bnpool_ok(a, N, H, W, P, Q, pad) || !dy || !arg || !dx) return hipErrorInvalidValue;
  const int C = a.C, cv = C / 8;
  BnFin f{};
  f.acc = a.ws + 10 * C + 32 + kBnCopies * 2 * C;
  f.ticket = reinterpret_cast<int*>(a.ws + 10 * C + 16);
  f.gamma = a.gamma;
  f.save_mean = a.save_mean;
  f.save_invstd = a.save_invstd;
  f.coef = a.ws + 6 * C;
  f.dgamma = dgamma;
  f.dbeta = dbeta;
  f.grad_assign = grad_assign ? 1 : 0;
  const int gx = ((W + 1) / 2 * cv + kBlock - 1) / kBlock, rows = N * ((H + 1) / 2);
  const dim3 gr(gx, std::min(rows, std::max(1, bnpool_blocks() / gx)));   // reduce: bounded atomics
  const unsigned ga = (unsigned)(((int64_t)rows * ((W + 1) / 2) * cv + kBlock - 1) / kBlock);   // apply: flat
  const FastDiv fb = make_fastdiv((W + 1) / 2), fh = make_fastdiv((H + 1) / 2);
  if (xam) {   // statistics from the pooled side (the forward stored x at every argmax)
    const int npos = N * P * Q;
    // (512 workgroups: each adds its 2 x C partial sums into the accumulator copies -- with the 2048
    // of bnpool_blocks that same-address atomic traffic bounded the pass, 37 us at b64)
    const int nb = (int)std::min<int64_t>(((int64_t)npos * cv + kBlock - 1) / kBlock, 512);
    bn_maxpool_bwd_reduce_am_kernel<<<nb, kBlock, 0, s>>>(xam, dy, a.dy2, arg, a.save_mean, a.save_invstd, f.acc,
                                                          npos, N * H * W, C, f, bn_ncop(true, nb));
    if (pad) bn_maxpool_bwd_apply_kernel<1><<<ga, kBlock, 0, s>>>(a.x, dy, a.dy2, arg, f.coef, dx, N, H, W, C, P, Q, fb, fh);
    else bn_maxpool_bwd_apply_kernel<0><<<ga, kBlock, 0, s>>>(a.x, dy, a.dy2, arg, f.coef, dx, N, H, W, C, P, Q, fb, fh);
  } else if (pad) {
    bn_maxpool_bwd_reduce_kernel<1><<<gr, kBlock, 0, s>>>(a.x, dy, a.dy2, arg, a.save_mean, a.save_invstd, f.acc, N,
                                                          H, W, C, P, Q, f, bn_ncop(true, gr.x * gr.y));
    bn_maxpool_bwd_apply_kernel<1><<<ga, kBlock, 0, s>>>(a.x, dy, a.dy2, arg, f.coef, dx, N, H, W, C, P, Q, fb, fh);
  } else {
    bn_maxpool_bwd_reduce_kernel<0><<<gr, kBlock, 0, s>>>(a.x, dy, a.dy2, arg, a.save_mean, a.save_invstd, f.acc, N,
                                                          H, W, C, P, Q, f, bn_ncop(true, gr.x * gr.y));
    bn_maxpool_bwd_apply_kernel<0><<<ga, kBlock, 0, s>>>(a.x, dy, a.dy2, arg, f.coef, dx, N, H, W, C, P, Q, fb, fh);
  }
  return hipGetLastError();
}

hipError_t bn_backward(const BnArgs& a, const uint16_t* dy, uint16_t* dx, uint16_t* dres, float* dgamma,
                       float* dbeta, hipStream_t s, bool grad_assign, bool stats_ready) {
  const int M = a.M, C = a.C;
  if (C % 8) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  const RedGeo g = red_geo(M, C);
  const dim3 grid(g.gx, g.gy);
  const RedGeo gr = red_geo(M, C, true);   // the reduce's own geometry (knobs above)
  const dim3 grid_r(gr.gx, gr.gy);
  BnFin f{};
  f.acc = a.ws + 10 * C + 32 + kBnCopies * 2 * C;
  f.ticket = reinterpret_cast<int*>(a.ws + 10 * C + 16);
  f.gamma = a.gamma;
  f.save_mean = a.save_mean;
  f.save_invstd = a.save_invstd;
  f.coef = a.ws + 6 * C;
  f.dgamma = dgamma;
  f.dbeta = dbeta;
  f.grad_assign = grad_assign ? 1 : 0;
  const Grp gg = grp_geo(M, C);
  const dim3 gs((C + 63) / 64, gg.ny);
  float* part = grp_part(a);
  int* tk = grp_tickets(a);
  if (stats_ready) {
    // (the producing dgrad's epilogue finalized f.coef / dgamma / dbeta)
  } else if (gg.on) {
    if (a.relu && a.mask)
      bn_reduce_small_kernel<true, true, true><<<gs, 256, 0, s>>>(a.x, dy, nullptr, a.save_mean, a.save_invstd, M, C,
                                                                  f, a.mask, a.dy2, part, tk, gg.rpb);
    else if (a.relu)
      bn_reduce_small_kernel<true, true><<<gs, 256, 0, s>>>(a.x, dy, a.y, a.save_mean, a.save_invstd, M, C, f, nullptr,
                                                            a.dy2, part, tk, gg.rpb);
    else
      bn_reduce_small_kernel<true, false><<<gs, 256, 0, s>>>(a.x, dy, nullptr, a.save_mean, a.save_invstd, M, C, f,
                                                             nullptr, a.dy2, part, tk, gg.rpb);
  } else if (a.relu && a.mask)
    bn_reduce_kernel<true, true, true><<<grid_r, 256, 0, s>>>(a.x, dy, nullptr, a.save_mean, a.save_invstd, f.acc, M,
                                                            C, gr.rpb, gr.lanes, gr.rl, f, a.mask,
                                                            bn_ncop(true, gr.gx * gr.gy), a.dy2);
  else if (a.relu)
    bn_reduce_kernel<true, true><<<grid_r, 256, 0, s>>>(a.x, dy, a.y, a.save_mean, a.save_invstd, f.acc, M, C, gr.rpb,
                                                      gr.lanes, gr.rl, f, nullptr, bn_ncop(true, gr.gx * gr.gy), a.dy2);
  else
    bn_reduce_kernel<true, false><<<grid_r, 256, 0, s>>>(a.x, dy, nullptr, a.save_mean, a.save_invstd, f.acc, M, C,
                                                       gr.rpb, gr.lanes, gr.rl, f, nullptr, bn_ncop(true, gr.gx * gr.gy),
                                                       a.dy2);
  if (a.relu && a.mask)
    bn_bwd_apply_kernel<true, true><<<grid, 256, 0, s>>>(a.x, dy, nullptr, f.coef, dx, dres, M, C, g.rpb, g.lanes,
                                                         g.rl, a.mask, a.dy2);
  else if (a.relu)
    bn_bwd_apply_kernel<true><<<grid, 256, 0, s>>>(a.x, dy, a.y, f.coef, dx, dres, M, C, g.rpb, g.lanes, g.rl, nullptr,
                                                   a.dy2);
  else
    bn_bwd_apply_kernel<false><<<grid, 256, 0, s>>>(a.x, dy, nullptr, f.coef, dx, dres, M, C, g.rpb, g.lanes, g.rl,
                                                    nullptr, a.dy2);
  return hipGetLastError();
}

hipError_t bn_dual_forward(const BnArgs& a, const BnArgs& b, bool ready_a, bool ready_b, hipStream_t s) {
  const int M = a.M, C = a.C;
  if (C % 8 || b.C != C || b.M != M || !a.relu || !a.training || !b.training) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  if (!ready_a) bn_forward_stats(a, s);
  if (!ready_b) bn_forward_stats(b, s);
  const RedGeo g = red_geo(M, C);
  const dim3 grid(g.gx, g.gy);
  if (a.mask)
    bn_apply_kernel<true, true, true, true><<<grid, 256, 0, s>>>(a.x, b.x, a.ws, a.ws + C, a.y, M, C, g.rpb, g.lanes,
                                                                 g.rl, a.mask, b.ws, b.ws + C);
  else
    bn_apply_kernel<true, true, false, true><<<grid, 256, 0, s>>>(a.x, b.x, a.ws, a.ws + C, a.y, M, C, g.rpb, g.lanes,
                                                                  g.rl, nullptr, b.ws, b.ws + C);
  return hipGetLastError();
}

namespace {
BnFin bn_backward_fin(const BnArgs& a, float* dgamma, float* dbeta, bool grad_assign) {
  const int C = a.C;
  BnFin f{};
  f.acc = a.ws + 10 * C + 32 + kBnCopies * 2 * C;
  f.ticket = reinterpret_cast<int*>(a.ws + 10 * C + 16);
  f.gamma = a.gamma;
  f.save_mean = a.save_mean;
  f.save_invstd = a.save_invstd;
  f.coef = a.ws + 6 * C;
  f.dgamma = dgamma;
  f.dbeta = dbeta;
  f.grad_assign = grad_assign ? 1 : 0;
  f.part = grp_part(a);
  f.tickets = grp_tickets(a);
  return f;
}
}  // namespace

BnFin bn_backward_fin_conv(const BnArgs& a, float* dgamma, float* dbeta, bool grad_assign) {
  return bn_backward_fin(a, dgamma, dbeta, grad_assign);
}

hipError_t bn_dual_backward(const BnArgs& a, const BnArgs& b, const uint16_t* dy, uint16_t* dx, uint16_t* dr,
                            float* dgamma_a, float* dbeta_a, float* dgamma_b, float* dbeta_b, bool assign_a,
                            bool assign_b, hipStream_t s) {
  const int M = a.M, C = a.C;
  if (C % 8 || b.C != C || b.M != M || !a.relu) return hipErrorInvalidValue;
  if (M <= 0) return hipSuccess;
  const BnFin fa = bn_backward_fin(a, dgamma_a, dbeta_a, assign_a);
  const BnFin fb = bn_backward_fin(b, dgamma_b, dbeta_b, assign_b);
  const RedGeo gr = red_geo(M, C, true);
  const dim3 grid_r(gr.gx, gr.gy);
  const int ncop = bn_ncop(true, gr.gx * gr.gy);
  const RedGeo g = red_geo(M, C);
  const dim3 grid(g.gx, g.gy);
  const Grp gg = grp_geo(M, C);
  const bool small = gg.on;
  const dim3 gs((C + 63) / 64, gg.ny);
  if (small && a.mask)
    bn_reduce_dual_small_kernel<true><<<gs, 256, 0, s>>>(a.x, b.x, dy, a.dy2, nullptr, a.mask, M, C, fa, fb,
                                                         grp_part(a), grp_part(b), grp_tickets(a), gg.rpb);
  else if (small)
    bn_reduce_dual_small_kernel<false><<<gs, 256, 0, s>>>(a.x, b.x, dy, a.dy2, a.y, nullptr, M, C, fa, fb,
                                                          grp_part(a), grp_part(b), grp_tickets(a), gg.rpb);
  if (a.mask) {
    if (!small)
      bn_reduce_dual_kernel<true><<<grid_r, 256, 0, s>>>(a.x, b.x, dy, a.dy2, nullptr, a.mask, M, C, gr.rpb, gr.lanes,
                                                         gr.rl, fa, fb, ncop);
    bn_bwd_apply_dual_kernel<true><<<grid, 256, 0, s>>>(a.x, b.x, dy, a.dy2, nullptr, a.mask, fa.coef, fb.coef, dx, dr,
                                                        M, C, g.rpb, g.lanes, g.rl);
  } else {
    if (!small)
      bn_reduce_dual_kernel<false><<<grid_r, 256, 0, s>>>(a.x, b.x, dy, a.dy2, a.y, nullptr, M, C, gr.rpb, gr.lanes,
                                                          gr.rl, fa, fb, ncop);
    bn_bwd_apply_dual_kernel<false><<<grid, 256, 0, s>>>(a.x, b.x, dy, a.dy2, a.y, nullptr, fa.coef, fb.coef, dx, dr,
                                                         M, C, g.rpb, g.lanes, g.rl);
  }
  return hipGetLastError();
}

hipError_t pool2d_fwd(const uint16_t* x, uint16_t* y, uint8_t* argmax, int N, int H, int W, int C, int P, int Q,
                      int R, int S, int stride, int pad, bool is_max, hipStream_t s, int nchw_c) {
  if (C % 8 || nchw_c < 0 || nchw_c > C) return hipErrorInvalidValue;
  if ((int64_t)N * P >= (1ll << 31) || (int64_t)Q * (C / 8) > (1 << 30)) return hipErrorInvalidValue;
  const dim3 g((Q * (C / 8) + kBlock - 1) / kBlock, std::min(N * P, 65535));
  const bool k3 = R == 3 && S == 3 && stride == 2;
  if (is_max && k3) pool_fwd_kernel<true, 3, 2><<<g, kBlock, 0, s>>>(x, y, argmax, N, H, W, C, P, Q, R, S, stride,
                                                                pad, nchw_c);
  else if (is_max) pool_fwd_kernel<true, 0, 1><<<g, kBlock, 0, s>>>(x, y, argmax, N, H, W, C, P, Q, R, S, stride,
                                                                pad, nchw_c);
  else pool_fwd_kernel<false, 0, 1><<<g, kBlock, 0, s>>>(x, y, argmax, N, H, W, C, P, Q, R, S, stride,
                                                                pad, nchw_c);
  return hipGetLastError();
}

hipError_t pool2d_bwd(const uint16_t* dy, const uint8_t* argmax, uint16_t* dx, int N, int H, int W, int C, int P,
                      int Q, int R, int S, int stride, int pad, bool is_max, hipStream_t s, const uint16_t* dy2,
                      int nchw_c) {
  if (C % 8 || nchw_c < 0 || nchw_c > C || (nchw_c && dy2)) return hipErrorInvalidValue;
  if ((int64_t)N * H >= (1ll << 31) || (int64_t)W * (C / 8) > (1 << 30)) return hipErrorInvalidValue;
  const dim3 g((W * (C / 8) + kBlock - 1) / kBlock, std::min(N * H, 65535));
  const bool k3 = R == 3 && S == 3 && stride == 2;
  if (is_max && k3)
    pool_bwd_kernel<true, 3, 2><<<g, kBlock, 0, s>>>(dy, argmax, dx, N, H, W, C, P, Q, R, S, stride, pad, dy2,
                                                   nchw_c);
  else if (is_max)
    pool_bwd_kernel<true, 0, 1><<<g, kBlock, 0, s>>>(dy, argmax, dx, N, H, W, C, P, Q, R, S, stride, pad, dy2,
                                                   nchw_c);
  else
    pool_bwd_kernel<false, 0, 1><<<g, kBlock, 0, s>>>(dy, argmax, dx, N, H, W, C, P, Q, R, S, stride, pad, dy2,
                                                   nchw_c);
  return hipGetLastError();
}

hipError_t global_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const int cv = C / 8;
  int L = 16;  // 16 lanes x 16 B = 256 contiguous bytes per row group
  while (L > 1 && cv % L) L >>= 1;
  if (HW >= 8 && (int64_t)N * (cv / L) <= INT32_MAX) {
    gap_fwd_split_kernel<<<(unsigned)((int64_t)N * (cv / L)), 256, 0, s>>>(x, y, HW, C, L);
    return hipGetLastError();
  }
  gap_fwd_kernel<<<grid_for((int64_t)N * C / 8), kBlock, 0, s>>>(x, y, N, HW, C);
  return hipGetLastError();
}

hipError_t global_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  gap_bwd_kernel<<<grid_for((int64_t)N * HW * C / 8), kBlock, 0, s>>>(dy, dx, N, HW, C);
  return hipGetLastError();
}

}  // namespace ldnn
