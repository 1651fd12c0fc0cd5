// Fused softmax cross-entropy forward + backward + accuracy (SURVEY §2.3 K14,
// K15, K21): one kernel replaces the reference's nn.CrossEntropyLoss forward
// (BAR/main.py:52, BAR/trainer.py:207), its autograd backward, the argmax /
// (pred == labels).sum() of BAR/trainer.py:213-215 and the three per-step
// .item() host syncs (loss and correct count are accumulated on the device).
// It also emits the last Linear layer's bias gradient (column sums of dlogits).
//
// One wave per row (lanes stride over classes), 4 waves per block, 16 rows per
// block; per-block partials are combined in LDS and added with one atomic per
// statistic / bias column.
#include <algorithm>

#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

constexpr int kRowsPerBlock = 16;  // 4 rows per wave: B = 4096 -> 256 blocks fill the chip
constexpr int kMaxColsPerLane = 16;  // C <= 1024

// Last-block finalize (fin.out set): every block's statistic atomics are made
// device-visible before its arrival is counted; the last arrival swaps the sums
// out of the accumulator (leaving it zero), writes [loss_sum * scale, #correct]
// and adds both into the running stats.
__device__ __forceinline__ void xent_finish(const XentFin& fin, float* stats) {
  if (fin.out == nullptr) return;
  __threadfence();
  __syncthreads();
  __shared__ int last;
  if (threadIdx.x == 0) last = atomicAdd(fin.cnt, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last || threadIdx.x != 0) return;
  __threadfence();
  const float l = atomicExch(fin.acc, 0.f), c = atomicExch(fin.acc + 1, 0.f);
  fin.out[0] = l * fin.scale;
  fin.out[1] = c;
  if (stats) {
    atomicAdd(stats, l);
    atomicAdd(stats + 1, c);
  }
  atomicExch(fin.cnt, 0u);
}

__global__ __launch_bounds__(256) void scale_bf16_kernel(const bf16_t* __restrict__ src, const float* __restrict__ scale,
                                                         bf16_t* __restrict__ out, int64_t n8) {
  const float k = *scale;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n8; i += stride) {
    const u16x8 v = reinterpret_cast<const u16x8*>(src)[i];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(v[j]) * k);
    reinterpret_cast<u16x8*>(out)[i] = o;
  }
}

__global__ __launch_bounds__(256) void xent_kernel(const bf16_t* __restrict__ logits,
                                                   const int64_t* __restrict__ labels,
                                                   bf16_t* __restrict__ dlogits, float* __restrict__ stats,
                                                   float* __restrict__ dbias, int B, int C, int ld,
                                                   float grad_scale, int rows_per_block, XentFin fin) {
  __shared__ float sdb[4][kMaxColsPerLane * 64];
  __shared__ float sstat[4][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nt = (ld + 63) / 64;
  float dacc[kMaxColsPerLane];
#pragma unroll
  for (int t = 0; t < kMaxColsPerLane; ++t) dacc[t] = 0.f;
  float loss_sum = 0.f, correct = 0.f;

  const int r_end = min(B, (blockIdx.x + 1) * rows_per_block);
  for (int r = blockIdx.x * rows_per_block + w; r < r_end; r += 4) {
    const bf16_t* row = logits + (size_t)r * ld;
    const int lab = (int)labels[r];
    float xv[kMaxColsPerLane];
    float mx = -INFINITY;
    int amax = 0x7fffffff;
#pragma unroll
    for (int t = 0; t < kMaxColsPerLane; ++t) {
      const int c = lane + 64 * t;
      xv[t] = -INFINITY;
      if (t < nt && c < C) {
        xv[t] = bf2f(row[c]);
        if (xv[t] > mx) { mx = xv[t]; amax = c; }
      }
    }
    // wave argmax (first index of the max)
    const float wmx = wave_max(mx);
    int cand = (mx == wmx) ? amax : 0x7fffffff;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) cand = min(cand, __shfl_xor(cand, o, 64));
    float se = 0.f, xl = 0.f;
#pragma unroll
    for (int t = 0; t < kMaxColsPerLane; ++t) {
      const int c = lane + 64 * t;
      if (t < nt && c < C) {
        se += __expf(xv[t] - wmx);
        if (c == lab) xl = xv[t];
      }
    }
    se = wave_sum(se);
    xl = wave_sum(xl);
    const float lse = wmx + __logf(se);
    const float inv = 1.f / se;
#pragma unroll
    for (int t = 0; t < kMaxColsPerLane; ++t) {
      const int c = lane + 64 * t;
      if (t < nt && c < ld) {
        float g = 0.f;
        if (c < C) g = (__expf(xv[t] - wmx) * inv - (c == lab ? 1.f : 0.f)) * grad_scale;
        const uint16_t gb = f2bf(g);
        dlogits[(size_t)r * ld + c] = gb;
        dacc[t] += bf2f(gb);
      }
    }
    if (lane == 0) {
      loss_sum += lse - xl;
      correct += (cand == lab) ? 1.f : 0.f;
    }
  }

  if (lane == 0) {
    sstat[w][0] = loss_sum;
    sstat[w][1] = correct;
  }
  if (dbias) {
#pragma unroll
    for (int t = 0; t < kMaxColsPerLane; ++t)
      if (t < nt) sdb[w][lane + 64 * t] = dacc[t];
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float* st = fin.out ? fin.acc : stats;
    atomicAdd(st + 0, sstat[0][0] + sstat[1][0] + sstat[2][0] + sstat[3][0]);
    atomicAdd(st + 1, sstat[0][1] + sstat[1][1] + sstat[2][1] + sstat[3][1]);
  }
  if (dbias) {
    for (int c = threadIdx.x; c < ld; c += blockDim.x)
      atomicAdd(dbias + c, sdb[0][c] + sdb[1][c] + sdb[2][c] + sdb[3][c]);
  }
  xent_finish(fin, stats);
}


// Small class counts (ld <= 64, e.g. 10 classes padded to 16): one ROW PER LANE.
// A lane reads its whole row with 16-B loads and needs no cross-lane reduction,
// so a 4096-row batch is one load round trip instead of a chain of wave
// shuffles per row.  Column sums for the bias gradient: per-column wave
// reduction, then one atomic per column per wave.
template <int LD>
__global__ __launch_bounds__(256) void xent_rows_kernel(const bf16_t* __restrict__ logits,
                                                        const int64_t* __restrict__ labels,
                                                        bf16_t* __restrict__ dlogits, float* __restrict__ stats,
                                                        float* __restrict__ dbias, int B, int C, int ld,
                                                        float grad_scale, XentFin fin) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = r < B;
  float x[LD];
  float loss = 0.f, correct = 0.f;
  float g[LD];
#pragma unroll
  for (int c = 0; c < LD; ++c) g[c] = 0.f;
  if (ok) {
    const u16x8* row = reinterpret_cast<const u16x8*>(logits + (size_t)r * ld);
#pragma unroll
    for (int v = 0; v < LD / 8; ++v) {
      const u16x8 q = row[v];
#pragma unroll
      for (int j = 0; j < 8; ++j) x[v * 8 + j] = bf2f(q[j]);
    }
    const int lab = (int)labels[r];
    float mx = -INFINITY;
    int am = 0;
#pragma unroll
    for (int c = 0; c < LD; ++c)
      if (c < C && x[c] > mx) { mx = x[c]; am = c; }
    float se = 0.f, xl = 0.f;
#pragma unroll
    for (int c = 0; c < LD; ++c)
      if (c == lab) xl = x[c];
#pragma unroll
    for (int c = 0; c < LD; ++c) {
      if (c < C) {
        x[c] = __expf(x[c] - mx);
        se += x[c];
      }
    }
    loss = mx + __logf(se) - xl;  // = logsumexp - x_label
    correct = (am == lab) ? 1.f : 0.f;
    const float inv = 1.f / se;
    u16x8 out[LD / 8];
#pragma unroll
    for (int c = 0; c < LD; ++c) {
      float v = 0.f;
      if (c < C) v = (x[c] * inv - (c == lab ? 1.f : 0.f)) * grad_scale;
      const uint16_t b = f2bf(v);
      out[c / 8][c % 8] = b;
      g[c] = bf2f(b);
    }
    u16x8* drow = reinterpret_cast<u16x8*>(dlogits + (size_t)r * ld);
#pragma unroll
    for (int v = 0; v < LD / 8; ++v) drow[v] = out[v];
  }
  // block-level reduction first: one atomic per statistic / bias column per BLOCK
  // (same-address fp32 atomics serialise in L2; per-wave atomics cost ~9 us here)
  __shared__ float part[4][LD + 2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  loss = wave_sum(loss);
  correct = wave_sum(correct);
  if (lane == 0) {
    part[w][LD] = loss;
    part[w][LD + 1] = correct;
  }
  if (dbias) {
#pragma unroll
    for (int c = 0; c < LD; ++c) {
      const float t = wave_sum(g[c]);
      if (lane == 0) part[w][c] = t;
    }
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (t < LD + 2 && (dbias || t >= LD)) {
    const float v = part[0][t] + part[1][t] + part[2][t] + part[3][t];
    atomicAdd(t < LD ? dbias + t : (fin.out ? fin.acc : stats) + (t - LD), v);
  }
  xent_finish(fin, stats);
}

}  // namespace

hipError_t softmax_xent(const uint16_t* logits, const int64_t* labels, uint16_t* dlogits, float* stats,
                        float* dbias, int B, int C, int ld, float grad_scale, hipStream_t s, const XentFin* finp) {
  if (ld > kMaxColsPerLane * 64 || C > ld) return hipErrorInvalidValue;
  const XentFin fin = finp ? *finp : XentFin{};
  if (fin.out && (fin.acc == nullptr || fin.cnt == nullptr)) return hipErrorInvalidValue;
  if (!fin.out && stats == nullptr) return hipErrorInvalidValue;
  if (B <= 0) return hipSuccess;
  const bool vec_ok = (ld % 8 == 0) && ((reinterpret_cast<uintptr_t>(logits) | reinterpret_cast<uintptr_t>(dlogits)) & 15) == 0;
  if (vec_ok && ld <= 64) {
    const int g = (B + 255) / 256;
    switch (ld) {
#define XENT_ROWS_CASE(L) \
      case L: xent_rows_kernel<L><<<g, 256, 0, s>>>(logits, labels, dlogits, stats, dbias, B, C, ld, grad_scale, fin); break;
      XENT_ROWS_CASE(8) XENT_ROWS_CASE(16) XENT_ROWS_CASE(24) XENT_ROWS_CASE(32) XENT_ROWS_CASE(40) XENT_ROWS_CASE(48) XENT_ROWS_CASE(56)
#undef XENT_ROWS_CASE
      default: xent_rows_kernel<64><<<g, 256, 0, s>>>(logits, labels, dlogits, stats, dbias, B, C, ld, grad_scale, fin); break;
    }
    return hipGetLastError();
  }
  // one row per wave while that still leaves < 256 blocks (a 64-row batch: 16 blocks
  // instead of 4 waves walking 16 rows each), 16 rows per block beyond
  const int rpb = B <= 4 * 256 ? 4 : kRowsPerBlock;
  const int g = (B + rpb - 1) / rpb;
  xent_kernel<<<g, 256, 0, s>>>(logits, labels, dlogits, stats, dbias, B, C, ld, grad_scale, rpb, fin);
  return hipGetLastError();
}

hipError_t scale_bf16_dev(const uint16_t* src, const float* scale, uint16_t* out, int64_t n, hipStream_t s) {
  if (n % 8 || ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(out)) & 15)) return hipErrorInvalidValue;
  if (n == 0) return hipSuccess;
  const int64_t n8 = n / 8;
  const int g = (int)std::min<int64_t>((n8 + 255) / 256, 1024);
  scale_bf16_kernel<<<g, 256, 0, s>>>(src, scale, out, n8);
  return hipGetLastError();
}

}  // namespace ldnn
