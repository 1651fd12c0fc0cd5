// Fused softmax cross-entropy forward + backward + accuracy (SURVEY §2.3 K14,
// K15, K21): one kernel replaces the reference's nn.CrossEntropyLoss forward
// (BAR/main.py:52, BAR/trainer.py:207), its autograd backward, the argmax /
// (pred == labels).sum() of BAR/trainer.py:213-215 and the three per-step
// .item() host syncs (loss and correct count are accumulated on the device).
// It also emits the last Linear layer's bias gradient (column sums of dlogits).
//
// One wave per row (lanes stride over classes), 4 waves per block, 64 rows per
// block; per-block partials are combined in LDS and added with one atomic per
// statistic / bias column.
#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

constexpr int kRowsPerBlock = 64;
constexpr int kMaxColsPerLane = 16;  // C <= 1024

__global__ __launch_bounds__(256) void xent_kernel(const bf16_t* __restrict__ logits,
                                                   const int64_t* __restrict__ labels,
                                                   bf16_t* __restrict__ dlogits, float* __restrict__ stats,
                                                   float* __restrict__ dbias, int B, int C, int ld,
                                                   float grad_scale) {
  __shared__ float sdb[4][kMaxColsPerLane * 64];
  __shared__ float sstat[4][2];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nt = (ld + 63) / 64;
  float dacc[kMaxColsPerLane];
#pragma unroll
  for (int t = 0; t < kMaxColsPerLane; ++t) dacc[t] = 0.f;
  float loss_sum = 0.f, correct = 0.f;

  const int r_end = min(B, (blockIdx.x + 1) * kRowsPerBlock);
  for (int r = blockIdx.x * kRowsPerBlock + w; r < r_end; r += 4) {
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
    atomicAdd(stats + 0, sstat[0][0] + sstat[1][0] + sstat[2][0] + sstat[3][0]);
    atomicAdd(stats + 1, sstat[0][1] + sstat[1][1] + sstat[2][1] + sstat[3][1]);
  }
  if (dbias) {
    for (int c = threadIdx.x; c < ld; c += blockDim.x)
      atomicAdd(dbias + c, sdb[0][c] + sdb[1][c] + sdb[2][c] + sdb[3][c]);
  }
}

}  // namespace

hipError_t softmax_xent(const uint16_t* logits, const int64_t* labels, uint16_t* dlogits, float* stats,
                        float* dbias, int B, int C, int ld, float grad_scale, hipStream_t s) {
  if (ld > kMaxColsPerLane * 64 || C > ld) return hipErrorInvalidValue;
  if (B <= 0) return hipSuccess;
  const int g = (B + kRowsPerBlock - 1) / kRowsPerBlock;
  xent_kernel<<<g, 256, 0, s>>>(logits, labels, dlogits, stats, dbias, B, C, ld, grad_scale);
  return hipGetLastError();
}

}  // namespace ldnn
