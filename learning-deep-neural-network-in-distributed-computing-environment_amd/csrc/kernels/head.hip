// Classifier-head kernels for a narrow last Linear layer (<= 64 classes).
//
// The reference runs the head as four separate ATen ops per step: the
// Linear (BAR/model.py:100, cuBLAS skinny GEMM), CrossEntropyLoss forward and
// backward (BAR/main.py:52, BAR/trainer.py:207-208), the argmax/correct count
// (BAR/trainer.py:213-215) and the head's weight/bias gradients inside
// loss.backward().  Generic GEMM tiles waste >= 7/8 of their MFMA work and pay
// split-K atomics at these shapes, so the head gets two kernels of its own:
//
//  head_fwd_xent:  logits = h W^T + b, softmax cross-entropy, dlogits,
//                  argmax -> loss / correct per workgroup (plain stores into a
//                  per-workgroup slot: no same-address atomics), one launch.
//                  16 rows per workgroup, 8 waves split K (skinny-N GEMM), the
//                  row softmax runs on the reduced accumulators in registers.
//  head_wgrad:     dW = dlogits^T h (+ db = column sums of dlogits).  The
//                  reduction runs over the batch, the strided dimension of both
//                  operands, so each wave stages its 32-row chunks through a
//                  private LDS image read back with ds_read_b64_tr_b16
//                  (hardware transpose) into MFMA fragments.  64 output
//                  columns x a batch slice per workgroup; slices combine with
//                  fp32 atomics into the (pre-cleared) gradient.
#include "ldnn_common.h"
#include "ldnn_gemm_tile.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

// ---------------------------------------------------------------------------
// forward + loss
// ---------------------------------------------------------------------------
constexpr int kFwdWaves = 8;

template <int NT>
__global__ __launch_bounds__(kFwdWaves * 64) void head_fwd_xent_kernel(HeadParams p) {
  __shared__ floatx4 red[kFwdWaves - 1][NT][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16;
  const int row = m0 + (lane & 15);
  const int kq = 8 * (lane >> 4);
  floatx4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = (p.K + 31) / 32;
  const bf16x8 zero = {};
#pragma unroll 8
  for (int st = w; st < nsteps; st += kFwdWaves) {
    const int k = st * 32 + kq;
    const bool kok = k < p.K;
    const bf16x8 a = (row < p.B && kok) ? *reinterpret_cast<const bf16x8*>(p.h + (size_t)row * p.ldh + k) : zero;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = j * 16 + (lane & 15);
      const bf16x8 b = (n < p.ldw_rows && kok) ? *reinterpret_cast<const bf16x8*>(p.W + (size_t)n * p.ldw + k) : zero;
      acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc[j], 0, 0, 0);
    }
  }
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j) red[w - 1][j][lane] = acc[j];
  }
  __syncthreads();
  if (w != 0) return;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int q = 0; q < kFwdWaves - 1; ++q) acc[j] += red[q][j][lane];

  // lane: row m0 + (lane & 15), classes c = j*16 + 4*(lane >> 4) + r
  const bool rok = row < p.B;
  const int cb = 4 * (lane >> 4);
  float x[NT][4];
  float mx = -INFINITY;
  int am = 0x7fffffff;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const floatx4 bias = *reinterpret_cast<const floatx4*>(p.bias + j * 16 + cb);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = j * 16 + cb + r;
      // logits are rounded to bf16 first: the loss sees exactly the stored logits
      x[j][r] = bf2f(f2bf(acc[j][r] + bias[r]));
      if (c < p.C && x[j][r] > mx) { mx = x[j][r]; am = c; }
    }
  }
  // combine the 4 lanes of a row (xor 16, 32): max, then first index of the max
#pragma unroll
  for (int o = 16; o <= 32; o <<= 1) {
    const float omx = __shfl_xor(mx, o, 64);
    const int oam = __shfl_xor(am, o, 64);
    if (omx > mx || (omx == mx && oam < am)) { mx = omx; am = oam; }
  }
  const int lab = rok ? (int)p.labels[row] : -1;
  float se = 0.f, xl = 0.f;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = j * 16 + cb + r;
      if (c < p.C) {
        const float e = __expf(x[j][r] - mx);
        if (c == lab) xl = x[j][r];
        x[j][r] = e;
        se += e;
      }
    }
  se += __shfl_xor(se, 16, 64);
  se += __shfl_xor(se, 32, 64);
  xl += __shfl_xor(xl, 16, 64);
  xl += __shfl_xor(xl, 32, 64);
  const float inv = 1.f / se;
  if (rok) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int c0 = j * 16 + cb;
      if (c0 >= p.ld) continue;
      u16x4 lo, g;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + r;
        const float logit = acc[j][r] + *(p.bias + c);
        lo[r] = f2bf(logit);
        g[r] = c < p.C ? f2bf((x[j][r] * inv - (c == lab ? 1.f : 0.f)) * p.grad_scale) : (uint16_t)0;
      }
      if (p.logits) *reinterpret_cast<u16x4*>(p.logits + (size_t)row * p.ld + c0) = lo;
      *reinterpret_cast<u16x4*>(p.dlogits + (size_t)row * p.ld + c0) = g;
    }
  }
  // per-workgroup loss / correct: lanes 0..15 hold one row each
  float loss = (rok && lane < 16) ? (mx + __logf(se) - xl) : 0.f;
  float corr = (rok && lane < 16 && am == lab) ? 1.f : 0.f;
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) {
    loss += __shfl_xor(loss, o, 64);
    corr += __shfl_xor(corr, o, 64);
  }
  if (lane == 0) {  // this workgroup's own slot: plain read-modify-write, replay-safe
    p.stats[2 * blockIdx.x] += loss;
    p.stats[2 * blockIdx.x + 1] += corr;
  }
}

// ---------------------------------------------------------------------------
// weight / bias gradient
// ---------------------------------------------------------------------------
constexpr int kWgWaves = 4;
constexpr int kWgCols = 64;   // output columns (h features) per workgroup
constexpr int kWgRows = 32;   // batch rows per wave step

template <int NT>
__global__ __launch_bounds__(kWgWaves * 64) void head_wgrad_kernel(HeadWgradParams p) {
  // per wave: h image [4 kb][4 rb][8][16] (4 KiB) + dz image [4 kb][NT][8][16]
  constexpr int kHBytes = kWgRows * kWgCols * 2;
  constexpr int kDBytes = kWgRows * 16 * NT * 2;
  __shared__ __attribute__((aligned(16))) char smem[kWgWaves * (kHBytes + kDBytes)];
  __shared__ floatx4 red[kWgWaves - 1][NT][4][64];
  __shared__ float dbred[kWgWaves][16 * NT];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  char* lh = smem + w * (kHBytes + kDBytes);
  char* ld = lh + kHBytes;
  const int col0 = blockIdx.x * kWgCols;
  const int split = blockIdx.y, nsplit = gridDim.y;
  const int rows_per_split = (p.B + nsplit - 1) / nsplit;
  const int b_begin = split * rows_per_split;
  const int b_end = min(p.B, b_begin + rows_per_split);
  const bool do_db = p.db != nullptr && blockIdx.x == 0;

  floatx4 acc[NT][4];
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[j][t] = floatx4{0.f, 0.f, 0.f, 0.f};
  float dbs[NT] = {};

  // loader lanes: h chunk [32 rows][64 cols] = 4 x (8 rows x 128 B); dz chunk [32][16 NT]
  const int hr = lane >> 3, hc = (lane & 7) * 8;
  for (int b0 = b_begin + w * kWgRows; b0 < b_end; b0 += kWgWaves * kWgRows) {
    u16x8 hv[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = b0 + i * 8 + hr, c = col0 + hc;
      hv[i] = (b < b_end && c < p.K) ? *reinterpret_cast<const u16x8*>(p.h + (size_t)b * p.ldh + c) : u16x8{};
    }
    u16x8 dv[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      // lane: row (lane >> 1), 8 classes at j*16 + (lane & 1)*8
      const int b = b0 + (lane >> 1), c = j * 16 + (lane & 1) * 8;
      dv[j] = (b < b_end && c < p.ld) ? *reinterpret_cast<const u16x8*>(p.dz + (size_t)b * p.ld + c) : u16x8{};
    }
    // stage into the transposed-read images (strided layout of ldnn_gemm_tile.h)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = i * 8 + hr;  // chunk row = reduction index
      *reinterpret_cast<u16x8*>(lh + lds_offset<false, kWgCols>(hc, r)) = hv[i];
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int r = lane >> 1;
      *reinterpret_cast<u16x8*>(ld + lds_offset<false, 16 * NT>(j * 16 + (lane & 1) * 8, r)) = dv[j];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
    bf16x8 fd[NT];
#pragma unroll
    for (int j = 0; j < NT; ++j) fd[j] = read_frag<false, 16 * NT>(ld, j, 0, lane);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const bf16x8 fh = read_frag<false, kWgCols>(lh, t, 0, lane);
#pragma unroll
      for (int j = 0; j < NT; ++j) acc[j][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fh, fd[j], acc[j][t], 0, 0, 0);
    }
    if (do_db) {
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) dbs[j] += (float)fd[j][q];
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // fragment reads done before the next chunk overwrites the image
    __builtin_amdgcn_wave_barrier();
  }

  // combine the waves' batch slices
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) red[w - 1][j][t][lane] = acc[j][t];
  }
  if (do_db) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      float v = dbs[j];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (lane < 16) dbred[w][j * 16 + lane] = v;
    }
  }
  __syncthreads();
  if (w != 0) return;
  const bool atomic = nsplit > 1;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    const int n = j * 16 + (lane & 15);  // output row (class)
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      floatx4 v = acc[j][t];
#pragma unroll
      for (int q = 0; q < kWgWaves - 1; ++q) v += red[q][j][t][lane];
      const int c = col0 + t * 16 + 4 * (lane >> 4);  // 4 consecutive h features
      if (n < p.nrows && c < p.K) {
        float* dst = p.dW + (size_t)n * p.lddw + c;
        if (atomic) {
#pragma unroll
          for (int r = 0; r < 4; ++r) atomicAdd(dst + r, v[r]);
        } else {
          *reinterpret_cast<floatx4*>(dst) = v;
        }
      }
    }
  }
  if (do_db && lane < 16) {
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = j * 16 + lane;
      if (n < p.nrows) {
        const float v = dbred[0][n] + dbred[1][n] + dbred[2][n] + dbred[3][n];
        if (atomic) atomicAdd(p.db + n, v);
        else p.db[n] = v;
      }
    }
  }
}

}  // namespace

hipError_t head_fwd_xent(const HeadParams& p, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  if (p.ld > 64 || p.ld % 16 != 0 || p.C > p.ld || p.ldw_rows > p.ld || p.K % 8 != 0) return hipErrorInvalidValue;
  const dim3 grid((p.B + 15) / 16), block(kFwdWaves * 64);
  switch (p.ld / 16) {
    case 1: head_fwd_xent_kernel<1><<<grid, block, 0, s>>>(p); break;
    case 2: head_fwd_xent_kernel<2><<<grid, block, 0, s>>>(p); break;
    case 3: head_fwd_xent_kernel<3><<<grid, block, 0, s>>>(p); break;
    default: head_fwd_xent_kernel<4><<<grid, block, 0, s>>>(p); break;
  }
  return hipGetLastError();
}

int head_wgrad_splits(int B, int K) {
  const int cols = (K + kWgCols - 1) / kWgCols;
  int s = (256 + cols - 1) / cols;                 // ~1 workgroup per CU (measured best: 11.6 vs 12.2 us at 2)
  const int max_by_rows = B / (kWgWaves * kWgRows * 2);  // >= 2 steps per wave
  if (s > max_by_rows) s = max_by_rows;
  return s < 1 ? 1 : (s > 64 ? 64 : s);
}

hipError_t head_wgrad(const HeadWgradParams& p, int splits, hipStream_t s) {
  if (p.B <= 0 || p.K <= 0) return hipSuccess;
  if (p.ld > 64 || p.ld % 16 != 0 || p.nrows > p.ld || p.K % 8 != 0 || p.ldh % 8 != 0) return hipErrorInvalidValue;
  if (splits < 1) splits = head_wgrad_splits(p.B, p.K);
  const dim3 grid((p.K + kWgCols - 1) / kWgCols, splits), block(kWgWaves * 64);
  switch (p.ld / 16) {
    case 1: head_wgrad_kernel<1><<<grid, block, 0, s>>>(p); break;
    case 2: head_wgrad_kernel<2><<<grid, block, 0, s>>>(p); break;
    case 3: head_wgrad_kernel<3><<<grid, block, 0, s>>>(p); break;
    default: head_wgrad_kernel<4><<<grid, block, 0, s>>>(p); break;
  }
  return hipGetLastError();
}

}  // namespace ldnn
