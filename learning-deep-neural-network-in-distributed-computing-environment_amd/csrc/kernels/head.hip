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
//                  With p.dh set it also runs the head's DGRAD: the workgroup's
//                  16 rows of h (<= 128 KiB) are staged in LDS as they stream in
//                  for the logits, so dh = (dlogits W) * act'(h) needs no second
//                  read of h, and the previous layer's bias gradient (column sums
//                  of dh) is reduced from per-workgroup slabs.  Measured on MI355X
//                  at 4096 x 4096 (scripts/bench_head.py) it is NOT faster than the
//                  separate K = 16 dgrad GEMM (fwd 11 -> 32 us fused vs 11 + 22.6):
//                  the 32 MB dh store (5.4 us), the class-loop FMAs (5.5 us) and the
//                  slab reduction (5 us) all land after the h stream instead of
//                  overlapping it.  At batch 16384 with the hipBLASLt dgrad it wins
//                  (129 us fused incl. the slab sum vs 51 + 68 us + the head fwd; step
//                  1.848 vs 1.887 ms), so the engine turns it on with library_dgrad.
//                  The dgrad re-reads h from global memory (L2 / Infinity Cache)
//                  (HeadParams::dgrad_mode 1) or stages it in LDS (mode 2) --
//                  measured equal (1.870 vs 1.868 ms/step).
//                  Mode 0 (default for <= 16 classes) instead runs the forward-only
//                  head kernel and then head_dgrad_stream_kernel: the dgrad as a
//                  pure h -> dh stream with the bias-gradient sums in the same pass
//                  (round 2: the fused kernel's per-16-row phases serialise on a CU
//                  and its 1024 per-workgroup slabs cost a 15 us reduction).
//  head_wgrad:     dW = dlogits^T h (+ db = column sums of dlogits).  The
//                  reduction runs over the batch, the strided dimension of both
//                  operands, so each wave stages its 32-row chunks through a
//                  private LDS image read back with ds_read_b64_tr_b16
//                  (hardware transpose) into MFMA fragments.  64 output
//                  columns x a batch slice per workgroup; slices combine with
//                  fp32 atomics into the (pre-cleared) gradient.
#include <algorithm>

#include <cstdlib>

#include "ldnn_common.h"
#include "ldnn_gemm_tile.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

// ---------------------------------------------------------------------------
// forward + loss
// ---------------------------------------------------------------------------
constexpr int kFwdWaves = 8;

constexpr int kHeadDgradMaxK = 4096;  // 16 rows x 4096 bf16 = 128 KiB of LDS

// 16-B chunk q of staged row r.  Rows are K rounded up to 128 elements apart (a
// whole number of 16-chunk groups), and the chunk is XORed with the row so the 16
// rows of one k-chunk land on different banks without leaving their row.
__device__ __forceinline__ int hs_off(int r, int q, int K) {
  return r * ((K + 127) & ~127) * 2 + ((q ^ (r & 15)) << 4);
}

// (acc: this wave's logits before the bias; red: nred more partial sums to add first;
// slot: the [loss, correct] pair of these 16 rows)
template <int NT, bool DG>
__device__ __forceinline__ void head_softmax_xent(const HeadParams& p, floatx4 (&acc)[NT], floatx4 (*red)[NT][64],
                                                  int nred, float* dls, int lane, int row, int slot) {
#pragma unroll
  for (int j = 0; j < NT; ++j)
    for (int q = 0; q < nred; ++q) acc[j] += red[q][j][lane];

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
  if constexpr (DG) {  // the same bf16-rounded dlogits the head wgrad reads back
    // (every lane's reads of red above are done before any lane writes dls over it)
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int c0 = j * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + r;
        const float gv = (rok && c < p.C) ? bf2f(f2bf((x[j][r] * inv - (c == lab ? 1.f : 0.f)) * p.grad_scale)) : 0.f;
        dls[(lane & 15) * p.ld + c] = gv;
      }
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
    p.stats[2 * slot] += loss;
    p.stats[2 * slot + 1] += corr;
  }
}

// dh[m0 + r][8q .. 8q+7] = act'(h) * sum_c dlogits[r][c] W[c][8q ..], for the 16 rows
// of this workgroup; thread t owns column chunks q = t, t + 512, ... (coalesced
// 16-B stores), keeps the 16 x 8 accumulators in registers over the classes, and
// adds its column sums to the previous layer's bias gradient.
template <int DEPI, bool HS>
__device__ __forceinline__ void head_dgrad_rows(const HeadParams& p, const char* hs, const float* dls, int m0) {
  const int nq = p.K >> 3;
  const int rows = min(16, p.B - m0);
  for (int q = threadIdx.x; q < nq; q += kFwdWaves * 64) {
    float acc[16][8];
#pragma unroll
    for (int r = 0; r < 16; ++r)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[r][i] = 0.f;
    for (int c = 0; c < p.C; ++c) {
      const u16x8 wv = *reinterpret_cast<const u16x8*>(p.W + (size_t)c * p.ldw + 8 * q);
      float wf[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) wf[i] = bf2f(wv[i]);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float g = dls[r * p.ld + c];
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[r][i] = fmaf(g, wf[i], acc[r][i]);
      }
    }
    float cs[8] = {};
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (r >= rows) continue;
      const u16x8 hv = HS ? *reinterpret_cast<const u16x8*>(hs + hs_off(r, q, p.K))
                          : *reinterpret_cast<const u16x8*>(p.h + (size_t)(m0 + r) * p.ldh + 8 * q);
      u16x8 o;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float hf = bf2f(hv[i]);
        float v = acc[r][i];
        if constexpr (DEPI == EPI_DRELU) v = hf > 0.f ? v : 0.f;
        else if constexpr (DEPI == EPI_DSIGMOID) v *= hf * (1.f - hf);
        o[i] = f2bf(v);
        cs[i] += bf2f(o[i]);
      }
      *reinterpret_cast<u16x8*>(p.dh + (size_t)(m0 + r) * p.lddh + 8 * q) = o;
    }
    if (p.dbias != nullptr) {  // this workgroup's column sums -> its slab (summed by slab_sum after)
      float* dst = p.dbias_ws + (size_t)blockIdx.x * p.K + 8 * q;
      reinterpret_cast<floatx4*>(dst)[0] = floatx4{cs[0], cs[1], cs[2], cs[3]};
      reinterpret_cast<floatx4*>(dst)[1] = floatx4{cs[4], cs[5], cs[6], cs[7]};
    }
  }
}

// DEPI: -1 = no fused dgrad; EPI_NONE / EPI_DRELU / EPI_DSIGMOID = dgrad with that
// activation derivative.  HS: the dgrad reads h from the workgroup's LDS copy
// (138 KiB of LDS: one workgroup per CU, so the h stream, the softmax and the dgrad
// of a CU never overlap) instead of re-reading its 16 rows from global memory,
// where they were just streamed through L2 / the 256 MB Infinity Cache and where
// the 7 KiB workgroups co-reside and overlap their phases.
template <int NT, int DEPI, bool HS>
__global__ __launch_bounds__(kFwdWaves * 64) void head_fwd_xent_kernel(HeadParams p) {
  constexpr bool DG = DEPI >= 0;
  constexpr int kRedBytes = (kFwdWaves - 1) * NT * 64 * 16;
  __shared__ __attribute__((aligned(16))) char smem[kRedBytes + (DG && HS ? 16 * kHeadDgradMaxK * 2 : 0)];
  floatx4(*red)[NT][64] = reinterpret_cast<floatx4(*)[NT][64]>(smem);
  char* hs = smem + kRedBytes;
  float* dls = reinterpret_cast<float*>(smem);  // [16][ld] dlogits, over red once wave 0 has consumed it
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16;
  const int row = m0 + (lane & 15);
  const int kq = 8 * (lane >> 4);
  floatx4 acc[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = (p.K + 31) / 32;
  const bf16x8 zero = {};
#pragma unroll 16  // (K = 4096: all 16 of a wave's loads in flight at once)
  for (int st = w; st < nsteps; st += kFwdWaves) {
    const int k = st * 32 + kq;
    const bool kok = k < p.K;
    const bf16x8 a = (row < p.B && kok) ? *reinterpret_cast<const bf16x8*>(p.h + (size_t)row * p.ldh + k) : zero;
    if constexpr (DG && HS) {
      if (kok) *reinterpret_cast<bf16x8*>(hs + hs_off(lane & 15, k >> 3, p.K)) = a;
    }
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
  if (w == 0) head_softmax_xent<NT, DG>(p, acc, red, kFwdWaves - 1, dls, lane, row, blockIdx.x);
  if constexpr (DG) {
    __syncthreads();  // dlogits of the 16 rows in LDS, h staged
    head_dgrad_rows<DEPI, HS>(p, hs, dls, m0);
  }
}

// Loss from partial logits (EPI_BIAS_RELU_HEAD forward, gemm_q.hip): one wave per 16
// rows sums the nparts [B][16] fp32 slabs in the head kernel's accumulator layout
// (lane: row l & 15, classes 4 (l >> 4) + r) -- 16 KiB per wave, the whole pass reads
// nparts x 64 B per row instead of the K x 2 B of h -- then the same softmax-xent.
constexpr int kPartWaves = 4;
__global__ __launch_bounds__(kPartWaves * 64) void head_xent_parts_kernel(HeadParams p, const float* parts,
                                                                          int nparts) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int slot = blockIdx.x * kPartWaves + w;
  const int m0 = slot * 16;
  if (m0 >= p.B) return;
  const int row = m0 + (lane & 15);
  floatx4 acc[1] = {floatx4{0.f, 0.f, 0.f, 0.f}};
  if (row < p.B) {
    const float* src = parts + (size_t)row * 16 + 4 * (lane >> 4);
    const size_t stride = (size_t)p.B * 16;
    int s = 0;
    for (; s + 4 <= nparts; s += 4) {  // four 16-B loads in flight per lane
      const floatx4 a = *reinterpret_cast<const floatx4*>(src + (s + 0) * stride);
      const floatx4 b = *reinterpret_cast<const floatx4*>(src + (s + 1) * stride);
      const floatx4 c = *reinterpret_cast<const floatx4*>(src + (s + 2) * stride);
      const floatx4 d = *reinterpret_cast<const floatx4*>(src + (s + 3) * stride);
      acc[0] += (a + b) + (c + d);
    }
    for (; s < nparts; ++s) acc[0] += *reinterpret_cast<const floatx4*>(src + s * stride);
  }
  head_softmax_xent<1, false>(p, acc, nullptr, 0, nullptr, lane, row, slot);
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
  u16x8 hv[4], dv[NT];
  // chunk loads are software-pipelined: chunk b0 + stride is in flight while
  // chunk b0 is staged and multiplied
  auto load_chunk = [&](int b0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int b = b0 + i * 8 + hr, c = col0 + hc;
      hv[i] = (b < b_end && c < p.K) ? *reinterpret_cast<const u16x8*>(p.h + (size_t)b * p.ldh + c) : u16x8{};
    }
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      // lane: row (lane >> 1), 8 classes at j*16 + (lane & 1)*8
      const int b = b0 + (lane >> 1), c = j * 16 + (lane & 1) * 8;
      dv[j] = (b < b_end && c < p.ld) ? *reinterpret_cast<const u16x8*>(p.dz + (size_t)b * p.ld + c) : u16x8{};
    }
  };
  constexpr int kStride = kWgWaves * kWgRows;
  if (b_begin + w * kWgRows < b_end) load_chunk(b_begin + w * kWgRows);
  for (int b0 = b_begin + w * kWgRows; b0 < b_end; b0 += kStride) {
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
    if (b0 + kStride < b_end) load_chunk(b0 + kStride);
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0) only: the prefetch stays in flight
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

// ---------------------------------------------------------------------------
// streaming head dgrad (<= 16 classes): dh = (dlogits W) * act'(h), dbias += colsums
// ---------------------------------------------------------------------------
// A pure stream over h (read) and dh (write) -- the two tensors that cost bytes --
// laid out like act_bwd_colsum (elementwise.hip): a thread owns 8 columns and walks
// rows 8 apart, so every h load / dh store is a 16-B piece of a 512-B row run.  The
// thread keeps W[c][its 8 columns] for all 16 (padded) classes in registers; each
// row's 16 bf16 dlogits (32 B, the same for the 32 lanes of a row) come from L1.
// The column sums are reduced over the workgroup's 8 row lanes in LDS and added
// with one atomic per column per workgroup.  Two rows per iteration keep 4 loads in
// flight per lane.
template <int DEPI>
__global__ __launch_bounds__(256) void head_dgrad_stream_kernel(HeadParams p, int rows_per_block) {
  __shared__ float part[8][256];
  const int cg = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + cg) * 8;
  const int r_begin = blockIdx.y * rows_per_block;
  const int r_end = min(p.B, r_begin + rows_per_block);
  const bool cok = c0 < p.K;
  float wf[16][8];
#pragma unroll
  for (int c = 0; c < 16; ++c) {
    u16x8 w = {};
    if (cok && c < p.ldw_rows) w = *reinterpret_cast<const u16x8*>(p.W + (size_t)c * p.ldw + c0);
#pragma unroll
    for (int i = 0; i < 8; ++i) wf[c][i] = bf2f(w[i]);
  }
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  auto row_out = [&](const u16x8& g0, const u16x8& g1, const u16x8& hv, int r) {
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const float gc = bf2f(c < 8 ? g0[c] : g1[c - 8]);  // padded classes hold 0
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = fmaf(gc, wf[c][i], v[i]);
    }
    u16x8 o;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float hf = bf2f(hv[i]);
      float x = v[i];
      if constexpr (DEPI == EPI_DRELU) x = hf > 0.f ? x : 0.f;
      else if constexpr (DEPI == EPI_DSIGMOID) x *= hf * (1.f - hf);
      o[i] = f2bf(x);
      s[i] += bf2f(o[i]);
    }
    *reinterpret_cast<u16x8*>(p.dh + (size_t)r * p.lddh + c0) = o;
  };
  auto hrow = [&](int r) -> u16x8 { return *reinterpret_cast<const u16x8*>(p.h + (size_t)r * p.ldh + c0); };
  if (cok) {
    int r = r_begin + ty;
    for (; r + 8 < r_end; r += 16) {
      const u16x8* gp0 = reinterpret_cast<const u16x8*>(p.dlogits + (size_t)r * p.ld);
      const u16x8* gp1 = reinterpret_cast<const u16x8*>(p.dlogits + (size_t)(r + 8) * p.ld);
      const u16x8 a0 = gp0[0], a1 = gp0[1], b0 = gp1[0], b1 = gp1[1];
      const u16x8 h0 = hrow(r), h1 = hrow(r + 8);
      row_out(a0, a1, h0, r);
      row_out(b0, b1, h1, r + 8);
    }
    for (; r < r_end; r += 8) {
      const u16x8* gp0 = reinterpret_cast<const u16x8*>(p.dlogits + (size_t)r * p.ld);
      row_out(gp0[0], gp0[1], hrow(r), r);
    }
  }
  if (p.dbias == nullptr) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) part[ty][cg * 8 + j] = s[j];
  __syncthreads();
  if (ty == 0 && cok) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) t += part[q][cg * 8 + j];
      atomicAdd(p.dbias + c0 + j, t);
    }
  }
}

template <int DEPI>
hipError_t launch_head_dgrad_stream(const HeadParams& p, hipStream_t s) {
  const int gx = (p.K + 255) / 256;
  int gy = (p.B + 255) / 256;
  if (gy > 256) gy = 256;
  const int rpb = (p.B + gy - 1) / gy;
  head_dgrad_stream_kernel<DEPI><<<dim3(gx, gy), 256, 0, s>>>(p, rpb);
  return hipGetLastError();
}

template <int DEPI, bool HS>
hipError_t launch_head_fwd(const HeadParams& p, hipStream_t s) {
  const dim3 grid((p.B + 15) / 16), block(kFwdWaves * 64);
  switch (p.ld / 16) {
    case 1: head_fwd_xent_kernel<1, DEPI, HS><<<grid, block, 0, s>>>(p); break;
    case 2: head_fwd_xent_kernel<2, DEPI, HS><<<grid, block, 0, s>>>(p); break;
    case 3: head_fwd_xent_kernel<3, DEPI, HS><<<grid, block, 0, s>>>(p); break;
    default: head_fwd_xent_kernel<4, DEPI, HS><<<grid, block, 0, s>>>(p); break;
  }
  return hipGetLastError();
}

template <int DEPI>
hipError_t launch_head_fwd_dg(const HeadParams& p, hipStream_t s) {
  return p.dgrad_mode == 2 ? launch_head_fwd<DEPI, true>(p, s) : launch_head_fwd<DEPI, false>(p, s);
}

template <int DEPI>
hipError_t head_dgrad_dispatch(const HeadParams& p, hipStream_t s) {
  if (p.dgrad_mode == 0) {  // streaming: forward-only head kernel, then the dgrad stream
    hipError_t e = launch_head_fwd<-1, false>(p, s);
    if (e != hipSuccess) return e;
    return launch_head_dgrad_stream<DEPI>(p, s);
  }
  hipError_t e = launch_head_fwd_dg<DEPI>(p, s);
  // per-workgroup column sums -> bias gradient: 256 same-address fp32 atomics per
  // column measured 100+ us; a slab reduction over the chip costs a few
  if (e != hipSuccess || p.dbias == nullptr) return e;
  return slab_sum(p.dbias_ws, p.dbias, p.K / 4, (p.B + 15) / 16, 1.f, s);
}

}  // namespace

hipError_t head_fwd_xent(const HeadParams& p, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  if (p.ld > 64 || p.ld % 16 != 0 || p.C > p.ld || p.ldw_rows > p.ld || p.K % 8 != 0) return hipErrorInvalidValue;
  if (p.dh == nullptr) return launch_head_fwd<-1, false>(p, s);
  if (p.lddh % 8 != 0) return hipErrorInvalidValue;
  if (p.dgrad_mode < 0 || p.dgrad_mode > 2 || (p.dgrad_mode == 0 && p.ld != 16)) return hipErrorInvalidValue;
  if ((p.dgrad_mode == 1 || p.dgrad_mode == 2) &&
      (p.K > kHeadDgradMaxK || (p.dbias != nullptr && p.dbias_ws == nullptr)))
    return hipErrorInvalidValue;
  switch (p.dgrad_epi) {
    case EPI_NONE: return head_dgrad_dispatch<EPI_NONE>(p, s);
    case EPI_DRELU: return head_dgrad_dispatch<EPI_DRELU>(p, s);
    case EPI_DSIGMOID: return head_dgrad_dispatch<EPI_DSIGMOID>(p, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t head_xent_parts(const HeadParams& p, const float* parts, int nparts, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  if (p.ld != 16 || p.C > 16 || nparts < 1 || parts == nullptr) return hipErrorInvalidValue;
  const int slots = (p.B + 15) / 16;
  head_xent_parts_kernel<<<(slots + kPartWaves - 1) / kPartWaves, kPartWaves * 64, 0, s>>>(p, parts, nparts);
  return hipGetLastError();
}

hipError_t head_dgrad_stream(const HeadParams& p, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  if (p.ld != 16 || p.dh == nullptr || p.lddh % 8 != 0 || p.K % 8 != 0 || p.ldw_rows > 16) return hipErrorInvalidValue;
  switch (p.dgrad_epi) {
    case EPI_NONE: return launch_head_dgrad_stream<EPI_NONE>(p, s);
    case EPI_DRELU: return launch_head_dgrad_stream<EPI_DRELU>(p, s);
    case EPI_DSIGMOID: return launch_head_dgrad_stream<EPI_DSIGMOID>(p, s);
    default: return hipErrorInvalidValue;
  }
}

// ---------------------------------------------------------------------------
// fused head backward: the head's dgrad AND wgrad in one pass over h (ld == 16)
// ---------------------------------------------------------------------------
//   dh[m][n] = act'(h[m][n]) * sum_c dlogits[m][c] W[c][n]      (bf16, dbias += column sums)
//   dW[c][n] += sum_m dlogits[m][c] h[m][n]                      (fp32 atomics, pre-cleared)
//   db[c]    += sum_m dlogits[m][c]
// Both products are rank-16 and run on v_mfma_f32_16x16x16_bf16 (the VALU form of
// head_dgrad_stream spends ~128 FMAs per 8 outputs: VALU-bound at ~62 us for a
// 16384 x 4096 h on MI355X, and head_wgrad re-read the same 128 MB of h for another
// ~34 us).  A wave owns a 64-column strip and walks 16-row blocks:
//  * dgrad: 4 MFMAs (one per 4-column group t), operand A = W^T with its rows mapped to
//    columns so that lane (g = l/16, r16 = l%16) ends up holding dh[m0 + r16][n0 + 8g ..
//    8g+7] and [n0 + 32 + 8g .. 32 + 8g + 7] -- the same columns it loaded from h for the
//    ReLU: two 16-B loads and two 16-B stores per lane, each instruction covering 64
//    contiguous bytes of 16 rows (measured +x % over 32-B lane pieces).
//  * wgrad: the block (h 16 x 64, dlogits 16 x 16) is staged in the wave's LDS slice and
//    read back k-major with ds_read_b64_tr_b16 as the MFMA operands (k = the 16 rows):
//    4 MFMAs per block accumulate dW^T[n][c] in 16 registers per lane.
// The 4 waves of a workgroup take the same strip, interleaved 16-row blocks, and combine
// their dW / dbias / db partials in LDS before one atomic per output per workgroup;
// gridDim.y row groups (~2 workgroups per CU) add up by fp32 atomics.
typedef short s16x4 __attribute__((ext_vector_type(4)));
constexpr int kHbUnroll = 4;  // 16-row blocks whose loads are in flight together per wave

template <bool RELU>
__global__ __launch_bounds__(256) void head_bwd_kernel(HeadParams p, int rows_per_wg) {
  constexpr int kH = 16 * 128, kD = 16 * 32, kSt = kH + kD;  // one 16-row block: h + dlogits
  constexpr int kWave = kHbUnroll * kSt;                      // a wave's staging slice
  __shared__ __attribute__((aligned(16))) char smem[4 * kWave];  // staging, then the cross-wave partials
  static_assert(4 * kWave >= 4 * 64 * 17 * 4, "the reduction scratch fits");
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int g = lane >> 4, r16 = lane & 15;
  const int n0 = blockIdx.x * 64;
  const int r_begin = blockIdx.y * rows_per_wg, r_end = min(p.B, r_begin + rows_per_wg);
  char* const st = smem + wid * kWave;
  typedef __attribute__((address_space(3))) bf16x4 lds_b4;

  // lane (g, r16) owns row r16 of a block and columns n0 + hcol(k), k = 0..15: 8g..8g+7 and
  // 32+8g..32+8g+7 (hcol(k) = 32*(k/8) + 8g + k%8), so each 16-B load / store instruction
  // covers 64 contiguous bytes of a row
  s16x4 wa[4];  // dgrad operand A_t: row i = r16 <-> column n0 + 32*(t/2) + 8*(i/4) + 4*(t%2) + i%4, k = classes 4g..4g+3
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n = n0 + (t >> 1) * 32 + 8 * (r16 >> 2) + (t & 1) * 4 + (r16 & 3);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int c = 4 * g + q;
      wa[t][q] = (c < p.ldw_rows && n < p.K) ? (short)p.W[(size_t)c * p.ldw + n] : (short)0;
    }
  }
  floatx4 acc2[4];  // dW^T partial: [nt][r] <-> column n0 + 16nt + 4g + r, class r16
#pragma unroll
  for (int t = 0; t < 4; ++t) acc2[t] = floatx4{0.f, 0.f, 0.f, 0.f};
  float cs[16];  // dh column sums over this lane's rows: columns hcol(k)
#pragma unroll
  for (int k = 0; k < 16; ++k) cs[k] = 0.f;
  float dbs[4] = {0.f, 0.f, 0.f, 0.f};  // db partial: classes 4g..4g+3
  const int q = r16 >> 2, pp = r16 & 3;  // tr-read: lane 4q+p addresses row 4g+q, elements 4p..4p+3

  for (int mb = r_begin + wid * 16; mb < r_end; mb += 64 * kHbUnroll) {
    u16x8 hv[kHbUnroll][2];
    uint2 dl[kHbUnroll];
#pragma unroll
    for (int u = 0; u < kHbUnroll; ++u) {
      const int m = mb + u * 64 + r16;
      hv[u][0] = hv[u][1] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
      dl[u] = uint2{0u, 0u};
      if (m < r_end) {
        const bf16_t* hr = p.h + (size_t)m * p.ldh + n0 + 8 * g;
        hv[u][0] = *reinterpret_cast<const u16x8*>(hr);
        hv[u][1] = *reinterpret_cast<const u16x8*>(hr + 32);
        dl[u] = *reinterpret_cast<const uint2*>(p.dlogits + (size_t)m * 16 + 4 * g);
      }
    }
    // stage every block first (h rows of 128 B, dlogits rows of 32 B): one LDS wait per
    // kHbUnroll blocks instead of two per block
    // (16-B chunks of an h row XOR-swizzled by row, 8-B slots of a dlogits row by row / 4: the
    // 16 rows of a store instruction hit distinct banks -- straight 128-B / 32-B rows were an 8-way /
    // 4-way conflict, 12.3 extra LDS cycles per instruction, profiles/r5/pmc_mlp3.txt)
#pragma unroll
    for (int u = 0; u < kHbUnroll; ++u) {
      char* sb = st + u * kSt;
      *reinterpret_cast<u16x8*>(sb + r16 * 128 + ((g ^ (r16 & 7)) << 4)) = hv[u][0];
      *reinterpret_cast<u16x8*>(sb + r16 * 128 + (((4 + g) ^ (r16 & 7)) << 4)) = hv[u][1];
      *reinterpret_cast<uint2*>(sb + kH + r16 * 32 + ((g ^ ((r16 >> 2) & 3)) << 3)) = dl[u];
    }
#pragma unroll
    for (int u = 0; u < kHbUnroll; ++u) {
      const int m = mb + u * 64 + r16;
      // ---- dgrad: lane holds dh[m][n0 + hcol(4t + r)] = d[t][r]
      const s16x4 bl = __builtin_bit_cast(s16x4, dl[u]);
      floatx4 d[4];
#pragma unroll
      for (int t = 0; t < 4; ++t)
        d[t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(wa[t], bl, floatx4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      u16x8 o[2];
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const uint16_t hb = hv[u][k >> 3][k & 7];
        float v = d[k >> 2][k & 3];
        if constexpr (RELU) v = (short)hb > 0 ? v : 0.f;  // bf16 > 0 <=> sign clear and nonzero
        const uint16_t ob = f2bf(v);
        o[k >> 3][k & 7] = ob;
        cs[k] += bf2f(ob);
      }
      if (m < r_end) {
        bf16_t* dst = p.dh + (size_t)m * p.lddh + n0 + 8 * g;
        *reinterpret_cast<u16x8*>(dst) = o[0];
        *reinterpret_cast<u16x8*>(dst + 32) = o[1];
      }
#pragma unroll
      for (int c = 0; c < 4; ++c) dbs[c] += bf2f((uint16_t)((c < 2 ? dl[u].x : dl[u].y) >> (16 * (c & 1))));
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own staging writes landed
    __builtin_amdgcn_wave_barrier();
    // ---- wgrad: the staged blocks read back k-major (k = row) as MFMA operands; the next
    // iteration's staging writes follow these reads in the wave's in-order LDS queue
#pragma unroll
    for (int u = 0; u < kHbUnroll; ++u) {
      const char* sb = st + u * kSt;
      const int row = 4 * g + q;  // (row >> 2) == g
      const bf16x4 bd = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4*)(sb + kH + row * 32 + ((pp ^ g) << 3)));
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const bf16x4 ah = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_b4*)(sb + row * 128 + (((2 * nt + (pp >> 1)) ^ (row & 7)) << 4) + (pp & 1) * 8));
        acc2[nt] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(__builtin_bit_cast(s16x4, ah),
                                                             __builtin_bit_cast(s16x4, bd), acc2[nt], 0, 0, 0);
      }
    }
  }

  // ---- reductions: over the 16 row lanes, then over the 4 waves (LDS), one atomic per output
#pragma unroll
  for (int k = 0; k < 16; ++k)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) cs[k] += __shfl_xor(cs[k], o, 64);
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) dbs[q] += __shfl_xor(dbs[q], o, 64);
  __syncthreads();  // every wave is done with its staging slice
  float* red = reinterpret_cast<float*>(smem);  // [4 waves][64 lanes][17]: 16 dW values, then cs / dbs
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(wid * 64 + lane) * 17 + nt * 4 + r] = acc2[nt][r];
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) t += red[(w * 64 + lane) * 17 + nt * 4 + r];
        const int n = n0 + 16 * nt + 4 * g + r;
        if (r16 < p.nrows_w && n < p.K) atomicAdd(p.dW + (size_t)r16 * p.lddw + n, t);
      }
  }
  __syncthreads();
  // column sums: lanes r16 == 0 hold columns n0 + hcol(k); db: classes 4g + q
  if (r16 == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) red[(wid * 4 + g) * 17 + k] = cs[k];
    red[(wid * 4 + g) * 17 + 16] = 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) red[16 * 17 + (wid * 4 + g) * 4 + q] = dbs[q];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int gg = threadIdx.x >> 4, k = threadIdx.x & 15;
    const int n = n0 + (k >> 3) * 32 + 8 * gg + (k & 7);
    if (p.dbias != nullptr && n < p.K) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) t += red[(w * 4 + gg) * 17 + k];
      atomicAdd(p.dbias + n, t);
    }
  } else if (threadIdx.x < 80 && blockIdx.x == 0 && p.db != nullptr) {
    const int c = threadIdx.x - 64, gg = c >> 2, q = c & 3;
    if (c < p.nrows_w) {
      float t = 0.f;
#pragma unroll
      for (int w = 0; w < 4; ++w) t += red[16 * 17 + (w * 4 + gg) * 4 + q];
      atomicAdd(p.db + c, t);
    }
  }
}

hipError_t head_bwd(const HeadParams& p, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  if (p.ld != 16 || p.dh == nullptr || p.dW == nullptr || p.lddh % 8 != 0 || p.ldh % 8 != 0 || p.K % 64 != 0 ||
      p.ldw_rows > 16 || p.nrows_w > 16 || (p.dgrad_epi != EPI_NONE && p.dgrad_epi != EPI_DRELU))
    return hipErrorInvalidValue;
  const int gx = p.K / 64;
  // ~3 workgroups per CU (the register-bound occupancy; profiles/r5/mlp_head_bwd_grid_ab.jsonl)
  constexpr int target = 768;
  int gy = std::max(1, std::min(256, target / gx));
  int rpw = (p.B + gy - 1) / gy;
  rpw = (rpw + 63) & ~63;
  gy = (p.B + rpw - 1) / rpw;
  const dim3 grid(gx, gy);
  if (p.dgrad_epi == EPI_DRELU) head_bwd_kernel<true><<<grid, 256, 0, s>>>(p, rpw);
  else head_bwd_kernel<false><<<grid, 256, 0, s>>>(p, rpw);
  return hipGetLastError();
}

size_t head_dgrad_ws_floats(int B, int K) { return (size_t)((B + 15) / 16) * K; }

int head_dgrad_max_k() { return kHeadDgradMaxK; }

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
