// Device-side pieces shared by the LDS-DMA convolution kernels -- conv_lds.hip (the gather,
// halo, weight-stationary and ring kernels) and conv_stem.hip (the C = 8 stem kernels): the
// launch arguments (LArgs), per-class row / tap geometry (Geo, KS), the buffer descriptor, the
// raw LDS barrier, the epilogues (bias / ReLU / BN statistics, row-staged stores) and conv_tail;
// plus the host helpers conv_lds.hip defines for both and the stem entry points conv_stem.hip
// defines for conv_lds.hip's dispatch.
#pragma once

#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ldnn_common.h"
#include "ldnn_fastdiv.h"
#include "ldnn_bn_fin.h"
#include "ldnn_gemm_tile.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace convlds {

constexpr uint32_t kOOB = 0x80000000u;      // >= num_records: reads as zero
constexpr int kSlabBytes4 = 16 * 256 * 16;  // one 4-wave workgroup's fp32 accumulators

struct LArgs {
  ConvShape s;
  void* out;
  const float* bias;
  float beta;        // fp32 outputs: out = acc + beta * out
  int M, N;          // GEMM rows / columns
  int nk_all;        // K-tiles of the reduction (largest class)
  int nk_split;      // K-tiles per gridDim.y slice
  int nb;            // fwd: C/64, dgrad: K/64 channel blocks per tap; 0 = wgrad
  int Kd;            // wgrad: NPQ (reduction length)
  int rsc, pq;
  int classes;       // 4 = stride-2 dgrad parity classes (grid.z), else 1
  int tiles_x;       // gridDim.x
  int dn, dp, dq;    // wgrad: 64 = dn*PQ + dp*Q + dq
  int taps_per_tile; // fwd with C < 64: 64 / C
  FastDiv f_pq, f_q, f_c, f_s;
  FastDiv f_p, f_w, f_h;         // row decompositions: fwd (P, Q), dgrad (H, W)
  FastDiv f_cw[2], f_ch[2];      // stride-2 dgrad class rows: (W - pw + 1) / 2, (H - ph + 1) / 2
  float* ws;         // split-K: combine slabs (with cnt) or wgrad partial slabs [split][M][N] (without)
  int* cnt;          // split-K arrival counters of the in-launch combine
  int bn_stats;      // fwd: accumulate + finalize the next BatchNorm's statistics (bn); weight-stationary
                     // dgrad: the backward statistics of the BN whose output's gradient dx is (bn, bnb_*)
  BnFin bn;
  const bf16_t* bnb_x;     // (ws64 dgrad with bn_stats) that BN's input [M][64]
  const uint8_t* bnb_mask; // its ReLU bits [M][8] (nullptr: no ReLU)
  int tap_major;     // fwd / dgrad K-tile order: 0 = channel block fastest, 1 = filter tap fastest
  int f32_rows;      // fp32 outputs (wgrad, split-K slabs) through the row-coalesced LDS epilogue
  int bf16_rows;     // bf16 outputs (fwd y, stride-1 dgrad dx) through the row-coalesced LDS epilogue
  int remap_rows;    // stride-2 dgrad dx (class row remap) through the row-coalesced LDS epilogue
  int xcd_split;     // split-K grids: the tiles of one K slice share an XCD (see split_coords)
  uint64_t* trace;   // XF bit 5 (phase-trace builds): [workgroup][8] s_memrealtime stamps
  int combine_last;  // in-launch split-K: the last K slice sums (splitk_combine_last), else the last arrival
};

// (tile, K slice) of this workgroup.  Default: tile = blockIdx.x, slice = blockIdx.y.  With
// xcd_split the linear workgroup id goes through the XCD remap first, so the gridDim.x tiles
// of one slice -- which read the same activation rows (a wgrad's filter-tap / channel tiles
// over one npq range) -- are dispatched to ONE XCD and share its L2 instead of each of 8
// XCDs fetching those rows from the Infinity Cache / HBM.
// The workgroup's grid coordinates: the hardware's, or virtual ones when two convolutions share
// one launch (conv_pair_kernel: a layer's dgrad and wgrad side by side).
struct VB {
  int x, y, z, gx, gy;
};
__device__ __forceinline__ VB hw_vb() {
  return VB{(int)blockIdx.x, (int)blockIdx.y, (int)blockIdx.z, (int)gridDim.x, (int)gridDim.y};
}

__device__ __forceinline__ void split_coords(const LArgs& a, const VB& vb, int& bx, int& by) {
  bx = vb.x;
  by = vb.y;
  if (a.xcd_split && vb.gy > 1) {
    const int id = xcd_remap(vb.x + vb.y * vb.gx, vb.gx * vb.gy);
    bx = id % vb.gx;
    by = id / vb.gx;
  }
}

// Per-workgroup geometry: which rows its class covers and which taps it sums.
struct Geo {
  int M;                   // GEMM rows of this class
  int rows_h, rows_w;      // row = (n, h2, w2) over rows_h x rows_w
  int hmul, hoff, woff;    // pixel h = hmul*h2 + hoff
  int r0, s0, step, nS;    // taps r = r0 + step*i (< R), s likewise
  int nk;                  // K-tiles of this class
  FastDiv f_rw, f_rh;      // division by rows_w / rows_h
};

__device__ __forceinline__ Geo make_geo(const LArgs& a, bool dgrad, int cls) {
  Geo g;
  const ConvShape& s = a.s;
  g.hmul = 1; g.hoff = 0; g.woff = 0; g.r0 = 0; g.s0 = 0; g.step = 1; g.nS = s.S;
  g.M = a.M;
  g.nk = a.nk_all;
  if (!dgrad) {  // fwd rows = output pixels
    g.rows_h = s.P; g.rows_w = s.Q;
    g.f_rh = a.f_p; g.f_rw = a.f_q;
    return g;
  }
  g.rows_h = s.H; g.rows_w = s.W;
  g.f_rh = a.f_h; g.f_rw = a.f_w;
  if (a.classes == 4) {
    const int ph = cls >> 1, pw = cls & 1;
    g.hmul = 2; g.hoff = ph; g.woff = pw;
    g.rows_h = (s.H - ph + 1) >> 1;
    g.rows_w = (s.W - pw + 1) >> 1;
    g.f_rh = a.f_ch[ph];
    g.f_rw = a.f_cw[pw];
    g.M = s.N * g.rows_h * g.rows_w;
    g.r0 = (ph + s.pad) & 1;
    g.s0 = (pw + s.pad) & 1;
    g.step = 2;
    const int nR = g.r0 < s.R ? (s.R - g.r0 + 1) >> 1 : 0;
    g.nS = g.s0 < s.S ? (s.S - g.s0 + 1) >> 1 : 0;
    g.nk = nR * g.nS * a.nb;
  }
  return g;
}

// Per-K-tile scalar state: tap (r, s) and channel block cb of K-tile kt.
struct KS {
  int kt, r, s, cb;
};

__device__ __forceinline__ KS ks_init(const LArgs& a, const Geo& g, int kt) {
  KS k;
  k.kt = kt;
  if (a.nb > 0 && g.nS > 0 && a.tap_major) {
    const int ntaps = g.nk / a.nb;  // taps of this class
    k.cb = kt / ntaps;
    const int t = kt - k.cb * ntaps;
    k.r = g.r0 + g.step * (t / g.nS);
    k.s = g.s0 + g.step * (t % g.nS);
  } else if (a.nb > 0 && g.nS > 0) {
    k.cb = kt % a.nb;
    const int t = kt / a.nb;
    k.r = g.r0 + g.step * (t / g.nS);
    k.s = g.s0 + g.step * (t % g.nS);
  } else {
    k.cb = k.r = k.s = 0;
  }
  return k;
}

__device__ __forceinline__ void ks_next(const LArgs& a, const Geo& g, KS& k) {
  ++k.kt;
  if (a.tap_major && a.nb > 0) {  // taps fastest: consecutive K-tiles re-read shifted rows of one channel block
    k.s += g.step;
    if (k.s >= a.s.S) {
      k.s = g.s0;
      k.r += g.step;
      if (k.r >= a.s.R) {
        k.r = g.r0;
        ++k.cb;
      }
    }
    return;
  }
  if (++k.cb == a.nb) {
    k.cb = 0;
    k.s += g.step;
    if (k.s >= a.s.S) {
      k.s = g.s0;
      k.r += g.step;
    }
  }
}


struct Rsrc {  // buffer descriptor (a struct: the builtin type cannot be a host-visible parameter)
  __amdgpu_buffer_rsrc_t r;
};

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

__device__ __forceinline__ int tiles_of(const LArgs& a) { return a.tiles_x; }

// LDS byte address of a __shared__ pointer (ds_read asm operands)
__device__ __forceinline__ uint32_t lds_off(const void* p) { return (uint32_t)(uintptr_t)(lds_void*)p; }

// The following training-mode BatchNorm's statistics from this tile's bf16 outputs
// (exactly the values BN reads): per channel sum and sum of squares over the
// tile's valid rows -- 16 row lanes by shuffles, the WM wave rows through LDS --
// then ONE pair of fp32 atomics per channel per tile, into one of bn_ncop
// accumulator copies (tile % kBnCopies: 8x less same-address serialisation; 64 copies
// measured no faster, profiles/r3/bn_copies_ab_r3.txt).  The
// last of the grid's `tiles` workgroups sums the copies and finalizes (mean,
// invstd, running-stat EMA, apply coefficients), so the BN needs no reduce pass.
// (A dgrad's BN backward statistics come from the slab pass or a post pass over dx instead:
// the epilogue form of round 5 cost 11-13 us per dgrad, profiles/r5/conv_bn_bwd_ab.txt.)
template <int WM, int WN>
__device__ __forceinline__ void bn_stats_epilogue(const LArgs& a, const Geo& g, floatx4 (&acc)[4][4], int mbase,
                                                  int n0, int wm, int wn, int lane, int tile, char* smem,
                                                  int lds_floats) {
  constexpr int BN = WN * 64;
  float* red = reinterpret_cast<float*>(smem);  // [WM][BN][2]
  __syncthreads();  // every wave is done with the operand stages
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float s0[4] = {0.f, 0.f, 0.f, 0.f}, s1[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (mbase + i * 16 + (lane & 15) >= g.M) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = bf2f(f2bf(acc[j][i][r]));
        s0[r] += v;
        s1[r] += v * v;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s0[r] += __shfl_xor(s0[r], o, 64);
        s1[r] += __shfl_xor(s1[r], o, 64);
      }
    }
    if ((lane & 15) == 0) {
      const int lc = wn * 64 + j * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        red[(wm * BN + lc + r) * 2] = s0[r];
        red[(wm * BN + lc + r) * 2 + 1] = s1[r];
      }
    }
  }
  __syncthreads();
  float* accc = a.bn.acc + (size_t)(tile % kBnCopies) * 2 * a.N;
  for (int t = threadIdx.x; t < BN; t += blockDim.x) {
    const int c = n0 + t;
    if (c >= a.N) continue;
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int q = 0; q < WM; ++q) {
      s0 += red[(q * BN + t) * 2];
      s1 += red[(q * BN + t) * 2 + 1];
    }
    bn_acc_add(accc + c, s0);
    bn_acc_add(accc + a.N + c, s1);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics have completed
  bn_finalize_last<false, kBnCopies>(a.bn, g.M, a.N, tiles_of(a), red, lds_floats);
}

// Direct epilogue with the class row remap: GEMM row m of a stride-2 dgrad
// class is pixel (n, 2*h2 + hoff, 2*w2 + woff) of dx.
__device__ __forceinline__ void store_remapped(const LArgs& a, const Geo& g, floatx4 (&acc)[4][4], int mbase,
                                               int nbase, int lane) {
  const ConvShape& s = a.s;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = mbase + i * 16 + (lane & 15);
    if (m >= g.M) continue;
    const int t = fdiv(m, g.f_rw), w2 = m - t * g.rows_w, n = fdiv(t, g.f_rh), h2 = t - n * g.rows_h;
    const size_t row = ((size_t)n * s.H + g.hmul * h2 + g.hoff) * s.W + g.hmul * w2 + g.woff;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int c = nbase + j * 16 + 4 * (lane >> 4);
      if (c >= a.N) continue;
      const floatx4 v = acc[j][i];
      *reinterpret_cast<u16x4*>(reinterpret_cast<bf16_t*>(a.out) + row * a.N + c) =
          u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
    }
  }
}

// Row-coalesced fp32 store of a wave's 64 x 64 tile (wgrad outputs, split-K slabs):
// the accumulators go to the wave's 16 KiB LDS slice ([64][64] fp32, 16-B chunks
// XOR-swizzled by row), then 16 lanes write each 256-B row run -- 4 full rows per
// instruction instead of 16 rows x 64 B straight from the MFMA layout.  The caller
// has barriered the operand stages away.  out = acc (+ beta * out).
__device__ __forceinline__ void store_f32_rows(const GemmParams& p, floatx4 (&acc)[4][4], char* wsm, int mbase,
                                               int nbase, int lane) {
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = i * 16 + (lane & 15);
      const int chunk = j * 4 + (lane >> 4);
      *reinterpret_cast<floatx4*>(wsm + row * 256 + ((chunk ^ (row & 15)) << 4)) = acc[j][i];
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes landed (private slice)
  __builtin_amdgcn_wave_barrier();
  const int c = lane & 15;
  const int n = nbase + c * 4;
#pragma unroll 4
  for (int it = 0; it < 16; ++it) {
    const int row = it * 4 + (lane >> 4);
    const int m = mbase + row;
    floatx4 v = *reinterpret_cast<const floatx4*>(wsm + row * 256 + ((c ^ (row & 15)) << 4));
    if (m < p.M && n < p.N) {
      float* o = reinterpret_cast<float*>(p.C) + (size_t)m * p.ldc + n;
      if (p.beta != 0.f) v = v + p.beta * *reinterpret_cast<const floatx4*>(o);
      *reinterpret_cast<floatx4*>(o) = v;
    }
  }
}

// The same staging for bf16 outputs with the bias / ReLU epilogue: 8 lanes write each
// 128-B row run (8 rows per instruction instead of 16 rows x 32 B).  HALVES = 2 stages
// the 64 rows as two 32-row halves (8 KiB per wave) for kernels with less LDS (the
// C = 8 stem's patch kernel).
template <int EPI, int HALVES = 1>
__device__ __forceinline__ void store_bf16_rows(const GemmParams& p, floatx4 (&acc)[4][4], char* wsm, int mbase,
                                                int nbase, int lane) {
  constexpr int RH = 64 / HALVES;  // rows staged per pass
  const int c8 = lane & 7;
  const int n = nbase + c8 * 8;
  const bool nok = n < p.N;
  float bias[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU) {
    if (nok) {
      const floatx4 b0 = *reinterpret_cast<const floatx4*>(p.bias + n);
      const floatx4 b1 = *reinterpret_cast<const floatx4*>(p.bias + n + 4);
      bias[0] = b0[0]; bias[1] = b0[1]; bias[2] = b0[2]; bias[3] = b0[3];
      bias[4] = b1[0]; bias[5] = b1[1]; bias[6] = b1[2]; bias[7] = b1[3];
    }
  }
#pragma unroll
  for (int h = 0; h < HALVES; ++h) {
#pragma unroll
    for (int i = 0; i < 4 / HALVES; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = i * 16 + (lane & 15);
        const int chunk = j * 4 + (lane >> 4);
        *reinterpret_cast<floatx4*>(wsm + row * 256 + ((chunk ^ (row & 15)) << 4)) = acc[j][h * (4 / HALVES) + i];
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes landed (private slice)
    __builtin_amdgcn_wave_barrier();
#pragma unroll 4
    for (int it = 0; it < RH / 8; ++it) {
      const int row = it * 8 + (lane >> 3);
      const int m = mbase + h * RH + row;
      const char* rb = wsm + row * 256;
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(rb + (((2 * c8) ^ (row & 15)) << 4));
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(rb + (((2 * c8 + 1) ^ (row & 15)) << 4));
      if (!(nok && m < p.M)) continue;
      u16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = f2bf(apply_epi<EPI>(q < 4 ? v0[q] : v1[q - 4], bias[q], 0.f));
      *reinterpret_cast<u16x8*>(reinterpret_cast<bf16_t*>(p.C) + (size_t)m * p.ldc + n) = o;
    }
    __builtin_amdgcn_wave_barrier();  // the slice is re-staged by the next half
  }
}

// store_remapped through the wave's LDS slice: each GEMM row (one dx pixel's
// channels) leaves as 128-B runs, 8 lanes a row, instead of 16 rows x 32 B.
__device__ __forceinline__ void store_remapped_rows(const LArgs& a, const Geo& g, floatx4 (&acc)[4][4], char* wsm,
                                                    int mbase, int nbase, int lane) {
  const ConvShape& s = a.s;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = i * 16 + (lane & 15);
      const int chunk = j * 4 + (lane >> 4);
      *reinterpret_cast<floatx4*>(wsm + row * 256 + ((chunk ^ (row & 15)) << 4)) = acc[j][i];
    }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's staging writes landed (private slice)
  __builtin_amdgcn_wave_barrier();
  const int c8 = lane & 7;
  const int c = nbase + c8 * 8;
  const bool cok = c < a.N;
#pragma unroll 4
  for (int it = 0; it < 8; ++it) {
    const int row = it * 8 + (lane >> 3);
    const int m = mbase + row;
    const char* rb = wsm + row * 256;
    const floatx4 v0 = *reinterpret_cast<const floatx4*>(rb + (((2 * c8) ^ (row & 15)) << 4));
    const floatx4 v1 = *reinterpret_cast<const floatx4*>(rb + (((2 * c8 + 1) ^ (row & 15)) << 4));
    if (!(cok && m < g.M)) continue;
    const int t = fdiv(m, g.f_rw), w2 = m - t * g.rows_w, n = fdiv(t, g.f_rh), h2 = t - n * g.rows_h;
    const size_t px = ((size_t)n * s.H + g.hmul * h2 + g.hoff) * s.W + g.hmul * w2 + g.woff;
    u16x8 o;
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = f2bf(q < 4 ? v0[q] : v1[q - 4]);
    *reinterpret_cast<u16x8*>(reinterpret_cast<bf16_t*>(a.out) + px * a.N + c) = o;
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Shared tail of the fwd / dgrad / wgrad kernels: split-K hand-off (in-launch
// combine, fp32 slab, or fp32 atomics), the stride-2 dgrad row remap, the fused
// epilogue and the next BatchNorm's statistics.  smem: the kernel's whole LDS
// (lds_floats floats), free once every wave is past its operand reads.
template <int WM, int WN, int EPI, bool OUT_F32, bool DGRAD>
__device__ __forceinline__ void conv_tail(const LArgs& a, const Geo& g, floatx4 (&acc)[4][4], int m0, int n0, int wm,
                                          int wn, int lane, char* smem, int lds_floats, int bx, int by,
                                          const VB& vb) {
  constexpr int NW = WM * WN;
  const bool combine = a.cnt != nullptr && vb.gy > 1;
  const int mb = m0 + wm * 64, nbase = n0 + wn * 64;
  if (vb.gy > 1) {
    if (combine) {
      lds_barrier();  // every wave is done with the operand stages (the ticket word lives there)
      const int tile = vb.z * a.tiles_x + bx;
      // (phase-trace builds: stamps 4..6 of this workgroup's trace row, see splitk_combine)
      uint64_t* tr = (a.trace != nullptr && threadIdx.x == 0)
                         ? a.trace + 8 * (size_t)(vb.x + vb.gx * (vb.y + vb.gy * vb.z))
                         : nullptr;
      if (a.xcd_split || !a.combine_last) {
        if (!splitk_combine<4, 4, NW * 64>(acc, a.ws, a.cnt, tile, vb.gy, by, smem, tr)) return;
      } else if (!splitk_combine_last<4, 4, NW * 64>(acc, a.ws, a.cnt, tile, vb.gy, by, smem, tr)) {
        return;
      }
    } else if (a.ws != nullptr) {
      // wgrad, and small-M fwd / stride-1 dgrad: this slice's fp32 partial tile into
      // its own slab; a separate chip-wide kernel sums the slabs (slab_sum_kernel /
      // conv_slab_epilogue_kernel with the bias / ReLU epilogue) -- deterministic, no
      // atomics, and no single workgroup re-reading every slice of its tile
      GemmParams p{};
      p.C = a.ws + (size_t)by * a.M * a.N;
      p.M = g.M;
      p.N = a.N;
      p.ldc = a.N;
      if (a.f32_rows && lds_floats >= NW * 4096) {
        lds_barrier();  // every wave is done with the operand stages
        store_f32_rows(p, acc, smem + (size_t)(wm * WN + wn) * 16384, mb, nbase, lane);
        return;
      }
      epilogue<EPI_NONE, true, 4, 4>(p, acc, mb, nbase, lane);
      return;
    } else {
      if constexpr (OUT_F32 && EPI == EPI_NONE) {  // fp32 atomics into the (cleared / accumulated) output
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = nbase + j * 16 + 4 * (lane >> 4);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = mb + i * 16 + (lane & 15);
            if (n < a.N && m < g.M) {
              float* c = reinterpret_cast<float*>(a.out) + (size_t)m * a.N + n;
#pragma unroll
              for (int r = 0; r < 4; ++r) atomicAdd(c + r, acc[j][i][r]);
            }
          }
        }
      }
      return;
    }
  }
  if constexpr (DGRAD && !OUT_F32) {
    if (g.hmul == 2) {
      if (a.remap_rows && lds_floats >= NW * 4096 && !combine) {
        lds_barrier();  // every wave is done with the operand stages
        store_remapped_rows(a, g, acc, smem + (size_t)(wm * WN + wn) * 16384, mb, nbase, lane);
        return;
      }
      store_remapped(a, g, acc, mb, nbase, lane);
      return;
    }
  }
  GemmParams p{};
  p.C = a.out;
  p.M = g.M;
  p.N = a.N;
  p.ldc = a.N;
  p.bias = a.bias;
  p.beta = a.beta;
  if constexpr (OUT_F32 && EPI == EPI_NONE) {
    if (a.f32_rows && lds_floats >= NW * 4096 && !combine) {
      lds_barrier();  // every wave is done with the operand stages
      store_f32_rows(p, acc, smem + (size_t)(wm * WN + wn) * 16384, mb, nbase, lane);
      return;
    }
  }
  if constexpr (!OUT_F32 && (EPI == EPI_NONE || EPI == EPI_BIAS || EPI == EPI_BIAS_RELU)) {
    if (a.bf16_rows && lds_floats >= NW * (a.bf16_rows >= 2 ? 2048 : 4096) && !combine) {
      lds_barrier();  // every wave is done with the operand stages
      if (lds_floats >= NW * 4096)
        store_bf16_rows<EPI>(p, acc, smem + (size_t)(wm * WN + wn) * 16384, mb, nbase, lane);
      else
        store_bf16_rows<EPI, 2>(p, acc, smem + (size_t)(wm * WN + wn) * 8192, mb, nbase, lane);
      if constexpr (EPI == EPI_NONE && !DGRAD) {
        if (a.bn_stats) bn_stats_epilogue<WM, WN>(a, g, acc, mb, n0, wm, wn, lane, bx, smem, lds_floats);
      }
      return;
    }
  }
  epilogue<EPI, OUT_F32, 4, 4>(p, acc, mb, nbase, lane);
  if constexpr (!OUT_F32 && EPI == EPI_NONE && !DGRAD) {
    if (a.bn_stats) bn_stats_epilogue<WM, WN>(a, g, acc, mb, n0, wm, wn, lane, bx, smem, lds_floats);
  }
}


// ---- host helpers (conv_lds.hip)
int env_int(const char* name, int dflt);
int ws_env();       // LDNN_CONV_WS: the weight-stationary kernels (ws64, patch_ws, s2d forward)
int cu_count();
int conv_xf_env();  // LDNN_CONV_XF experiment bits (32: phase trace)
LArgs base_args(const ConvShape& s);

}  // namespace convlds

// ---- the stem paths (conv_stem.hip)
bool stem_s2d_ok(const ConvShape& s);            // the space-to-depth stem wgrad takes this shape
size_t stem_s2d_ws_bytes(const ConvShape& s);    // its workspace (slabs, sum, packed image)
// forward on the packed image (stem_s2d_fwd_ok): packs x into xs and runs conv_s2d_ws_kernel
hipError_t stem_s2d_fwd(convlds::LArgs a, const uint16_t* x, const uint16_t* w, uint16_t* xs, hipStream_t st);
// weight gradient (stem_s2d_ok, ws of stem_s2d_ws_bytes); xs: the forward's packed image, or nullptr
hipError_t stem_s2d_wgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* x, float* dw, float beta,
                          hipStream_t st, float* ws, const uint16_t* xs);
bool patch_ok(const ConvShape& s);               // the patch kernels take this C = 8 forward
hipError_t launch_patch(convlds::LArgs a, int epi, const bf16_t* x, size_t bx, const bf16_t* w, hipStream_t st);

}  // namespace ldnn
