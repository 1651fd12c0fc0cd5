// The C = 8 stem convolutions (split out of conv_lds.hip in round 6; they run on its LDS-DMA
// machinery, ldnn_conv_lds.h):
//   * conv_s2d_ws_kernel / stem_s2d_wgrad_kernel: the ResNet-type 7x7 / 2 / pad-3 stem with <= 4
//     data channels, forward and weight gradient on the 2x2 space-to-depth image (a 4x4 stride-1
//     conv over 16 channels: no gather, no masks);
//   * conv_patch_kernel / conv_patch_ws_kernel: other C = 8 stems (3x3 / 5x5 / 7x7, stride 1 or 2),
//     one DMA of the tile's whole input patch, taps read from it in LDS.
// (conv.hip keeps the MFMA kernels for the C = 8, K <= 16 LeNet-5 convs.)
#include "ldnn_conv_lds.h"

namespace ldnn {

namespace convlds {

// ---- stem forward on the space-to-depth image (the mapping of stem_s2d_wgrad_kernel below) ----
//   y[n][p][q][k] = sum_{a,b < 4} w'[k][a][b][.] . xs[n][p + a][q + b][.],  16 s2d channels (32 B)
// per pixel, w'[k][a][b][(dh, dw, c)] = w[k][2a + dh - 1][2b + dw - 1][c]: K = 256 (8 MFMA k-steps)
// instead of the 7x7x8 patch kernel's 13, and the input of a 256-pixel tile is <= kRows whole s2d rows,
// ONE contiguous run of bytes (a linear DMA, no gather).  Persistent: one 4-wave workgroup per CU keeps
// w' in registers (8 k-steps x 4 filter tiles, gathered from w once), walks a contiguous run of
// 256-pixel tiles through a 3-buffer ring (the DMA of tiles t+1 and t+2 in flight behind tile t's
// MFMAs: the patch kernels' loops are bound by the DMA round trip), stages the outputs through LDS
// for whole-row stores and keeps the next BN's statistics in registers.  Needs P*Q % 256 == 0 (a
// tile never spans two images) and rows * Ws * 32 <= kBuf (stem_s2d_fwd_ok).
namespace s2dfwd {
constexpr int kPieces = 28, kBuf = kPieces * 1024, kNB = 3;
}
__global__ __launch_bounds__(256, 1) void conv_s2d_ws_kernel(LArgs a, const bf16_t* pxs, uint32_t bytes_xs, int Hs,
                                                             int Ws, const bf16_t* pw) {
  using namespace s2dfwd;
  constexpr int BM = 256, NW = 4, PPW = kPieces / NW, KS = 8;
  constexpr int kOutPitch = 144, kOutWave = 64 * kOutPitch;
  constexpr int LDS = kNB * kBuf + NW * kOutWave + 16;
  static_assert(PPW * NW == kPieces && LDS <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  const ConvShape& sh = a.s;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  char* const ostage = smem + kNB * kBuf + wid * kOutWave;
  const int PQ = sh.P * sh.Q;
  const int T = a.M / BM;
  const int t0 = (int)((int64_t)blockIdx.x * T / gridDim.x);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * T / gridDim.x);
  const int g4 = lane >> 4;   // k-elements 8 g4 .. 8 g4 + 7 of a step: tap 2k + (g4 >> 1), channels 8 (g4 & 1) ..

  // w' fragments of every k-step (filter j*16 + (lane & 15)): registers for the launch, all loads in flight
  bf16x8 fb[KS][4];
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = 2 * k + (g4 >> 1), ta = t >> 2, tb = t & 3;
      const bf16_t* wn = pw + (size_t)(j * 16 + (lane & 15)) * a.rsc;
      u16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const int cc = (g4 & 1) * 8 + e, d = cc >> 2, c = cc & 3;
        const int r = 2 * ta + (d >> 1) - 1, s = 2 * tb + (d & 1) - 1;
        v[e] = (r >= 0 && s >= 0) ? reinterpret_cast<const uint16_t*>(wn)[(r * 7 + s) * 8 + c] : (uint16_t)0;
      }
      fb[k][j] = __builtin_bit_cast(bf16x8, v);
    }
  Rsrc rx;
  rx.r = __builtin_amdgcn_make_buffer_rsrc((void*)pxs, (short)0, (int)bytes_xs, 0x00020000);
  // tile t: s2d rows (n, p_lo ..) are contiguous from ((n Hs + p_lo) Ws) * 32 B; bytes past the
  // buffer read as zeros, bytes of rows past the tile's are loaded and never read
  auto dma = [&](int t, int b) {
    const int m0 = t * BM, n_img = m0 / PQ, p_lo = (m0 - n_img * PQ) / sh.Q;
    const uint32_t base = (uint32_t)(n_img * Hs + p_lo) * (uint32_t)Ws * 32u;
    char* const dst = smem + b * kBuf;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const int pc = q * NW + wid;
      const uint32_t o = base + (uint32_t)pc * 1024u + (uint32_t)lane * 16u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx.r, (lds_void*)(dst + pc * 1024), 16, o < bytes_xs ? (int)o : (int)kOOB,
                                               0, 0, 0);
    }
  };
  if (t0 < t1) {
    dma(t0, 0);
    if (t0 + 1 < t1) dma(t0 + 1, 1);
  }
  // this lane's tap offset (bytes) per k-step
  uint32_t toff[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int t = 2 * k + (g4 >> 1);
    toff[k] = (uint32_t)(((t >> 2) * Ws + (t & 3)) * 32 + (g4 & 1) * 16);
  }
  if (t0 < t1) {
    if (t0 + 1 < t1) wait_vm<PPW>();  // tile t0's pieces landed (and the w' loads, issued before them)
    else wait_vm<0>();
  }
  float bs0[4][4], bs1[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bs0[j][r] = bs1[j][r] = 0.f;
  bf16_t* const out = reinterpret_cast<bf16_t*>(a.out);
  for (int t = t0; t < t1; ++t) {
    const int m0 = t * BM, n_img = m0 / PQ, mi0 = m0 - n_img * PQ, p_lo = mi0 / sh.Q;
    lds_barrier();  // every wave waited for its own pieces of tile t; every wave is done with tile t-1's buffer
    if (t + 2 < t1) dma(t + 2, (t + 2 - t0) % kNB);
    const uint32_t patch = lds_off(smem + ((t - t0) % kNB) * kBuf);
    uint32_t base[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int mi = mi0 + wid * 64 + i * 16 + (lane & 15);
      const int p = fdiv(mi, a.f_q), q = mi - p * sh.Q;
      base[i] = patch + (uint32_t)(((p - p_lo) * Ws + q) * 32);
    }
    auto read_step = [&](int k, bf16x8 (&f)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t ad = base[i] + toff[k];
        asm volatile("ds_read_b128 %0, %1" : "=v"(f[i]) : "v"(ad));
      }
    };
    floatx4 acc[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa[3][4];
    read_step(0, fa[0]);
    read_step(1, fa[1]);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      bf16x8 (&f)[4] = fa[k % 3];
      if (k + 2 < KS) read_step(k + 2, fa[(k + 2) % 3]);
      if (k + 2 < KS) asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
      else if (k + 1 < KS) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[k][j], f[i], acc[j][i], 0, 0, 0);
    }
    // tile t+1's pieces (issued a tile ago; only tile t+2's were issued after them)
    if (t + 1 < t1) {
      if (t + 2 < t1) wait_vm<PPW>();
      else wait_vm<0>();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = i * 16 + (lane & 15);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = j * 16 + 4 * (lane >> 4);
        const floatx4 v = acc[j][i];
        const u16x4 o = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
        *reinterpret_cast<u16x4*>(ostage + rl * kOutPitch + c * 2) = o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float bv = bf2f(o[r]);
          bs0[j][r] += bv;
          bs1[j][r] += bv * bv;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (a wave's LDS operations run in order)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int rl = q * 8 + (lane >> 3);
      const u32x4 v = *reinterpret_cast<const u32x4*>(ostage + rl * kOutPitch + (lane & 7) * 16);
      *reinterpret_cast<u32x4*>(out + (size_t)(m0 + wid * 64 + rl) * 64 + (lane & 7) * 8) = v;
    }
  }
  if (a.bn_stats) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          bs0[j][r] += __shfl_xor(bs0[j][r], o, 64);
          bs1[j][r] += __shfl_xor(bs1[j][r], o, 64);
        }
    float* red = reinterpret_cast<float*>(smem);  // [4][64][2]
    __syncthreads();
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = j * 16 + 4 * (lane >> 4) + r;
          red[(wid * 64 + c) * 2] = bs0[j][r];
          red[(wid * 64 + c) * 2 + 1] = bs1[j][r];
        }
    }
    __syncthreads();
    float* accc = a.bn.acc + (size_t)(blockIdx.x % kBnCopies) * 2 * 64;
    if (threadIdx.x < 64) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        s0 += red[(q * 64 + threadIdx.x) * 2];
        s1 += red[(q * 64 + threadIdx.x) * 2 + 1];
      }
      bn_acc_add(accc + threadIdx.x, s0);
      bn_acc_add(accc + 64 + threadIdx.x, s1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics have completed
    bn_finalize_last<false, kBnCopies>(a.bn, a.M, 64, gridDim.x, red, LDS / 4);
  }
}

// ---- stem wgrad via space-to-depth (7x7 stride-2 pad-3, C = 8 with <= 4 real channels) ----
// The split-K wgrad gathers the C = 8 stem's activation as one 16-B pixel per (tap, pixel)
// element: 40 KiB of 16-B pieces per K-tile, ~300 TFLOP/s, the largest kernel of the
// ResNet-18 b64 step (131 us).  Rewritten on the 2x2 space-to-depth image
//   xs[n][i][j][(dh*2 + dw)*4 + c] = x[n][2(i-2) + dh][2(j-2) + dw][c]   (zero outside),
// the stem is a 4x4 stride-1 unpadded conv with 16 channels:
//   y[p][q] = sum_{a,b<4} w'[a][b][.] . xs[p+a][q+b][.],  w'[a][b][dh,dw,c] = w[2a+dh-1][2b+dw-1][c]
// so its weight gradient dW'[k][a][b][16] = sum_pq dy[p][q][k] xs[p+a][q+b][.] needs no
// gather and no masks: per K-step (32 output pixels of one row) a workgroup DMAs the dy rows
// (4 KiB) and 4 activation row segments of 36 s2d pixels (4 x 1.1 KiB), wave a multiplies
// taps (a, 0..3) -- 16 MFMAs; 256 x 64 fp32 partial blocks per slice, summed and scattered
// back to dW[k][r][s][c] by stem_s2d_sum_kernel.
namespace s2d {
constexpr int kDy = 32 * 128, kSeg = 2048, kStage = kDy + 4 * kSeg;  // 12 KiB per stage
constexpr int kStages = 4;  // K-steps t+1 .. t+2 in flight while t is multiplied (t+3 issued after its barrier)
}

__global__ __launch_bounds__(256) void stem_s2d_pack_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ xs,
                                                            int N, int H, int W, int Hs, int Ws) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // s2d pixel
  if (i >= (int64_t)N * Hs * Ws) return;
  const int jj = (int)(i % Ws);
  const int64_t t = i / Ws;
  const int ii = (int)(t % Hs), n = (int)(t / Hs);
  u16x8 o[2];
#pragma unroll
  for (int d = 0; d < 4; ++d) {  // d = dh*2 + dw
    const int h = 2 * (ii - 2) + (d >> 1), w = 2 * (jj - 2) + (d & 1);
    u16x4 v = {0, 0, 0, 0};
    if (h >= 0 && h < H && w >= 0 && w < W)
      v = *reinterpret_cast<const u16x4*>(x + (((size_t)n * H + h) * W + w) * 8);  // channels 0..3
#pragma unroll
    for (int c = 0; c < 4; ++c) o[d >> 1][(d & 1) * 4 + c] = v[c];
  }
  u16x8* dst = reinterpret_cast<u16x8*>(xs + i * 16);
  dst[0] = o[0];
  dst[1] = o[1];
}

struct S2dArgs {
  int N, P, Q, Hs, Ws, K;   // output P x Q, s2d image Hs x Ws (= P + 3, Q + 3), filters K (= 64)
  int nchunk, steps, steps_per;  // 32-pixel chunks per output row; total K-steps; per slice
  float* slab;              // [slices][64][256]
};

__global__ __launch_bounds__(256, 3) void stem_s2d_wgrad_kernel(S2dArgs a, const bf16_t* pdy, uint32_t bytes_dy,
                                                                const bf16_t* pxs, uint32_t bytes_xs) {
  using namespace s2d;
  __shared__ __attribute__((aligned(1024))) char smem[kStages * kStage];  // 48 KiB
  typedef __attribute__((address_space(3))) bf16x4 lds_b4;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // = filter-row tap a
  const int g = lane >> 4, r16 = lane & 15, qq = r16 >> 2, pp = r16 & 3;
  const int st0 = blockIdx.x * a.steps_per;
  const int nst = min(a.steps - st0, a.steps_per);
  floatx4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
  if (nst > 0) {
    Rsrc rdy, rxs;
    rdy.r = __builtin_amdgcn_make_buffer_rsrc((void*)pdy, (short)0, (int)bytes_dy, 0x00020000);
    rxs.r = __builtin_amdgcn_make_buffer_rsrc((void*)pxs, (short)0, (int)bytes_xs, 0x00020000);
    // K-step st = (n * P + p) * nchunk + chunk: dy rows of pixels (n, p, 32 chunk ..), the 4 s2d
    // row segments (n, p + a, 32 chunk .. + 35); wave `wid` DMAs dy piece wid and segment a = wid
    auto load = [&](int st, char* dst) {
      const int chunk = st % a.nchunk, row = st / a.nchunk;  // row = n * P + p
      const int p = row % a.P, n = row / a.P;
      const int q0 = chunk * 32;
      {
        const int j = wid * 8 + (lane >> 3);
        const int k = (lane & 7) ^ (j & 7);
        const int o = q0 + j < a.Q ? (int)(((uint32_t)(row * a.Q + q0 + j) * (uint32_t)a.K + (uint32_t)(k * 8)) * 2u)
                                   : (int)kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rdy.r, (lds_void*)(dst + wid * 1024), 16, o, 0, 0, 0);
      }
      const uint32_t pix0 = ((uint32_t)(n * a.Hs + p + wid) * (uint32_t)a.Ws + (uint32_t)q0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // s2d pixels q0 .. q0 + 34 x 32 B (the taps read 35): the second
        // piece's lanes past pixel 34 are out of range (no memory traffic; the per-CU fill rate
        // bounds this kernel)
        const int px = h * 32 + (lane >> 1);
        const uint32_t o = (pix0 + (uint32_t)px) * 32u + (uint32_t)(lane & 1) * 16u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rxs.r, (lds_void*)(dst + kDy + wid * kSeg + h * 1024), 16,
                                                 px < 35 ? (int)o : (int)kOOB, 0, 0, 0);
      }
    };
    // three DMA instructions per wave per K-step; steps 0..2 in the prologue, step t+3 after
    // the barrier of step t (into the stage of step t-1), a counted wait keeps two in flight
#pragma unroll
    for (int t = 0; t < kStages - 1; ++t)
      if (t < nst) load(st0 + t, smem + t * kStage);
    for (int t = 0; t < nst; ++t) {
      const int ahead = min(nst, t + kStages - 1) - t - 1;  // steps issued after t
      if (ahead >= 2) wait_vm<6>();
      else if (ahead == 1) wait_vm<3>();
      else wait_vm<0>();
      lds_barrier();  // publishes step t; every wave is done with step t-1's stage
      if (t + kStages - 1 < nst) load(st0 + t + kStages - 1, smem + ((t + kStages - 1) % kStages) * kStage);
      const char* stg = smem + (t % kStages) * kStage;
      const int rl = 8 * g + qq;
      bf16x8 fa[4];  // dy: rows = filters 16i + r16, k = the step's 32 pixels
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int c = 2 * i + (pp >> 1);
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_b4*)(stg + rl * 128 + ((c ^ (rl & 7)) << 4) + 8 * (pp & 1)));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_b4*)(stg + (rl + 4) * 128 + ((c ^ ((rl + 4) & 7)) << 4) + 8 * (pp & 1)));
        fa[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
      }
      const char* seg = stg + kDy + wid * kSeg;
#pragma unroll
      for (int b = 0; b < 4; ++b) {  // tap (a = wid, b): s2d pixel q + b, 16 channels
        const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4*)(seg + (rl + b) * 32 + 8 * pp));
        const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_b4*)(seg + (rl + 4 + b) * 32 + 8 * pp));
        const bf16x8 fb = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[b][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa[i], acc[b][i], 0, 0, 0);
      }
    }
  }
  // lane holds dW'[filter 16i + r16][tap (wid, b) * 16 + 4g + 0..3]
  float* o = a.slab + (size_t)blockIdx.x * 64 * 256;
#pragma unroll
  for (int b = 0; b < 4; ++b)
#pragma unroll
    for (int i = 0; i < 4; ++i)
      *reinterpret_cast<floatx4*>(o + (size_t)(16 * i + r16) * 256 + (wid * 4 + b) * 16 + 4 * g) = acc[b][i];
}

// dW[k][r][s][c] (7 x 7 x 8) = sum over slices of dW'[k][a][b][(dh,dw,c)], r = 2a+dh-1, s = 2b+dw-1
// (channels 4..7 of the padded C = 8 carry no activation: their gradient is 0) (+ beta * dW)
__global__ __launch_bounds__(256) void stem_s2d_sum_kernel(const float* __restrict__ slab, float* __restrict__ dw,
                                                           int slices, float beta) {
  const int e = blockIdx.x * 256 + threadIdx.x;  // dW element
  if (e >= 64 * 49 * 8) return;
  const int c = e & 7, rs = (e >> 3) % 49, k = e / (49 * 8);
  float v = 0.f;
  if (c < 4) {
    const int r = rs / 7, sx = rs % 7;
    const int aa = (r + 1) >> 1, dh = (r + 1) & 1, bb = (sx + 1) >> 1, dwv = (sx + 1) & 1;
    const int j = (aa * 4 + bb) * 16 + (dh * 2 + dwv) * 4 + c;
    const float* p = slab + (size_t)k * 256 + j;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int sl = 0;
    for (; sl + 3 < slices; sl += 4) {
      s0 += p[(size_t)sl * 64 * 256];
      s1 += p[(size_t)(sl + 1) * 64 * 256];
      s2 += p[(size_t)(sl + 2) * 64 * 256];
      s3 += p[(size_t)(sl + 3) * 64 * 256];
    }
    for (; sl < slices; ++sl) s0 += p[(size_t)sl * 64 * 256];
    v = (s0 + s1) + (s2 + s3);
  }
  dw[e] = beta != 0.f ? v + beta * dw[e] : v;
}


// ---- patch path: small-C stems (C = 8: 3 / 1 real channels) -------------------
// FwdASmallC gathers one 16-B (tap, 8-channel) chunk per lane per tap: every input
// pixel crosses the L1 / texture path once per filter tap that covers it (49x for
// the 7x7 ResNet stem, ~12x per output at stride 2), each chunk its own address --
// the stem ran at ~75 TFLOP/s (profiles/).  Here a 256-pixel output tile (one
// image, P*Q % 256 == 0) DMAs its whole input patch ONCE: input rows
// stride*p_lo - pad ... , every column -pad .. W+pad-1, 16 B per pixel, zero-filled
// outside the image by the buffer range check.  The A fragment of tap t for output
// pixel (p, q) is the 16-B patch cell (stride*(p - p_lo) + r, stride*q + s): one
// ds_read_b128 at a per-lane base plus a per-(k-step, lane-group) tap offset.
// B (the [K][R*S*8] weights, a few tens of KB, L2-resident) is read straight from
// global memory into registers, one k-step ahead.  4 waves x 64 output pixels x
// 64 filters, v_mfma_f32_16x16x32_bf16 (a k-step = 4 taps x 8 channels).
constexpr int kPatchBytes = 48 * 1024;

template <int KS, int STR, int EPI>
__global__ __launch_bounds__(256, 2) void conv_patch_kernel(LArgs a, const bf16_t* px, uint32_t bytes_x,
                                                            const bf16_t* pw) {
  constexpr int WM = 4, WN = 1, BM = 256, BN = 64;
  __shared__ __attribute__((aligned(1024))) char smem[kPatchBytes];
  const ConvShape& sh = a.s;
  const Geo g = make_geo(a, false, (int)blockIdx.z);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid, wn = 0;
  int m0, n0;
  tile_coords(g.M, a.N, BM, BN, m0, n0);
  const int PQ = sh.P * sh.Q;
  const int n_img = m0 / PQ, mi0 = m0 - n_img * PQ;  // tiles never straddle images (PQ % 256 == 0)
  const int p_lo = mi0 / sh.Q;
  const int PW = sh.W + 2 * sh.pad;                   // patch columns
  const int PH = ((mi0 + BM - 1) / sh.Q - p_lo) * STR + sh.R;
  const int cells = PH * PW;

  // ---- patch DMA: cell e = (i, j) -> input (STR*p_lo - pad + i, j - pad)
  {
    Rsrc rx;
    rx.r = __builtin_amdgcn_make_buffer_rsrc((void*)px, (short)0, (int)bytes_x, 0x00020000);
    const int ih0 = STR * p_lo - sh.pad;
    const int npieces = (cells + 63) >> 6;
    for (int pc = wid; pc < npieces; pc += 4) {
      const int e = pc * 64 + lane;
      const int i = fdiv(e, a.f_w), j = e - i * PW;   // f_w: division by PW (host)
      const int ih = ih0 + i, iw = j - sh.pad;
      const bool ok = e < cells && (unsigned)ih < (unsigned)sh.H && (unsigned)iw < (unsigned)sh.W;
      const int o = ok ? (int)((((unsigned)n_img * sh.H + ih) * (unsigned)sh.W + iw) * 16u) : (int)kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx.r, (lds_void*)(smem + pc * 1024), 16, o, 0, 0, 0);
    }
  }
  // ---- per-lane geometry: patch cell of tap (0, 0) for each of the wave's 4 row tiles,
  // and this lane group's tap offsets for each k-step (-1: a padding tap past R*S)
  int base[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int mi = mi0 + wm * 64 + i * 16 + (lane & 15);
    const int p = mi / sh.Q, q = mi - p * sh.Q;
    base[i] = (STR * (p - p_lo)) * PW + STR * q;
  }
  int toff[KS];
  const int RS = sh.R * sh.S;
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int t = k * 4 + (lane >> 4);
    const int r = t / sh.S;
    toff[k] = t < RS ? r * PW + (t - r * sh.S) : -1;
  }
  // B fragment of k-step k, filter tile j: filter n0 + j*16 + (lane & 15), k = 8 * tap
  const int rsc = a.rsc;
  auto bfrag = [&](int k, int j) -> bf16x8 {
    const int t = k * 4 + (lane >> 4);
    const int n = n0 + j * 16 + (lane & 15);
    if (t >= RS || n >= a.N) return bf16x8{};
    return *reinterpret_cast<const bf16x8*>(pw + (size_t)n * rsc + t * 8);
  };

  floatx4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
  bf16x8 fb[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) fb[0][j] = bfrag(0, j);
  wait_vm<0>();
  lds_barrier();  // the patch landed
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    if (k + 1 < KS) {
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[(k + 1) & 1][j] = bfrag(k + 1, j);
    }
    bf16x8 fa[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cell = base[i] + toff[k];
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(smem + (toff[k] >= 0 ? cell : 0) * 16);
      fa[i] = toff[k] >= 0 ? v : bf16x8{};
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[k & 1][j], fa[i], acc[j][i], 0, 0, 0);
  }
  conv_tail<WM, WN, EPI, false, false>(a, g, acc, m0, n0, wm, wn, lane, smem, kPatchBytes / 4, blockIdx.x,
                                       blockIdx.y, hw_vb());
}

// Persistent weight-stationary variant of conv_patch_kernel for 64-filter stems (the ResNet-18
// 7x7 / 2 stem: 384 us of the b256 step, ~15 us per 256-pixel tile-pair per CU, its B fragments
// streamed from L2 one k-step ahead).  One 4-wave workgroup per CU keeps the whole [64][R*S*8]
// weight matrix in registers (each wave: 64 rows x all 64 filters, KS x 4 fragments), walks a
// contiguous run of 256-pixel tiles, DMAs each tile's input patch into a double buffer one tile
// ahead (a fixed 48 pieces per tile: rows below the patch load harmlessly), and reads the A
// fragments two k-steps ahead (asm + counted lgkmcnt, as conv_ws64_kernel).  Padding taps
// (t >= R*S) read cell 0: their weights are zero.  The next BN's statistics stay in registers
// over all tiles.  EPI_NONE, K = 64.
__device__ __forceinline__ int wid_stage_offset(int wid, int bytes) { return wid * bytes; }

template <int KS, int STR, int XF = 0>
__global__ __launch_bounds__(256, 1) void conv_patch_ws_kernel(LArgs a, const bf16_t* px, uint32_t bytes_x,
                                                               const bf16_t* pw) {
  constexpr int BM = 256, NW = 4;
  constexpr int PIECES = kPatchBytes / 1024, PPW = PIECES / NW;
  static_assert(PPW * NW == PIECES && KS >= 3, "patch pieces / k-steps");
  // output staging: each wave's 64 rows x 128 B at a 144-B pitch, re-read row-wise so the stores
  // are whole 128-B rows (16 B per lane) instead of 8-B pieces of 16 rows per instruction
  constexpr int kOutPitch = 144, kOutWave = 64 * kOutPitch;
  constexpr int LDS = 2 * kPatchBytes + NW * kOutWave + 16;
  static_assert(LDS <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  char* const ostage = smem + 2 * kPatchBytes + wid_stage_offset(threadIdx.x >> 6, kOutWave);
  const ConvShape& sh = a.s;
  const Geo g = make_geo(a, false, (int)blockIdx.z);
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int PQ = sh.P * sh.Q, PW = sh.W + 2 * sh.pad, RS = sh.R * sh.S;
  const int T = g.M / BM;
  const int t0 = (int)((int64_t)blockIdx.x * T / gridDim.x);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * T / gridDim.x);
  uint64_t* trace = nullptr;
  if constexpr ((XF & 32) != 0) {
    if (threadIdx.x == 0 && a.trace != nullptr) {
      trace = a.trace + 8 * (size_t)blockIdx.x;
      trace[0] = __builtin_amdgcn_s_memrealtime();
    }
  }

  Rsrc rx;
  rx.r = __builtin_amdgcn_make_buffer_rsrc((void*)px, (short)0, (int)bytes_x, 0x00020000);
  // patch of tile t into buffer b: cell e = (i, j) -> input (STR*p_lo - pad + i, j - pad)
  auto dma = [&](int t, int b) {
    const int m0 = t * BM, n_img = m0 / PQ, p_lo = (m0 - n_img * PQ) / sh.Q;
    const int ih0 = STR * p_lo - sh.pad;
    char* const dst = smem + b * kPatchBytes;
#pragma unroll
    for (int q = 0; q < PPW; ++q) {
      const int pc = q * NW + wid;
      const int e = pc * 64 + lane;
      const int i = fdiv(e, a.f_w), j = e - i * PW;
      const int ih = ih0 + i, iw = j - sh.pad;
      const bool ok = (unsigned)ih < (unsigned)sh.H && (unsigned)iw < (unsigned)sh.W;
      const int o = ok ? (int)((((unsigned)n_img * sh.H + ih) * (unsigned)sh.W + iw) * 16u) : (int)kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rx.r, (lds_void*)(dst + pc * 1024), 16, o, 0, 0, 0);
    }
  };
  if (t0 < t1) {
    dma(t0, 0);
    if (t0 + 1 < t1) dma(t0 + 1, 1);
  }
  // B fragments of every k-step (filter j*16 + (lane & 15), taps 4k + lane/16): registers for the launch
  bf16x8 fb[KS][4];
#pragma unroll
  for (int k = 0; k < KS; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = k * 4 + (lane >> 4);
      fb[k][j] = t < RS ? *reinterpret_cast<const bf16x8*>(pw + (size_t)(j * 16 + (lane & 15)) * a.rsc + t * 8)
                        : bf16x8{};
    }
  // this lane group's tap offset (in patch cells) per k-step; padding taps read cell 0 (zero weights)
  int toff[KS];
#pragma unroll
  for (int k = 0; k < KS; ++k) {
    const int t = k * 4 + (lane >> 4);
    const int r = t / sh.S;
    toff[k] = t < RS ? r * PW + (t - r * sh.S) : 0;
  }
  if (t0 < t1) {
    if (t0 + 1 < t1) wait_vm<PPW>();  // tile t0's patch landed (loads retire in order)
    else wait_vm<0>();
  }
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[1] = __builtin_amdgcn_s_memrealtime();
  }
  float bs0[4][4], bs1[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bs0[j][r] = bs1[j][r] = 0.f;
  bf16_t* const out = reinterpret_cast<bf16_t*>(a.out);
  for (int t = t0; t < t1; ++t) {
    const int m0 = t * BM, n_img = m0 / PQ, mi0 = m0 - n_img * PQ, p_lo = mi0 / sh.Q;
    const uint32_t patch = lds_off(smem + ((t - t0) & 1) * kPatchBytes);
    uint32_t base[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int mi = mi0 + wid * 64 + i * 16 + (lane & 15);
      const int p = fdiv(mi, a.f_q), q = mi - p * sh.Q;
      base[i] = patch + (uint32_t)((STR * (p - p_lo)) * PW + STR * q) * 16u;
    }
    auto read_step = [&](int k, bf16x8 (&f)[4]) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t ad = base[i] + (uint32_t)toff[k] * 16u;
        asm volatile("ds_read_b128 %0, %1" : "=v"(f[i]) : "v"(ad));
      }
    };
    floatx4 acc[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
    lds_barrier();  // every wave waited for its own pieces of tile t: the whole patch is visible
    bf16x8 fa[3][4];
    read_step(0, fa[0]);
    read_step(1, fa[1]);
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      bf16x8 (&f)[4] = fa[k % 3];
      if (k + 2 < KS) read_step(k + 2, fa[(k + 2) % 3]);
      if (k + 2 < KS) asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
      else if (k + 1 < KS) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[k][j], f[i], acc[j][i], 0, 0, 0);
    }
    lds_barrier();  // every wave is done reading this buffer
    if (t + 2 < t1) dma(t + 2, (t - t0) & 1);
    if (t + 1 < t1) {  // tile t+1's patch (issued a tile ago; see conv_ws64_kernel for why vmcnt(PPW) holds)
      if (t + 2 < t1) wait_vm<PPW>();
      else wait_vm<0>();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = i * 16 + (lane & 15);   // this wave's row
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = j * 16 + 4 * (lane >> 4);
        const floatx4 v = acc[j][i];
        const u16x4 o = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
        *reinterpret_cast<u16x4*>(ostage + rl * kOutPitch + c * 2) = o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float bv = bf2f(o[r]);
          bs0[j][r] += bv;
          bs1[j][r] += bv * bv;
        }
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (a wave's LDS operations run in order)
#pragma unroll
    for (int q = 0; q < 8; ++q) {   // 8 rows x 8 lanes x 16 B per store
      const int rl = q * 8 + (lane >> 3);
      const u32x4 v = *reinterpret_cast<const u32x4*>(ostage + rl * kOutPitch + (lane & 7) * 16);
      *reinterpret_cast<u32x4*>(out + (size_t)(m0 + wid * 64 + rl) * 64 + (lane & 7) * 8) = v;
    }
  }
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[2] = __builtin_amdgcn_s_memrealtime();
  }
  if (a.bn_stats) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          bs0[j][r] += __shfl_xor(bs0[j][r], o, 64);
          bs1[j][r] += __shfl_xor(bs1[j][r], o, 64);
        }
    float* red = reinterpret_cast<float*>(smem);  // [4][64][2]
    __syncthreads();
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = j * 16 + 4 * (lane >> 4) + r;
          red[(wid * 64 + c) * 2] = bs0[j][r];
          red[(wid * 64 + c) * 2 + 1] = bs1[j][r];
        }
    }
    __syncthreads();
    float* accc = a.bn.acc + (size_t)(blockIdx.x % kBnCopies) * 2 * 64;
    if (threadIdx.x < 64) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int q = 0; q < NW; ++q) {
        s0 += red[(q * 64 + threadIdx.x) * 2];
        s1 += red[(q * 64 + threadIdx.x) * 2 + 1];
      }
      bn_acc_add(accc + threadIdx.x, s0);
      bn_acc_add(accc + 64 + threadIdx.x, s1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics have completed
    bn_finalize_last<false, kBnCopies>(a.bn, g.M, 64, gridDim.x, red, LDS / 4);
  }
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[3] = __builtin_amdgcn_s_memrealtime();
  }
}

}  // namespace convlds

using namespace convlds;

// Space-to-depth stem wgrad (stem_s2d_*): the 7x7 / 2 / pad-3 C = 8 stem with <= 4 data
// channels (ResNet-18's 3), even H and W.  LDNN_CONV_STEM_S2D=0 turns it off (A/B knob).
int g_stem_s2d = -2;
void set_conv_stem_s2d(int mode) { g_stem_s2d = mode; }
bool stem_s2d_ok(const ConvShape& s) {
  if (g_stem_s2d == -2) g_stem_s2d = env_int("LDNN_CONV_STEM_S2D", 1);
  return g_stem_s2d != 0 && s.C == 8 && s.c_real > 0 && s.c_real <= 4 && s.K == 64 && s.R == 7 && s.S == 7 &&
         s.stride == 2 && s.pad == 3 && s.H % 2 == 0 && s.W % 2 == 0 && s.P == s.H / 2 && s.Q == s.W / 2 &&
         (size_t)s.N * (s.P + 3) * (s.Q + 3) * 32 < kOOBLimit;
}
// The stem forward on the packed s2d image (conv_s2d_ws_kernel): the wgrad's conditions, bf16 EPI_NONE,
// tiles that never span two images and whose s2d rows fit one ring buffer.
bool stem_s2d_fwd_ok(const ConvShape& s) {
  if (!stem_s2d_ok(s) || g_stem_s2d != 1 || ws_env() == 0) return false;   // (LDNN_CONV_STEM_S2D=2: wgrad only)
  const int PQ = s.P * s.Q, Ws = s.Q + 3;
  const int rows = (s.Q - 1 + 255) / s.Q + 1 + 3;   // output rows a 256-pixel tile touches, + the 4x4 taps
  return PQ % 256 == 0 && (int64_t)rows * Ws * 32 <= s2dfwd::kBuf && (int64_t)s.N * PQ >= 256;
}
struct S2dPlan {
  int Hs, Ws, nchunk, steps, slices, steps_per;
  size_t slab_floats, tmp_floats, xs_floats;
};
S2dPlan plan_s2d(const ConvShape& s) {
  S2dPlan p;
  p.Hs = s.P + 3;
  p.Ws = s.Q + 3;
  p.nchunk = (s.Q + 31) / 32;
  p.steps = s.N * s.P * p.nchunk;
  // three 48-KiB workgroups per CU: the K-step loop is bound by the DMA round trip of its 3 steps
  // in flight, not by bytes, so throughput scales with the workgroups resident per CU
  constexpr int target = 768;
  int slices = std::max(1, std::min(target, p.steps / 8));
  p.steps_per = (p.steps + slices - 1) / slices;
  p.slices = (p.steps + p.steps_per - 1) / p.steps_per;
  p.slab_floats = (size_t)p.slices * 64 * 256;
  p.tmp_floats = 64 * 256;
  p.xs_floats = (size_t)s.N * p.Hs * p.Ws * 8;  // bf16 x 16 channels
  return p;
}

// Patch path for C = 8 stems (conv_patch_kernel): 3x3 / 5x5 / 7x7 taps, stride 1 or 2,
// P*Q % 256 == 0 (tiles inside one image), K % 64 == 0, the patch within 48 KiB.
// LDNN_CONV_PATCH=0 turns it off (A/B knob).
int patch_env() {
  static const int v = env_int("LDNN_CONV_PATCH", 1);
  return v;
}
int patch_ks(const ConvShape& s) {
  const int rs = s.R * s.S;
  return rs == 9 ? 3 : rs == 25 ? 7 : rs == 49 ? 13 : 0;
}
bool patch_ok(const ConvShape& s) {
  if (patch_env() == 0 || s.C != 8 || s.K % 64 != 0 || patch_ks(s) == 0 || (s.stride != 1 && s.stride != 2)) return false;
  const int pq = s.P * s.Q;
  if (pq % 256 != 0) return false;
  const int rows_out = (255 + s.Q - 1) / s.Q + 1;  // output rows a 256-pixel tile can touch
  const int ph = (rows_out - 1) * s.stride + s.R;
  return (size_t)ph * (s.W + 2 * s.pad) * 16 <= (size_t)kPatchBytes;
}
template <int KS, int STR>
hipError_t launch_patch_e(const LArgs& a, int epi, const bf16_t* x, size_t bx, const bf16_t* w, hipStream_t st) {
  const dim3 grid(a.tiles_x), block(256);
  switch (epi) {
    case EPI_NONE: conv_patch_kernel<KS, STR, EPI_NONE><<<grid, block, 0, st>>>(a, x, (uint32_t)bx, w); break;
    case EPI_BIAS: conv_patch_kernel<KS, STR, EPI_BIAS><<<grid, block, 0, st>>>(a, x, (uint32_t)bx, w); break;
    case EPI_BIAS_RELU: conv_patch_kernel<KS, STR, EPI_BIAS_RELU><<<grid, block, 0, st>>>(a, x, (uint32_t)bx, w); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
template <int KS, int STR>
hipError_t launch_patch_ws_e(LArgs a, const bf16_t* x, size_t bx, const bf16_t* w, hipStream_t st) {
  const int grid = std::max(1, std::min(a.M / 256, cu_count()));
  a.tiles_x = grid;
  if (conv_xf_env() == 32)
    conv_patch_ws_kernel<KS, STR, 32><<<grid, 256, 0, st>>>(a, x, (uint32_t)bx, w);
  else
    conv_patch_ws_kernel<KS, STR><<<grid, 256, 0, st>>>(a, x, (uint32_t)bx, w);
  return hipGetLastError();
}

hipError_t launch_patch(LArgs a, int epi, const bf16_t* x, size_t bx, const bf16_t* w, hipStream_t st) {
  a.f_w = make_fastdiv(a.s.W + 2 * a.s.pad);  // patch row length (cell -> row, column)
  a.tiles_x = (a.M / 256) * (a.N / 64);
  const int ks = patch_ks(a.s);
  if (ws_env() != 0 && epi == EPI_NONE && a.N == 64 && ks == 13 && a.s.stride == 2)  // (LDNN_CONV_WS, as ws64)
    return launch_patch_ws_e<13, 2>(a, x, bx, w, st);
  if (a.s.stride == 1) {
    if (ks == 3) return launch_patch_e<3, 1>(a, epi, x, bx, w, st);
    if (ks == 7) return launch_patch_e<7, 1>(a, epi, x, bx, w, st);
    return launch_patch_e<13, 1>(a, epi, x, bx, w, st);
  }
  if (ks == 3) return launch_patch_e<3, 2>(a, epi, x, bx, w, st);
  if (ks == 7) return launch_patch_e<7, 2>(a, epi, x, bx, w, st);
  return launch_patch_e<13, 2>(a, epi, x, bx, w, st);
}

size_t stem_s2d_ws_bytes(const ConvShape& s) {
  const S2dPlan p = plan_s2d(s);
  return (p.slab_floats + p.tmp_floats + p.xs_floats) * 4;
}

hipError_t stem_s2d_fwd(LArgs a, const uint16_t* x, const uint16_t* w, uint16_t* s2d_xs, hipStream_t st) {
  const ConvShape& s = a.s;
  const int Hs = s.P + 3, Ws = s.Q + 3;
  const int64_t npix = (int64_t)s.N * Hs * Ws;
  if (!s.s2d_packed)   // (packed already: the graph's input staging wrote it, nchw_to_nhwc_s2d)
    stem_s2d_pack_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, st>>>(reinterpret_cast<const bf16_t*>(x),
                                                                          reinterpret_cast<bf16_t*>(s2d_xs), s.N, s.H,
                                                                          s.W, Hs, Ws);
  const int grid = std::max(1, std::min(a.M / 256, cu_count()));
  a.tiles_x = grid;
  conv_s2d_ws_kernel<<<grid, 256, 0, st>>>(a, reinterpret_cast<const bf16_t*>(s2d_xs), (uint32_t)(npix * 32), Hs, Ws,
                                           reinterpret_cast<const bf16_t*>(w));
  return hipGetLastError();
}

hipError_t stem_s2d_wgrad(const ConvShape& s, const uint16_t* dy, const uint16_t* x, float* dw, float beta,
                          hipStream_t st, float* ws, const uint16_t* s2d_xs) {
  const S2dPlan p = plan_s2d(s);
  float* slab = ws;
  float* tmp = ws + p.slab_floats;
  const int64_t npix = (int64_t)s.N * p.Hs * p.Ws;
  const bf16_t* xs = reinterpret_cast<const bf16_t*>(s2d_xs);
  if (xs == nullptr) {   // (the forward's packed image when it ran conv_s2d_ws_kernel)
    bf16_t* xsw = reinterpret_cast<bf16_t*>(tmp + p.tmp_floats);
    stem_s2d_pack_kernel<<<(unsigned)((npix + 255) / 256), 256, 0, st>>>(reinterpret_cast<const bf16_t*>(x), xsw, s.N,
                                                                          s.H, s.W, p.Hs, p.Ws);
    xs = xsw;
  }
  S2dArgs a{};
  a.N = s.N; a.P = s.P; a.Q = s.Q; a.Hs = p.Hs; a.Ws = p.Ws; a.K = s.K;
  a.nchunk = p.nchunk;
  a.steps = p.steps;
  a.steps_per = p.steps_per;
  a.slab = slab;
  const size_t bdy = (size_t)s.N * s.P * s.Q * s.K * 2, bxs = (size_t)npix * 32;
  stem_s2d_wgrad_kernel<<<p.slices, 256, 0, st>>>(a, reinterpret_cast<const bf16_t*>(dy), (uint32_t)bdy, xs,
                                                  (uint32_t)bxs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = slab_sum(slab, tmp, 64 * 256 / 4, p.slices, 0.f, st);
  if (e != hipSuccess) return e;
  stem_s2d_sum_kernel<<<(64 * 49 * 8 + 255) / 256, 256, 0, st>>>(tmp, dw, 1, beta);
  return hipGetLastError();
}

}  // namespace ldnn
