// LDS-DMA implicit-GEMM convolution for gfx950 (the fast path of conv.hip).
//
// Same GEMM views as conv.hip (fwd: y[NPQ][K] = x~[NPQ][RSC] . w[K][RSC]^T,
// dgrad: dx[NHW][C] = dy~[NHW][RSK] . w~[RSK][C], wgrad: dw[K][RSC] =
// dy[NPQ][K]^T . x~[NPQ][RSC]), but every operand tile is gathered straight
// from HBM/L2 into LDS by buffer_load_dwordx4 ... lds (no VGPR round trip).
// The DMA destination is lane-linear, so the whole GATHER lives in each lane's
// source offset; an out-of-image tap (zero padding, ragged edges) is an offset
// past the buffer's num_records, which the buffer unit returns as zeros.  No
// im2col buffer and no integer division in the main loop:
//
//   * fwd / dgrad need C (resp. K) % 64 == 0, so each 64-deep K-tile is ONE
//     filter tap (r, s) and 64 consecutive channels.  (r, s, channel block)
//     advances incrementally in scalar registers; each lane keeps the
//     decomposed pixel coordinates of its DMA rows, so an address is two bounds
//     checks and an add.
//   * stride-2 dgrad is split into the 4 output-parity classes (grid.z): pixel
//     (h, w) with h = 2 h2 + ph only receives taps r == (ph + pad) mod 2, so
//     each class is a dense problem over its own taps -- no zero-inserted MFMA
//     work (the generic kernel wastes 3/4 of it).
//   * wgrad reduces over output pixels npq; each lane carries (n, p, q) of its
//     DMA column and advances it by 64 pixels per K-tile with host-computed
//     carries (64 = dn*PQ + dp*Q + dq).  Small K x RSC outputs split npq over
//     gridDim.y and combine with fp32 atomics.
//   * small-M fwd / dgrad (the 2x2 / 4x4 tail stages) split the reduction over
//     gridDim.y and combine IN the launch (ldnn_gemm_tile.h splitk_combine):
//     deterministic, any epilogue, no fp32 round trip through a second kernel.
//
// Tiles: 64x64 per wave (4x4 v_mfma_f32_16x16x32_bf16 accumulators), wave grid
// WM x WN -> 128x128 (2x2), 256x64 (4x1: 64-channel layers), 64x256 (1x4:
// wgrad of 64-filter layers).  Two LDS stages, the DMA of K-tile t+1 in flight
// across the MFMAs of tile t (one raw s_barrier per K-tile, never
// __syncthreads while a DMA is outstanding); 2 workgroups per CU.  LDS images
// and fragment reads are those of gemm.hip (ldnn_gemm_tile.h).
// The launch arguments, geometry and epilogues shared with the C = 8 stem kernels live in
// ldnn_conv_lds.h; the stem kernels themselves (space-to-depth, patch) in conv_stem.hip.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "ldnn_conv_lds.h"

namespace ldnn {

namespace convlds {

// ---- operand gather policies ------------------------------------------------
// init(): per-lane state of this wave's PPW DMA pieces (1 KiB of LDS each);
// off(i, ks): byte offset of piece i's 16-B chunk for K-tile ks (kOOB = zeros);
// advance(): once per K-tile, after that tile's offsets were issued.

template <int ROWS, int PPW, int NW>
struct FwdA {  // x gathered: row = output pixel npq, k = (r, s, c), C % 64 == 0
  static constexpr bool KC = true;
  static constexpr int kRows = ROWS, kPieces = PPW;
  int base[PPW], ih0[PPW], iw0[PPW];
  __device__ void init(const LArgs& a, const Geo& g, int r0, int wid, int lane, int) {
    const ConvShape& s = a.s;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      int row, k;
      lds_slot_to_rk<true, ROWS>((i * NW + wid) * 1024 + lane * 16, row, k);
      const int m = r0 + row;
      const int t = fdiv(m, g.f_rw), q = m - t * s.Q, n = fdiv(t, g.f_rh), p = t - n * s.P;
      ih0[i] = p * s.stride - s.pad;
      iw0[i] = q * s.stride - s.pad;
      base[i] = (int)((unsigned)((n * s.H + ih0[i]) * s.W + iw0[i]) * (unsigned)s.C) + k;
      if (m >= a.M) ih0[i] = -(1 << 20);  // never inside the image
    }
  }
  __device__ __forceinline__ uint32_t off(const LArgs& a, int i, const KS& ks) const {
    const int ih = ih0[i] + ks.r, iw = iw0[i] + ks.s;
    const bool ok = (unsigned)ih < (unsigned)a.s.H && (unsigned)iw < (unsigned)a.s.W;
    const unsigned e = (unsigned)base[i] + (unsigned)((ks.r * a.s.W + ks.s) * a.s.C + ks.cb * 64);
    return ok ? e * 2u : kOOB;
  }
  __device__ __forceinline__ void advance(const LArgs&) {}
};

template <int ROWS, int PPW, int NW>
struct FwdASmallC {  // x gathered for C in {8, 16, 32}: a 64-deep K-tile spans 64/C filter taps
  static constexpr bool KC = true;
  static constexpr int kRows = ROWS, kPieces = PPW;
  int base[PPW], ih0[PPW], iw0[PPW], tl[PPW], cc[PPW];
  __device__ void init(const LArgs& a, const Geo& g, int r0, int wid, int lane, int) {
    const ConvShape& s = a.s;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      int row, k;
      lds_slot_to_rk<true, ROWS>((i * NW + wid) * 1024 + lane * 16, row, k);
      const int m = r0 + row;
      const int t = fdiv(m, g.f_rw), q = m - t * s.Q, n = fdiv(t, g.f_rh), p = t - n * s.P;
      ih0[i] = p * s.stride - s.pad;
      iw0[i] = q * s.stride - s.pad;
      base[i] = (int)((unsigned)((n * s.H + ih0[i]) * s.W + iw0[i]) * (unsigned)s.C);
      if (m >= a.M) ih0[i] = -(1 << 20);  // never inside the image
      tl[i] = k >> __builtin_ctz(s.C);    // tap within the K-tile (C is a power of two)
      cc[i] = k & (s.C - 1);              // channel offset within the tap
    }
  }
  __device__ __forceinline__ uint32_t off(const LArgs& a, int i, const KS& ks) const {
    const int tap = ks.kt * a.taps_per_tile + tl[i];
    const int r = fdiv(tap, a.f_s), sx = tap - r * a.s.S;
    const int ih = ih0[i] + r, iw = iw0[i] + sx;
    const bool ok = tap < a.s.R * a.s.S && (unsigned)ih < (unsigned)a.s.H && (unsigned)iw < (unsigned)a.s.W;
    const unsigned e = (unsigned)base[i] + (unsigned)((r * a.s.W + sx) * a.s.C + cc[i]);
    return ok ? e * 2u : kOOB;
  }
  __device__ __forceinline__ void advance(const LArgs&) {}
};

template <int ROWS, int PPW, int NW>
struct WeightKC {  // w as a [K][RSC] k-contiguous matrix (fwd B operand)
  static constexpr bool KC = true;
  static constexpr int kRows = ROWS, kPieces = PPW;
  int base[PPW], kl[PPW];
  __device__ void init(const LArgs& a, const Geo&, int r0, int wid, int lane, int) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      int row, k;
      lds_slot_to_rk<true, ROWS>((i * NW + wid) * 1024 + lane * 16, row, k);
      const int n = r0 + row;
      base[i] = n < a.N ? n * a.rsc + k : -1;
      kl[i] = k;
    }
  }
  __device__ __forceinline__ uint32_t off(const LArgs& a, int i, const KS& ks) const {
    if (a.nb > 0)  // one tap x 64 channels (either K-tile order)
      return base[i] >= 0 ? (uint32_t)(base[i] + (ks.r * a.s.S + ks.s) * a.s.C + ks.cb * 64) * 2u : kOOB;
    const bool ok = base[i] >= 0 && ks.kt * 64 + kl[i] < a.rsc;  // RSC % 64 != 0 for small C
    return ok ? (uint32_t)(base[i] + ks.kt * 64) * 2u : kOOB;
  }
  __device__ __forceinline__ void advance(const LArgs&) {}
};

template <int ROWS, int PPW, int NW>
struct DgradA {  // dy gathered: row = input pixel (class-local), k = (r, s, ko), K % 64 == 0
  static constexpr bool KC = true;
  static constexpr int kRows = ROWS, kPieces = PPW;
  int nP[PPW], hp[PPW], wp[PPW], kc[PPW];
  int sh;  // 1: stride-2 parity class (p = (h + pad - r) / 2, exact by construction)
  __device__ void init(const LArgs& a, const Geo& g, int r0, int wid, int lane, int) {
    const ConvShape& s = a.s;
    sh = g.hmul == 2 ? 1 : 0;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      int row, k;
      lds_slot_to_rk<true, ROWS>((i * NW + wid) * 1024 + lane * 16, row, k);
      const int m = r0 + row;
      const int t = fdiv(m, g.f_rw), w2 = m - t * g.rows_w, n = fdiv(t, g.f_rh), h2 = t - n * g.rows_h;
      nP[i] = n * s.P;
      hp[i] = m < g.M ? g.hmul * h2 + g.hoff + s.pad : -(1 << 20);
      wp[i] = g.hmul * w2 + g.woff + s.pad;
      kc[i] = k;
    }
  }
  __device__ __forceinline__ uint32_t off(const LArgs& a, int i, const KS& ks) const {
    const int p = (hp[i] - ks.r) >> sh, q = (wp[i] - ks.s) >> sh;
    const bool ok = (unsigned)p < (unsigned)a.s.P && (unsigned)q < (unsigned)a.s.Q;
    const unsigned e = ((unsigned)(nP[i] + p) * (unsigned)a.s.Q + (unsigned)q) * (unsigned)a.s.K +
                       (unsigned)(ks.cb * 64 + kc[i]);
    return ok ? e * 2u : kOOB;
  }
  __device__ __forceinline__ void advance(const LArgs&) {}
};

template <int ROWS, int PPW, int NW>
struct DgradB {  // w[ko][r][s][c]: n = c (8 consecutive), k = (r, s, ko)
  static constexpr bool KC = false;
  static constexpr int kRows = ROWS, kPieces = PPW;
  int base[PPW];
  __device__ void init(const LArgs& a, const Geo&, int r0, int wid, int lane, int) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      int row, k;
      lds_slot_to_rk<false, ROWS>((i * NW + wid) * 1024 + lane * 16, row, k);
      const int c = r0 + row;
      base[i] = c < a.N ? k * a.rsc + c : -1;
    }
  }
  __device__ __forceinline__ uint32_t off(const LArgs& a, int i, const KS& ks) const {
    const int u = ks.cb * 64 * a.rsc + (ks.r * a.s.S + ks.s) * a.s.C;
    return base[i] >= 0 ? (uint32_t)(base[i] + u) * 2u : kOOB;
  }
  __device__ __forceinline__ void advance(const LArgs&) {}
};

template <int ROWS, int PPW, int NW>
struct WgradA {  // dy as [NPQ][K]: row = ko (8 consecutive), k = npq
  static constexpr bool KC = false;
  static constexpr int kRows = ROWS, kPieces = PPW;
  int ko[PPW], kl[PPW];
  __device__ void init(const LArgs& a, const Geo&, int r0, int wid, int lane, int) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      int row, k;
      lds_slot_to_rk<false, ROWS>((i * NW + wid) * 1024 + lane * 16, row, k);
      ko[i] = r0 + row < a.M ? r0 + row : -1;
      kl[i] = k;
    }
  }
  __device__ __forceinline__ uint32_t off(const LArgs& a, int i, const KS& ks) const {
    const int npq = ks.kt * 64 + kl[i];
    return (ko[i] >= 0 && npq < a.Kd) ? (uint32_t)(npq * a.s.K + ko[i]) * 2u : kOOB;
  }
  __device__ __forceinline__ void advance(const LArgs&) {}
};

template <int ROWS, int PPW, int NW>
struct WgradB {  // x gathered: row = j = (r, s, c..c+7), k = npq (carried incrementally)
  static constexpr bool KC = false;
  static constexpr int kRows = ROWS, kPieces = PPW;
  int r[PPW], s[PPW], c[PPW], n[PPW], p[PPW], q[PPW];
  __device__ void init(const LArgs& a, const Geo&, int r0, int wid, int lane, int kt0) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      int row, k;
      lds_slot_to_rk<false, ROWS>((i * NW + wid) * 1024 + lane * 16, row, k);
      const int j = r0 + row;
      const int rs = fdiv(j, a.f_c);
      c[i] = j - rs * a.s.C;
      r[i] = fdiv(rs, a.f_s);
      s[i] = rs - r[i] * a.s.S;
      if (j >= a.N) r[i] = -(1 << 20);  // never inside the image
      const int npq = kt0 * 64 + k;
      n[i] = fdiv(npq, a.f_pq);
      const int pq = npq - n[i] * a.pq;
      p[i] = fdiv(pq, a.f_q);
      q[i] = pq - p[i] * a.s.Q;
    }
  }
  __device__ __forceinline__ uint32_t off(const LArgs& a, int i, const KS&) const {
    const ConvShape& sh = a.s;
    const int ih = p[i] * sh.stride - sh.pad + r[i], iw = q[i] * sh.stride - sh.pad + s[i];
    const bool ok = n[i] < sh.N && (unsigned)ih < (unsigned)sh.H && (unsigned)iw < (unsigned)sh.W;
    const unsigned e = (((unsigned)n[i] * (unsigned)sh.H + (unsigned)ih) * (unsigned)sh.W + (unsigned)iw) *
                           (unsigned)sh.C + (unsigned)c[i];
    return ok ? e * 2u : kOOB;
  }
  __device__ __forceinline__ void advance(const LArgs& a) {
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      q[i] += a.dq;
      if (q[i] >= a.s.Q) {
        q[i] -= a.s.Q;
        ++p[i];
      }
      p[i] += a.dp;
      if (p[i] >= a.s.P) {
        p[i] -= a.s.P;
        ++n[i];
      }
      n[i] += a.dn;
    }
  }
};


// DMA one operand tile (K-tile ks) into LDS at dst: PPW x buffer_load_dwordx4 ... lds per lane.
// (The voffset goes through an explicit int: with the unsigned call result passed
// straight to the builtin, hipcc silently emits no host launch stub.)
#define DMA_TILE(op, PPW, rsrc, dst, ks)                                                        \
  do {                                                                                               \
    _Pragma("unroll") for (int i_ = 0; i_ < (PPW); ++i_) {                                           \
      const int o_ = (int)(op).off(a, i_, (ks));                                                     \
      __builtin_amdgcn_raw_ptr_buffer_load_lds((rsrc).r, (lds_void*)((dst) + (i_ * NW + wid) * 1024), \
                                               16, o_, 0, 0, 0);                                     \
    }                                                                                                \
  } while (0)

// NS = LDS stages in the ring.  NS = 2: two workgroups per CU, the DMA of K-tile
// kt+1 in flight while kt is multiplied.  NS = 3 / 4 (grids of at most one
// workgroup per CU): K-tiles kt+1 .. kt+NS-1 in flight, a counted vmcnt (never 0
// in the steady state) retires only tile kt before the barrier that publishes it.
// XF (experiment builds only, LDNN_CONV_XF, on the 128x128 fwd / dgrad / wgrad and the narrow
// wgrad kernels): bit0 no in-loop DMA, bit1 (fwd only) the A operand DMAs contiguous
// 16-KiB-aligned chunks instead of the im2col gather, bit2 no fragment reads / MFMAs, bit5 phase
// trace: wave 0 stamps s_memrealtime (100 MHz) at entry, after the first K-tile landed, after
// the main loop and at exit into a.trace[workgroup][4] (scripts/conv_phase_trace.py).
// (Round 6 built and measured two more operand forms here -- B fragments straight to VGPRs and a
// BN + ReLU fold on the A fragments -- 1.8x / 1.74x slower, profiles/r6/conv_proto_ab.jsonl; their
// code was removed after the A/B, commit 0e684d8 has it.)
// (the body of conv_lds_kernel: smem = its NS-stage LDS ring, vb = its grid coordinates)
template <int WM, int WN, class OA, class OB, int EPI, bool OUT_F32, bool DGRAD, int NS, int XF = 0>
__device__ __forceinline__ void conv_lds_body(const LArgs& a, const bf16_t* pa, uint32_t bytes_a, const bf16_t* pb,
                                              uint32_t bytes_b, const VB& vb, char* smem) {
  constexpr int NW = WM * WN, BM = WM * 64, BN = WN * 64;
  static_assert(NW == 4, "4-wave workgroups (the launch bounds and the split-K slab size assume it)");
  static_assert(OA::kRows == BM && OB::kRows == BN && OA::kPieces == BM / 8 / NW && OB::kPieces == BN / 8 / NW,
                "operand policy geometry");
  constexpr int A_BYTES = BM * 128, B_BYTES = BN * 128, STAGE = A_BYTES + B_BYTES;
  constexpr int PPA = BM / 8 / NW, PPB = BN / 8 / NW;
  static_assert(PPA >= 1 && PPB >= 1 && PPA * NW * 8 == BM && PPB * NW * 8 == BN, "DMA pieces");
  constexpr int PER_TILE = PPA + PPB;  // DMA instructions per lane per K-tile
  static_assert(NS >= 2 && NS * STAGE <= 160 * 1024 && PER_TILE * (NS - 2) < 64, "LDS ring");

  const Geo g = make_geo(a, DGRAD, vb.z);
  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  uint64_t* trace = nullptr;
  if constexpr ((XF & 32) != 0) {
    if (threadIdx.x == 0 && a.trace != nullptr) {
      trace = a.trace + 8 * (size_t)(vb.x + vb.gx * (vb.y + vb.gy * vb.z));
      trace[0] = __builtin_amdgcn_s_memrealtime();
    }
  }
  int bx, by;
  split_coords(a, vb, bx, by);
  if (bx >= tiles_m * tiles_n) return;  // a smaller parity class: whole workgroup exits
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;
  int m0, n0;
  if (a.xcd_split && vb.gy > 1) {  // the XCD placement is split_coords'; tiles in row-major order
    m0 = (bx / tiles_n) * BM;
    n0 = (bx % tiles_n) * BN;
  } else {
    tile_coords_id(g.M, a.N, BM, BN, vb.x, m0, n0);
  }
  const int kt0 = by * a.nk_split;
  const int nk = max(0, min(g.nk - kt0, a.nk_split));
  const bool combine = a.cnt != nullptr && vb.gy > 1;
  if (nk == 0 && vb.gy > 1 && !combine && a.ws == nullptr) return;  // an empty atomic slice adds nothing

  floatx4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    OA oa;
    OB ob;
    oa.init(a, g, m0, wid, lane, kt0);
    ob.init(a, g, n0, wid, lane, kt0);
    Rsrc ra, rb;
    ra.r = __builtin_amdgcn_make_buffer_rsrc((void*)pa, (short)0, (int)bytes_a, 0x00020000);
    rb.r = __builtin_amdgcn_make_buffer_rsrc((void*)pb, (short)0, (int)bytes_b, 0x00020000);
    KS ks = ks_init(a, g, kt0);
    // prologue: K-tiles 0 .. NS-2 into stages 0 .. NS-2
#pragma unroll
    for (int t = 0; t < NS - 1; ++t) {
      if (t < nk) {
        if (t > 0) {
          ks_next(a, g, ks);
          oa.advance(a);
          ob.advance(a);
        }
        if constexpr (!(XF & 16)) DMA_TILE(oa, PPA, ra, smem + t * STAGE, ks);
        if constexpr (!(XF & 8)) DMA_TILE(ob, PPB, rb, smem + t * STAGE + A_BYTES, ks);
      }
    }

    int cur = 0;  // stage of K-tile kt
    for (int kt = 0; kt < nk; ++kt) {
      // own DMA of tile kt landed (tiles kt+1 .. kt+NS-2 may stay in flight)
      if (NS == 2 || kt + NS - 2 >= nk) {
        wait_vm<0>();
      } else {
        wait_vm<PER_TILE * (NS - 2)>();
      }
      lds_barrier();  // publishes tile kt; every wave is done reading tile kt-1's stage
      if constexpr ((XF & 32) != 0) {
        if (kt == 0 && trace != nullptr) trace[1] = __builtin_amdgcn_s_memrealtime();
      }
      if (!(XF & 1) && kt + NS - 1 < nk) {
        ks_next(a, g, ks);
        oa.advance(a);
        ob.advance(a);
        char* nxt = smem + (cur == 0 ? NS - 1 : cur - 1) * STAGE;  // stage of tile kt-1
        if constexpr ((XF & 2) != 0) {  // contiguous A chunks: the fill without the gather
          const uint32_t span = (bytes_a >> 1) & ~16383u;
          const uint32_t tb = (uint32_t)(bx * 9 + ks.kt) * (uint32_t)A_BYTES % span;
#pragma unroll
          for (int i_ = 0; i_ < PPA; ++i_)
            __builtin_amdgcn_raw_ptr_buffer_load_lds(ra.r, (lds_void*)(nxt + (i_ * NW + wid) * 1024), 16,
                                                     (int)(tb + (i_ * NW + wid) * 1024 + lane * 16), 0, 0, 0);
        } else if constexpr (!(XF & 16)) {
          DMA_TILE(oa, PPA, ra, nxt, ks);
        }
        if constexpr (!(XF & 8)) DMA_TILE(ob, PPB, rb, nxt + A_BYTES, ks);  // XF 8 / 16: no B / A fill
      }
      const char* la = smem + cur * STAGE;
      const char* lb = la + A_BYTES;
      if constexpr ((XF & 4) != 0) {
        cur = cur == NS - 1 ? 0 : cur + 1;
        continue;
      }
      __builtin_amdgcn_s_setprio(1);
      // all 16 fragments of the K-tile first (64 VGPRs): the reads of the second
      // K-half are in flight while the first half's 16 MFMAs run
      bf16x8 fa[2][4], fb[2][4];
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[kk][i] = read_frag<OA::KC, BM>(la, wm * 4 + i, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[kk][j] = read_frag<OB::KC, BN>(lb, wn * 4 + j, kk, lane);
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk][j], fa[kk][i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      cur = cur == NS - 1 ? 0 : cur + 1;
    }
  }

  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[2] = __builtin_amdgcn_s_memrealtime();
  }
  conv_tail<WM, WN, EPI, OUT_F32, DGRAD>(a, g, acc, m0, n0, wm, wn, lane, smem, NS * STAGE / 4, bx, by, vb);
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[3] = __builtin_amdgcn_s_memrealtime();
  }
}

template <int WM, int WN, class OA, class OB, int EPI, bool OUT_F32, bool DGRAD, int NS, int XF = 0>
__global__ __launch_bounds__(256, NS == 2 ? 2 : 1) void conv_lds_kernel(LArgs a, const bf16_t* pa, uint32_t bytes_a,
                                                                       const bf16_t* pb, uint32_t bytes_b) {
  constexpr int STAGE = (WM + WN) * 64 * 128;
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  conv_lds_body<WM, WN, OA, OB, EPI, OUT_F32, DGRAD, NS, XF>(a, pa, bytes_a, pb, bytes_b, hw_vb(), smem);
}

// Two independent convolution GEMMs in ONE launch: workgroups [0, n0) run body 0 over its
// (gx0, gy0, gz0) grid, the rest body 1 over (gx1, gy1, gz1) -- a layer's dgrad and wgrad (both
// read dy), or a downsampling block's 3x3 and 1x1 shortcut forward convs (both read x) -- so the
// two share the chip instead of each leaving CUs idle behind a small grid (EnhancedCNN's
// 16x16 .. 2x2 stages, ResNet-18 at b64).  n0 is a multiple of 8, so body 1's virtual ids keep
// their XCD placement.  F / D: the body's fp32-output / dgrad flags.
struct PairArgs {
  LArgs a[2];
  const bf16_t* pa[2];
  const bf16_t* pb[2];
  uint32_t ba[2], bb[2];
  int gx[2], gy[2], gz[2];
  int n0;
};
template <int WM0, int WN0, class OA0, class OB0, bool F0, bool D0, int WM1, int WN1, class OA1, class OB1, bool F1,
          bool D1>
__global__ __launch_bounds__(256, 2) void conv_pair_kernel(PairArgs p) {
  constexpr int ST0 = (WM0 + WN0) * 64 * 128, ST1 = (WM1 + WN1) * 64 * 128;
  constexpr int LDS = 2 * (ST0 > ST1 ? ST0 : ST1);
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  int b = (int)blockIdx.x;
  const int k = b >= p.n0 ? 1 : 0;
  if (k) b -= p.n0;
  const int gx = p.gx[k], gy = p.gy[k];
  if (b >= gx * gy * p.gz[k]) return;  // (the dgrad's id range is padded to a multiple of 8)
  const VB vb{b % gx, (b / gx) % gy, b / (gx * gy), gx, gy};
  if (k == 0)
    conv_lds_body<WM0, WN0, OA0, OB0, EPI_NONE, F0, D0, 2>(p.a[0], p.pa[0], p.ba[0], p.pb[0], p.bb[0], vb, smem);
  else
    conv_lds_body<WM1, WN1, OA1, OB1, EPI_NONE, F1, D1, 2>(p.a[1], p.pa[1], p.ba[1], p.pb[1], p.bb[1], vb, smem);
}

// A downsampling block's two convs' dgrads AND wgrads (four independent GEMMs) in ONE launch:
// slots 0 / 2 are the dgrads (128x128 or 256x64 gather kind), 1 / 3 the wgrads (128x128 or
// narrow); slot k's workgroups are [start[k], start[k+1]), every start a multiple of 8 (XCD
// placement kept).  Slot fields are read with compile-time indices (a runtime index into the
// kernel-argument arrays would copy them to scratch).
enum MultiKind { MK_DG128 = 0, MK_DG256, MK_WG128, MK_WGN };
struct MultiSlot {
  LArgs a;
  const bf16_t* pa;
  const bf16_t* pb;
  uint32_t ba, bb;
  int gx, gy, gz, kind, start;
};
template <bool DG>
__device__ __forceinline__ void multi_slot(const MultiSlot& q, int b, char* smem) {
  b -= q.start;
  const int gx = q.gx, gy = q.gy;
  if (b >= gx * gy * q.gz) return;  // (slot ranges are padded to multiples of 8)
  const VB vb{b % gx, (b / gx) % gy, b / (gx * gy), gx, gy};
  if constexpr (DG) {
    if (q.kind == MK_DG256)
      conv_lds_body<4, 1, DgradA<256, 8, 4>, DgradB<64, 2, 4>, EPI_NONE, false, true, 2>(q.a, q.pa, q.ba, q.pb, q.bb,
                                                                                        vb, smem);
    else
      conv_lds_body<2, 2, DgradA<128, 4, 4>, DgradB<128, 4, 4>, EPI_NONE, false, true, 2>(q.a, q.pa, q.ba, q.pb, q.bb,
                                                                                         vb, smem);
  } else {
    if (q.kind == MK_WGN)
      conv_lds_body<1, 4, WgradA<64, 2, 4>, WgradB<256, 8, 4>, EPI_NONE, true, false, 2>(q.a, q.pa, q.ba, q.pb, q.bb,
                                                                                        vb, smem);
    else
      conv_lds_body<2, 2, WgradA<128, 4, 4>, WgradB<128, 4, 4>, EPI_NONE, true, false, 2>(q.a, q.pa, q.ba, q.pb, q.bb,
                                                                                         vb, smem);
  }
}
// (four kernel parameters rather than one array: each slot's fields stay kernel-argument loads)
__global__ __launch_bounds__(256, 2) void conv_multi_kernel(MultiSlot q0, MultiSlot q1, MultiSlot q2, MultiSlot q3) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * 5 * 64 * 128];  // the largest kind's 2-stage ring
  const int b = (int)blockIdx.x;
  if (b >= q3.start) multi_slot<false>(q3, b, smem);
  else if (b >= q2.start) multi_slot<true>(q2, b, smem);
  else if (b >= q1.start) multi_slot<false>(q1, b, smem);
  else multi_slot<true>(q0, b, smem);
}

// ---- halo path: 3x3 stride-1 pad-1 fwd / dgrad with the A operand staged ONCE --
// The gather kernel above DMAs a fresh 64-channel A tile for every filter tap, so
// each activation row crosses the L1 / texture path 9 times per channel block --
// and that fill rate, not the MFMA, bounds it (11-15 % MFMA busy, profiles/).  For
// a stride-1 3x3 convolution the 9 taps of a tile read ONE contiguous run of
// flattened pixels: rows m0 - (W+1) .. m0 + BM + W of the NHWC activation.  This
// kernel DMAs that halo (BM + 2W + 2 rows x 64 channels, 128-B rows, XOR-swizzled
// like every KC image) once per channel block and reads each tap's A fragments
// from it at a row offset dr*W + ds; a lane whose tap falls outside the image
// (top / bottom / left / right edge, or a row past M) reads a zero row instead.
// The B operand (weights) streams per K-tile through a 2-stage ring as before.
// K-tile order is taps fastest inside a channel block; the halo buffer is reloaded
// at each channel block (two workgroups per CU cover that reload's latency).
// fwd: rows = output pixels, tap (r, s) reads x at (p + r - 1, q + s - 1);
// dgrad: rows = input pixels, tap (r, s) reads dy at (h + 1 - r, w + 1 - s).
constexpr int kHaloExtra = 120;  // 2W + 2 rows of halo, rounded up to 8, at most (W <= 59)

// (Measured negative, removed: a double-buffered variant for the 128x128 tiles -- the next
// channel block's halo DMAd into a second buffer over taps 0..7 -- cuts the fill per
// K-tile from 32 to ~19 KiB, yet ran slower than the gather kernel on every ResNet-18 /
// EnhancedCNN shape, e.g. C256 H14 b256 fwd 75 -> 106 us, dgrad 101 -> 112 us;
// profiles/r3/conv_fill_knockout_r3.txt.)
// XF bit5: the phase trace of conv_lds_kernel (entry / first K-tile landed / loop end / exit)
template <int WM, int WN, class OB, int EPI, bool DGRAD, int XF = 0>
__global__ __launch_bounds__(256, 2) void conv_halo_kernel(LArgs a, const bf16_t* pa, uint32_t bytes_a,
                                                           const bf16_t* pb, uint32_t bytes_b) {
  constexpr int NW = WM * WN, BM = WM * 64, BN = WN * 64;
  static_assert(NW == 4 && OB::kRows == BN && OB::kPieces == BN / 8 / NW, "operand policy geometry");
  constexpr int HR = BM + kHaloExtra;            // halo image rows (max)
  constexpr int H_BYTES = HR * 128, Z_BYTES = 128, B_BYTES = BN * 128;
  // B ring depth: 2 = K-tile kt+1 in flight (measured faster than 3 on the ResNet-18
  // shapes: the 3-stage ring's counted waits did not pay for its extra LDS)
  constexpr int NSB = 2;
  constexpr int LDS = H_BYTES + Z_BYTES + NSB * B_BYTES;
  static_assert(2 * LDS <= 160 * 1024, "two workgroups per CU");
  constexpr int PPB = OB::kPieces;
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  char* const halo = smem;
  char* const zrow = smem + H_BYTES;  // 128 zero bytes: the A fragment of a tap outside the image
  char* const bst = smem + H_BYTES + Z_BYTES;

  const Geo g = make_geo(a, DGRAD, (int)blockIdx.z);
  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  uint64_t* trace = nullptr;
  if constexpr ((XF & 32) != 0) {
    if (threadIdx.x == 0 && a.trace != nullptr) {
      trace = a.trace + 8 * (size_t)(blockIdx.x + gridDim.x * blockIdx.y);
      trace[0] = __builtin_amdgcn_s_memrealtime();
    }
  }
  if ((int)blockIdx.x >= tiles_m * tiles_n) return;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;
  int m0, n0;
  tile_coords(g.M, a.N, BM, BN, m0, n0);
  const int kt0 = blockIdx.y * a.nk_split;
  const int nk = max(0, min(g.nk - kt0, a.nk_split));

  floatx4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    const int W = g.rows_w, P = g.rows_h;
    const int cin = DGRAD ? a.s.K : a.s.C;            // channels of the A tensor
    const int hrows = (BM + 2 * W + 2 + 7) & ~7;      // halo rows of this shape (<= HR)
    const int hbase = m0 - (W + 1);                   // flattened pixel of halo row 0
    // per row-tile: this lane's halo row at tap offset 0, and its edge flags
    int lrow[4], edge[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * 64 + i * 16 + (lane & 15);
      const int m = m0 + r;
      const int t = fdiv(m, g.f_rw), q = m - t * W, n = fdiv(t, g.f_rh), p = t - n * P;
      lrow[i] = r + W + 1;
      edge[i] = (p == 0 ? 1 : 0) | (p == P - 1 ? 2 : 0) | (q == 0 ? 4 : 0) | (q == W - 1 ? 8 : 0) | (m >= g.M ? 16 : 0);
    }
    if (threadIdx.x < 8) *reinterpret_cast<floatx4*>(zrow + threadIdx.x * 16) = floatx4{0.f, 0.f, 0.f, 0.f};

    OB ob;
    ob.init(a, g, n0, wid, lane, kt0);
    Rsrc ra, rb;
    ra.r = __builtin_amdgcn_make_buffer_rsrc((void*)pa, (short)0, (int)bytes_a, 0x00020000);
    rb.r = __builtin_amdgcn_make_buffer_rsrc((void*)pb, (short)0, (int)bytes_b, 0x00020000);
    KS ks = ks_init(a, g, kt0);   // K-tile whose B is issued next
    KS kc = ks;                   // K-tile being multiplied

    // halo of channel block cb: 1-KiB pieces, 8 rows each, spread over the 4 waves
    auto load_halo = [&](int cb) {
      const int npieces = hrows >> 3;
      for (int pc = wid; pc < npieces; pc += NW) {
        const int j = pc * 8 + (lane >> 3);
        const int k = ((lane & 7) ^ (j & 7)) * 8;
        const int gp = hbase + j;
        const int o = gp >= 0 ? (int)(((unsigned)gp * (unsigned)cin + (unsigned)(cb * 64 + k)) * 2u) : (int)kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra.r, (lds_void*)(halo + pc * 1024), 16, o, 0, 0, 0);
      }
    };

    // prologue: B of K-tiles 0 .. NSB-2
#pragma unroll
    for (int t = 0; t < NSB - 1; ++t) {
      if (t < nk) {
        if (t > 0) {
          ks_next(a, g, ks);
          ob.advance(a);
        }
        DMA_TILE(ob, PPB, rb, bst + t * B_BYTES, ks);
      }
    }
    int cur = 0;
    for (int kt = 0; kt < nk; ++kt) {
      const int tap = kc.r * 3 + kc.s;
      if (kt == 0 || tap == 0) {
        if (kt > 0) lds_barrier();  // every wave is done reading the previous block's halo
        load_halo(kc.cb);
        wait_vm<0>();               // the halo (issued last) and with it every B in flight
      } else if (NSB > 2 && kt + 1 < nk) {
        wait_vm<PPB * (NSB - 2)>();  // B(kt) landed; later tiles may stay in flight
      } else {
        wait_vm<0>();
      }
      lds_barrier();  // publishes them; every wave is done with B(kt-1)'s stage
      if constexpr ((XF & 32) != 0) {
        if (kt == 0 && trace != nullptr) trace[1] = __builtin_amdgcn_s_memrealtime();
      }
      if (kt + NSB - 1 < nk) {  // B(kt+NSB-1) into the stage B(kt-1) used
        ks_next(a, g, ks);
        ob.advance(a);
        DMA_TILE(ob, PPB, rb, bst + (cur == 0 ? NSB - 1 : cur - 1) * B_BYTES, ks);
      }
      const int dr = DGRAD ? 1 - kc.r : kc.r - 1, ds = DGRAD ? 1 - kc.s : kc.s - 1;
      const int toff = dr * W + ds;
      const int emask = 16 | (dr < 0 ? 1 : 0) | (dr > 0 ? 2 : 0) | (ds < 0 ? 4 : 0) | (ds > 0 ? 8 : 0);
      const char* lb = bst + cur * B_BYTES;
      __builtin_amdgcn_s_setprio(1);
      bf16x8 fa[2][4], fb[2][4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int hr = lrow[i] + toff;
        const bool zero = (edge[i] & emask) != 0;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
          const int chunk = kk * 4 + (lane >> 4);
          const char* src = zero ? zrow + (chunk << 4) : halo + hr * 128 + ((chunk ^ (hr & 7)) << 4);
          fa[kk][i] = *reinterpret_cast<const bf16x8*>(src);
        }
      }
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 4; ++j) fb[kk][j] = read_frag<OB::KC, BN>(lb, wn * 4 + j, kk, lane);
#pragma unroll
      for (int kk = 0; kk < 2; ++kk)
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk][j], fa[kk][i], acc[j][i], 0, 0, 0);
      __builtin_amdgcn_s_setprio(0);
      cur = cur == NSB - 1 ? 0 : cur + 1;
      ks_next(a, g, kc);
    }
  }
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[2] = __builtin_amdgcn_s_memrealtime();
  }
  conv_tail<WM, WN, EPI, false, DGRAD>(a, g, acc, m0, n0, wm, wn, lane, smem, LDS / 4, blockIdx.x, blockIdx.y,
                                       hw_vb());
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[3] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---- big-tile halo conv: 3x3 stride-1 pad-1 fwd / dgrad, 256 x 128 tiles, 8 waves ----------
// The 128x128 gather kernel above moves 32 KiB through the LDS-DMA path per 2.1 MFLOP K-tile and
// runs at 18.5-19 % MFMA busy on ResNet-18's 128..512-channel stages (fill-bound: its per-CU
// LDS-DMA rate, not the MFMA pipe, sets the K-tile time, profiles/r3/conv_fill_knockout_r3.txt).
// Here one 8-wave workgroup per CU owns a 256-row x 128-column tile and cuts the bytes per MAC
// three ways: (a) the activation operand is a HALO -- the BM + 2W + 2 flattened pixels a tile's 9
// taps read, one 64-channel block of them, DMA'd ONCE per channel block (not once per tap) into
// rows of 160 B (8 data + 2 pad slots: a tap shift is a plain address offset and no shift
// conflicts, the conv_ws64_kernel layout); (b) the tile is 2x the gather kernel's, so each weight
// K-tile (16 KiB, the only per-K-tile stream left) feeds 4.2 MFLOP; (c) the weight stream runs 2
// K-tiles ahead in a 3-stage LDS ring and the next channel block's halo fills a second halo
// buffer during the current block's taps (counted vmcnt waits, raw barriers: nothing drains the
// DMA queue inside the loop).  Per K-tile ~20.5 KiB for 4.2 MFLOP against 32 KiB for 2.1.
// Waves: 4 row strips x 2 column halves, 64 x 64 each (the gather kernel's fragment map and
// MFMA order, so the shared epilogue / split-K / BN-statistics tail applies unchanged).  K-tile
// order: channel blocks, taps fastest (r-major); a split-K slice holds whole channel blocks.
// fwd: rows = output pixels, tap (r, s) reads x at (p + r - 1, q + s - 1); dgrad: rows = input
// pixels, tap (r, s) reads dy at (h + 1 - r, w + 1 - s).  W <= 32.
namespace hb {
constexpr int kBM = 256, kBN = 128, kNW = 8, kNT = 512;
constexpr int kPitch = 160;                   // halo row pitch: 8 data chunks + 2 zero pad slots
constexpr int kSlots = kPitch / 16;
constexpr int kMaxW = 32;                     // 2W + 2 rounded up to 8 <= 72 halo rows past the tile
constexpr int kHaloBytes = ((kBM + 72) * kPitch + 1023) / 1024 * 1024;   // 52 KiB (whole 1-KiB DMA pieces)
constexpr int kNSB = 3;                       // weight ring: K-tiles kt+1, kt+2 in flight
constexpr int kBBytes = kBN * 128;
constexpr int kLds = 2 * kHaloBytes + kNSB * kBBytes + 128;
static_assert(kLds <= 160 * 1024, "LDS");
}  // namespace hb

// s_waitcnt vmcnt(n) for a wave-uniform n (a scalar branch to the immediate)
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    case 8: wait_vm<8>(); break;
    case 9: wait_vm<9>(); break;
    case 10: wait_vm<10>(); break;
    case 11: wait_vm<11>(); break;
    default: wait_vm<0>(); break;
  }
}

template <class OB, int EPI, bool DGRAD>
__global__ __launch_bounds__(512, 1) void conv_hb_kernel(LArgs a, const bf16_t* pa, uint32_t bytes_a,
                                                         const bf16_t* pb, uint32_t bytes_b) {
  using namespace hb;
  constexpr int NW = kNW, WM = 4, WN = 2, BM = kBM, BN = kBN;
  constexpr int PPB = OB::kPieces;
  static_assert(OB::kRows == BN && PPB * NW * 8 == BN, "weight policy geometry");
  __shared__ __attribute__((aligned(1024))) char smem[kLds];
  char* const bst = smem + 2 * kHaloBytes;
  char* const zrow = bst + kNSB * kBBytes;  // 128 zero bytes: the A fragment of a tap outside the image

  const Geo g = make_geo(a, DGRAD, (int)blockIdx.z);
  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = (a.N + BN - 1) / BN;
  const int bx = blockIdx.x, by = blockIdx.y;
  if (bx >= tiles_m * tiles_n) return;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid / WN, wn = wid % WN;
  int m0, n0;
  tile_coords(g.M, a.N, BM, BN, m0, n0);
  const int kt0 = by * a.nk_split;  // a multiple of 9: slices hold whole channel blocks
  const int nk = max(0, min(g.nk - kt0, a.nk_split));

  floatx4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    const int W = g.rows_w, P = g.rows_h;
    const int cin = DGRAD ? a.s.K : a.s.C;             // channels of the A tensor
    const int hrows = BM + ((2 * W + 2 + 7) & ~7);     // halo rows of this shape
    const int npieces = (hrows * kSlots + 63) / 64;    // 1-KiB DMA pieces per halo
    const int hp = (npieces - wid + NW - 1) / NW;      // ... issued by this wave
    const int hbase = m0 - (W + 1);                    // flattened pixel of halo row 0
    const int cb0 = kt0 / 9, nblk = nk / 9;
    // per row tile: this lane's halo row offset at tap shift 0, and its image-edge flags
    int rowoff[4], edge[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = wm * 64 + i * 16 + (lane & 15);
      const int m = m0 + r;
      const int t = fdiv(m, g.f_rw), q = m - t * W, n = fdiv(t, g.f_rh), p = t - n * P;
      rowoff[i] = (r + W + 1) * kPitch + (lane >> 4) * 16;
      edge[i] = (p == 0 ? 1 : 0) | (p == P - 1 ? 2 : 0) | (q == 0 ? 4 : 0) | (q == W - 1 ? 8 : 0) | (m >= g.M ? 16 : 0);
    }
    if (threadIdx.x < 8) *reinterpret_cast<floatx4*>(zrow + threadIdx.x * 16) = floatx4{0.f, 0.f, 0.f, 0.f};

    Rsrc ra, rb;
    ra.r = __builtin_amdgcn_make_buffer_rsrc((void*)pa, (short)0, (int)bytes_a, 0x00020000);
    rb.r = __builtin_amdgcn_make_buffer_rsrc((void*)pb, (short)0, (int)bytes_b, 0x00020000);
    OB ob;
    ob.init(a, g, n0, wid, lane, kt0);
    KS ks = ks_init(a, g, kt0);  // K-tile whose weights are issued next

    // halo of channel block cb into buffer buf: lane-linear 16-B slots of kPitch-B rows (slots
    // 8, 9 of a row are padding and read as zeros, like rows outside the tensor)
    auto load_halo = [&](int cb, int buf) {
      char* const dst = smem + buf * kHaloBytes;
      for (int pc = wid; pc < npieces; pc += NW) {
        const int slot = pc * 64 + lane;
        const int j = slot / kSlots, c = slot - j * kSlots;
        const int gp = hbase + j;
        const int o = gp >= 0 && c < 8 ? (int)(((unsigned)gp * (unsigned)cin + (unsigned)(cb * 64 + c * 8)) * 2u)
                                       : (int)kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra.r, (lds_void*)(dst + pc * 1024), 16, o, 0, 0, 0);
      }
    };

    // prologue: the first block's halo, weights of K-tiles 0 and 1
    load_halo(cb0, 0);
    DMA_TILE(ob, PPB, rb, bst, ks);
    if (nk > 1) {
      ks_next(a, g, ks);
      ob.advance(a);
      DMA_TILE(ob, PPB, rb, bst + kBBytes, ks);
      wait_vm<PPB>();  // halo + weights(0) landed (loads retire in order)
    } else {
      wait_vm<0>();
    }
    lds_barrier();

    int kt = 0;
    for (int blk = 0; blk < nblk; ++blk) {
      const char* const hbuf = smem + (blk & 1) * kHaloBytes;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap, ++kt) {
        if (kt > 0) {
          // weights(kt) landed: what may stay in flight is what was issued after them --
          // weights(kt+1), and at taps 1 / 2 the next block's halo (issued at tap 0 after
          // weights(kt+2)); from tap 3 on that halo has to have landed too (it is read 6+ K-tiles later)
          const bool halo_after = (tap == 1 || tap == 2) && blk + 1 < nblk;
          wait_vm_n((kt + 1 < nk ? PPB : 0) + (halo_after ? hp : 0));
          lds_barrier();  // publishes weights(kt); every wave is done with K-tile kt-1
        }
        if (kt + 2 < nk) {  // weights(kt+2) into the stage K-tile kt-1 used
          ks_next(a, g, ks);
          ob.advance(a);
          DMA_TILE(ob, PPB, rb, bst + ((kt + 2) % kNSB) * kBBytes, ks);
        }
        if (tap == 0 && blk + 1 < nblk) load_halo(cb0 + blk + 1, (blk + 1) & 1);  // its buffer's last reader was K-tile kt-1
        const int dr = DGRAD ? 1 - tap / 3 : tap / 3 - 1, ds = DGRAD ? 1 - tap % 3 : tap % 3 - 1;
        const int emask = 16 | (dr < 0 ? 1 : 0) | (dr > 0 ? 2 : 0) | (ds < 0 ? 4 : 0) | (ds > 0 ? 8 : 0);
        const int toff = (dr * W + ds) * kPitch;
        const char* lb = bst + (kt % kNSB) * kBBytes;
        __builtin_amdgcn_s_setprio(1);
        bf16x8 fa[2][4], fb[2][4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const char* src = (edge[i] & emask) != 0 ? zrow + (lane >> 4) * 16 : hbuf + rowoff[i] + toff;
#pragma unroll
          for (int kk = 0; kk < 2; ++kk) fa[kk][i] = *reinterpret_cast<const bf16x8*>(src + kk * 64);
        }
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int j = 0; j < 4; ++j) fb[kk][j] = read_frag<OB::KC, BN>(lb, wn * 4 + j, kk, lane);
#pragma unroll
        for (int kk = 0; kk < 2; ++kk)
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[kk][j], fa[kk][i], acc[j][i], 0, 0, 0);
        __builtin_amdgcn_s_setprio(0);
      }
    }
  }
  conv_tail<WM, WN, EPI, false, DGRAD>(a, g, acc, m0, n0, wm, wn, lane, smem, hb::kLds / 4, bx, by, hw_vb());
}

// ---- weight-stationary persistent halo conv: 64 -> 64 channels, 3x3 stride 1 pad 1 ----
// conv_halo_kernel above streams the 8-KiB weight tile of every filter tap through a 2-stage
// LDS ring, and each tap waits for a DMA issued one tap earlier: at ResNet-18 layer 1 (C64 H56
// b256) its K loop takes 10.3 us for 9 taps -- 1.14 us per tap, the LDS-DMA issue -> landed
// latency (~1.1 us, MI355X_MICROARCH.md ldsdma-fill), against ~0.2 us of MFMA work
// (profiles/r4/conv_phase_trace_rn256.jsonl).  Here the whole 64 x 576 weight matrix lives in
// REGISTERS: a persistent grid (one 4-wave workgroup per CU, 512 registers per lane) stages it
// through LDS once, each wave keeps the B fragments of its 32 output channels for all 9 taps
// (144 VGPRs), and the loop over the workgroup's contiguous run of BM-row tiles only moves
// activations: one halo image per tile (BM + 128 rows of 64 channels, DMA'd into a double buffer
// one tile ahead), 9 taps x 2 x 2 x RT MFMAs per wave per tile with no wait inside the tile (the
// A fragments of step s+1 are read while step s multiplies).  Waves: 2 row strips of RT x 16
// rows x 2 column halves.  fwd: rows = output pixels, B[n][c] = w[n][r][s][c], tap shift (r-1,
// s-1); dgrad: rows = input pixels, B[c][k] = w[k][r][s][c], shift (1-r, 1-s).  Same MFMA order
// per accumulator as conv_halo_kernel (taps r-major, then kk), so the two agree bit for bit.  The
// fwd epilogue accumulates the next BatchNorm's statistics per lane over all of the workgroup's
// tiles and adds them once per workgroup.
namespace ws64 {
constexpr int kPitch = 1152 + 16;      // LDS row pitch of the staged weights (16-B aligned, rows spread over banks)
constexpr int kHPitch = 160;           // LDS row pitch of the halo: 8 chunks + 2 pad slots -- no swizzle, so a
                                       // tap shift is a plain address offset, and no bank conflict for any row
                                       // offset (144 B: 2-way, 4.1 extra LDS cycles per read measured)
constexpr int kSlots = kHPitch / 16;
constexpr int kWBytes = 64 * kPitch;   // 74,752 B
}  // namespace ws64

// XF = 32 (LDNN_CONV_XF=32 builds): the phase trace.  (The round-4 knockout builds -- no halo DMA,
// no stores, no fragment reads, no waits, register operands: profiles/r4/conv_ws64_micro.jsonl --
// were removed in round 6.)
template <int RT, bool DGRAD, int XF = 0>
__global__ __launch_bounds__(256, 1) void conv_ws64_kernel(LArgs a, const bf16_t* pa, uint32_t bytes_a,
                                                           const bf16_t* pw) {
  constexpr int NW = 4, NT = 256, BM = 2 * RT * 16;
  constexpr int HROWS = BM + 128;         // halo rows DMA'd per tile (>= BM + 2W + 2 for W <= 63)
  constexpr int HB = HROWS * ws64::kHPitch; // one halo buffer: rows of 8 16-B chunks + pad slots
  constexpr int PPW = HB / 1024 / NW;     // 1-KiB DMA pieces per wave per tile
  static_assert(PPW * NW * 1024 == HB && PPW < 64, "halo pieces");
  constexpr int REGION = 2 * HB + ws64::kWBytes;  // halo double buffer, then the staged weights
  constexpr int LDS = REGION + 128;
  static_assert(LDS <= 160 * 1024 && RT == 4, "LDS / tile rows (RT 8 spills, see launch_ws64)");
  __shared__ __attribute__((aligned(1024))) char smem[LDS];
  char* const wst = smem + 2 * HB;        // weight image (prologue only)
  char* const zrow = smem + REGION;       // 128 zero bytes: the A fragment of a tap outside the image

  uint64_t* trace = nullptr;
  if constexpr ((XF & 32) != 0) {
    if (threadIdx.x == 0 && a.trace != nullptr) {
      trace = a.trace + 8 * (size_t)blockIdx.x;
      trace[0] = __builtin_amdgcn_s_memrealtime();
    }
  }
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  const Geo g = make_geo(a, DGRAD, (int)blockIdx.z);
  const int W = g.rows_w, P = g.rows_h;
  const int T = (g.M + BM - 1) / BM;
  const int t0 = (int)((int64_t)blockIdx.x * T / gridDim.x);
  const int t1 = (int)((int64_t)(blockIdx.x + 1) * T / gridDim.x);

  Rsrc ra;
  ra.r = __builtin_amdgcn_make_buffer_rsrc((void*)pa, (short)0, (int)bytes_a, 0x00020000);
  // dgrad with bn_stats: the BN input tile (BM rows at kHPitch, as the halo) and its ReLU bits,
  // staged in the weight region; mask rows beyond M (or no mask: all ones) read as ...
  constexpr int XPW = BM * ws64::kHPitch / 1024 / NW;   // BN-input pieces per wave per tile
  static_assert(XPW * NW * 1024 == BM * ws64::kHPitch && BM * ws64::kHPitch + 1024 <= ws64::kWBytes, "x stage");
  char* const xst = wst;
  char* const mst = wst + BM * ws64::kHPitch;
  // output staging (also in the weight region): the tile's BM rows x 128 B at a 144-B pitch,
  // written in the MFMA layout and stored row-wise as whole 128-B rows
  constexpr int kOPitch = 144, kOStage = 24 * 1024;
  static_assert(kOStage >= BM * ws64::kHPitch + 1024 && kOStage + BM * kOPitch <= ws64::kWBytes, "out stage");
  char* const ost = wst + kOStage;
  Rsrc rbx, rbm;
  if constexpr (DGRAD) {
    rbx.r = __builtin_amdgcn_make_buffer_rsrc((void*)a.bnb_x, (short)0, a.bn_stats ? (int)((uint32_t)g.M * 128u) : 0,
                                              0x00020000);
    rbm.r = __builtin_amdgcn_make_buffer_rsrc((void*)a.bnb_mask, (short)0,
                                              a.bn_stats && a.bnb_mask ? (int)((uint32_t)g.M * 8u) : 0, 0x00020000);
  }
  // the halo of tile t into buffer b, lane-linear 16-B slots of kHPitch-B rows (slots 8.. of a
  // row are padding: zero reads); rows outside the tensor read as zeros
  auto dma = [&](int t, int b) {
    const int hbase = t * BM - (W + 1);
    char* const dst = smem + b * HB;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int pc = i * NW + wid;
      const int slot = pc * 64 + lane;
      const int j = slot / ws64::kSlots, c = slot - j * ws64::kSlots;
      const int gp = hbase + j;
      const int o = gp >= 0 && c < 8 ? (int)(((unsigned)gp * 64u + (unsigned)c * 8u) * 2u) : (int)kOOB;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra.r, (lds_void*)(dst + pc * 1024), 16, o, 0, 0, 0);
    }
  };

  float bs0[2][4], bs1[2][4];  // fwd: the next BN's per-channel sums over this workgroup's rows;
                              // dgrad: sum g, sum g xhat of the BN whose output's gradient dx is
  float bmu[2][4], bis[2][4];   // (dgrad: that BN's saved mean / invstd of this lane's channels)
#pragma unroll
  for (int j = 0; j < 2; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) bs0[j][r] = bs1[j][r] = bmu[j][r] = bis[j][r] = 0.f;
  if constexpr (DGRAD) {
    if (a.bn_stats) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = wn * 32 + j * 16 + 4 * (lane >> 4) + r;
          bmu[j][r] = a.bn.save_mean[c];
          bis[j][r] = a.bn.save_invstd[c];
        }
    }
  }

  // the first two tiles' halos DMA while the weights are staged (separate LDS regions)
  if (t0 < t1) {
    dma(t0, 0);
    if (t0 + 1 < t1) dma(t0 + 1, 1);
  }
  // weights -> LDS ([64][1152 B] at pitch kPitch) -> this wave's B fragments
  {
    constexpr int NQ = 64 * 72 / NT;  // 16-B pieces per thread, all loads in flight together
    static_assert(NQ * NT == 64 * 72, "weight pieces");
    uint4 wv[NQ];
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int q = threadIdx.x + k * NT, n = q / 72, c16 = q - n * 72;
      wv[k] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(pw) + (size_t)n * 1152 + c16 * 16);
    }
#pragma unroll
    for (int k = 0; k < NQ; ++k) {
      const int q = threadIdx.x + k * NT, n = q / 72, c16 = q - n * 72;
      *reinterpret_cast<uint4*>(wst + n * ws64::kPitch + c16 * 16) = wv[k];
    }
  }
  if (threadIdx.x < 8) *reinterpret_cast<floatx4*>(zrow + threadIdx.x * 16) = floatx4{0.f, 0.f, 0.f, 0.f};
  __syncthreads();
  bf16x8 fb[9][2][2];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = wn * 32 + j * 16 + (lane & 15), k0 = kk * 32 + (lane >> 4) * 8;
        if constexpr (!DGRAD) {
          fb[t][kk][j] = *reinterpret_cast<const bf16x8*>(wst + n * ws64::kPitch + t * 128 + k0 * 2);
        } else {
          u16x8 v;
#pragma unroll
          for (int e = 0; e < 8; ++e)
            v[e] = *reinterpret_cast<const uint16_t*>(wst + (k0 + e) * ws64::kPitch + t * 128 + n * 2);
          fb[t][kk][j] = __builtin_bit_cast(bf16x8, v);
        }
      }

  if (t0 < t1) {
    if (t0 + 1 < t1) wait_vm<PPW>();  // tile t0's pieces landed (loads retire in order)
    else wait_vm<0>();
  }
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[1] = __builtin_amdgcn_s_memrealtime();
  }
  bf16_t* const out = reinterpret_cast<bf16_t*>(a.out);
  for (int t = t0; t < t1; ++t) {
    const uint32_t halo = lds_off(smem + ((t - t0) & 1) * HB + (lane >> 4) * 16);
    const uint32_t zr = lds_off(zrow + (lane >> 4) * 16);
    // per (row tile, tap): this lane's A row address (the zero row for a tap outside the image);
    // a step's fragment is then one ds_read_b128 at that address + kk * 64, no address math
    uint32_t ab[RT][9];
#pragma unroll
    for (int i = 0; i < RT; ++i) {
      const int r = wm * RT * 16 + i * 16 + (lane & 15);
      const int m = t * BM + r;
      const int tq = fdiv(m, g.f_rw), q = m - tq * W, n = fdiv(tq, g.f_rh), p = tq - n * P;
      const int edge = (p == 0 ? 1 : 0) | (p == P - 1 ? 2 : 0) | (q == 0 ? 4 : 0) | (q == W - 1 ? 8 : 0) | (m >= g.M ? 16 : 0);
      const uint32_t rowp = halo + (r + W + 1) * ws64::kHPitch;
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        const int dr = DGRAD ? 1 - tap / 3 : tap / 3 - 1, ds = DGRAD ? 1 - tap % 3 : tap % 3 - 1;
        const int emask = 16 | (dr < 0 ? 1 : 0) | (dr > 0 ? 2 : 0) | (ds < 0 ? 4 : 0) | (ds > 0 ? 8 : 0);
        ab[i][tap] = (edge & emask) != 0 ? zr : rowp + (dr * W + ds) * ws64::kHPitch;
      }
    }
    // the fragment reads are asm (the compiler would otherwise sink each read next to its MFMAs
    // and wait on it there); their waits are the counted lgkmcnt below, tied to the registers
    auto read_step = [&](int st, bf16x8 (&f)[RT]) {
#pragma unroll
      for (int i = 0; i < RT; ++i) {
        if ((st & 1) == 0) {
          asm volatile("ds_read_b128 %0, %1" : "=v"(f[i]) : "v"(ab[i][st >> 1]));
        } else {
          asm volatile("ds_read_b128 %0, %1 offset:64" : "=v"(f[i]) : "v"(ab[i][st >> 1]));
        }
      }
    };
    floatx4 acc[2][RT];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < RT; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
    lds_barrier();  // every wave waited for its own pieces of tile t: the whole halo is visible
    if constexpr (DGRAD) {
      // (bn_stats) this tile's BN input rows and ReLU bits DMA'd into the weight staging region
      // (free after the prologue; every wave is past the last tile's epilogue reads here) while
      // the MFMA steps run; the epilogue reads them after the tile's vmcnt wait + a barrier
      if (a.bn_stats) {
#pragma unroll
        for (int i = 0; i < XPW; ++i) {
          const int pc = i * NW + wid;
          const int slot = pc * 64 + lane;
          const int j = slot / ws64::kSlots, c = slot - j * ws64::kSlots;
          const int gp = t * BM + j;
          const int o = gp < g.M && c < 8 ? (int)(((unsigned)gp * 64u + (unsigned)c * 8u) * 2u) : (int)kOOB;
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rbx.r, (lds_void*)(xst + pc * 1024), 16, o, 0, 0, 0);
        }
        if (wid == 0)   // 128 rows x 8 B of ReLU bits: one piece
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rbm.r, (lds_void*)mst, 16, (int)((unsigned)t * BM * 8u + lane * 16u),
                                                   0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(1);
    // step st = tap * 2 + kk: its RT fragment reads are issued two steps ahead
    static_assert(RT == 4, "the counted waits below name 4 fragments");
    bf16x8 fa[3][RT];
    read_step(0, fa[0]);
    read_step(1, fa[1]);
#pragma unroll
    for (int st = 0; st < 18; ++st) {
      bf16x8 (&f)[RT] = fa[st % 3];
      if (st + 2 < 18) read_step(st + 2, fa[(st + 2) % 3]);
      // step st's reads landed; steps st+1, st+2 (<= 2 RT reads) may be in flight
      if (st + 2 < 18) asm volatile("s_waitcnt lgkmcnt(8)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
      else if (st + 1 < 18) asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
      else asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]));
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < RT; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[st >> 1][st & 1][j], f[i], acc[j][i], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    lds_barrier();  // every wave is done reading this buffer
    if (t + 2 < t1) dma(t + 2, (t - t0) & 1);
    if (t + 1 < t1) {
      // tile t+1's pieces: issued a whole tile ago, followed only by the stores of tile t-1 and
      // tile t+2's pieces -- vmcnt(PPW) holds whether or not stores retire in order with loads
      if (t + 2 < t1) wait_vm<PPW>();
      else wait_vm<0>();
    }
    // epilogue: bf16 rows (8 B = 4 channels per lane), the BN sums of the rounded values
    u16x4 bxv[RT][2];
    uint32_t bmb[RT];
    if constexpr (DGRAD) {
      if (a.bn_stats) {
        if (t + 1 >= t1) wait_vm<0>();   // (the last tile has no vmcnt wait above)
        lds_barrier();   // every wave's BN-input pieces of this tile landed
#pragma unroll
        for (int i = 0; i < RT; ++i) {
          const int r = wm * RT * 16 + i * 16 + (lane & 15);
#pragma unroll
          for (int j = 0; j < 2; ++j)
            bxv[i][j] = *reinterpret_cast<const u16x4*>(xst + r * ws64::kHPitch + (wn * 32 + j * 16 + 4 * (lane >> 4)) * 2);
          // the 32 ReLU bits of channels 32 wn .. 32 wn + 31: bytes 4 wn .. 4 wn + 3 of the row
          bmb[i] = a.bnb_mask ? *reinterpret_cast<const uint32_t*>(mst + r * 8 + wn * 4) : 0xffffffffu;
        }
      }
    }
#pragma unroll
    for (int i = 0; i < RT; ++i) {
      const int r = wm * RT * 16 + i * 16 + (lane & 15);
      const int m = t * BM + r;
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = wn * 32 + j * 16 + 4 * (lane >> 4);
        const floatx4 v = acc[j][i];
        const u16x4 o = u16x4{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
        *reinterpret_cast<u16x4*>(ost + r * kOPitch + c * 2) = o;
        if constexpr (!DGRAD) {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float b = bf2f(o[r]);
            bs0[j][r] += b;
            bs1[j][r] += b * b;
          }
        } else {
          if (a.bn_stats) {
            // channel c + r is bit (c + r) - 32 wn of the 32-bit word at byte 4 wn of the row
            const uint32_t bits = bmb[i] >> (j * 16 + 4 * (lane >> 4));
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              const float gv = ((bits >> r) & 1u) ? bf2f(o[r]) : 0.f;
              bs0[j][r] += gv;
              bs1[j][r] += gv * (bf2f(bxv[i][j][r]) - bmu[j][r]) * bis[j][r];
            }
          }
        }
      }
    }
    lds_barrier();   // both column halves of every row are staged
#pragma unroll
    for (int q = 0; q < BM * 8 / NT; ++q) {   // 8 lanes x 16 B per 128-B row
      const int idx = q * NT + (int)threadIdx.x, r = idx >> 3, ch = idx & 7;
      const int m = t * BM + r;
      if (m < g.M)
        *reinterpret_cast<u32x4*>(out + (size_t)m * 64 + ch * 8) =
            *reinterpret_cast<const u32x4*>(ost + r * kOPitch + ch * 16);
    }
  }
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[2] = __builtin_amdgcn_s_memrealtime();
  }
  {
    if (a.bn_stats) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            bs0[j][r] += __shfl_xor(bs0[j][r], o, 64);
            bs1[j][r] += __shfl_xor(bs1[j][r], o, 64);
          }
      float* red = reinterpret_cast<float*>(smem);  // [2][64][2]
      __syncthreads();  // (the last tile's barrier already retired every halo read)
      if ((lane & 15) == 0) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = wn * 32 + j * 16 + 4 * (lane >> 4) + r;
            red[(wm * 64 + c) * 2] = bs0[j][r];
            red[(wm * 64 + c) * 2 + 1] = bs1[j][r];
          }
      }
      __syncthreads();
      float* accc = a.bn.acc + (size_t)(blockIdx.x % kBnCopies) * 2 * 64;
      if (threadIdx.x < 64) {
        const float s0 = red[threadIdx.x * 2] + red[(64 + threadIdx.x) * 2];
        const float s1 = red[threadIdx.x * 2 + 1] + red[(64 + threadIdx.x) * 2 + 1];
        bn_acc_add(accc + threadIdx.x, s0);
        bn_acc_add(accc + 64 + threadIdx.x, s1);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's atomics have completed
      bn_finalize_last<DGRAD, kBnCopies>(a.bn, g.M, 64, gridDim.x, red, LDS / 4);
    }
  }
  if constexpr ((XF & 32) != 0) {
    if (trace != nullptr) trace[3] = __builtin_amdgcn_s_memrealtime();
  }
}

// ---- ring wgrad: 3x3 stride-1 pad-1 weight gradient, activation rows staged once ----
// The split-K wgrad above re-gathers x for every filter tap: a 128x128 tile's K-tile
// moves 32 KiB through the LDS-DMA path for 2 MFLOP, and the pass is fill-bound (its
// DMA alone takes 100-122 of 113-131 us at ResNet-18 C128 H28 b256,
// profiles/r3/conv_fill_knockout_r3.txt).  Here ONE workgroup computes the whole
// 64 x (9 taps x 64 channels) gradient block of a (64-filter, 64-channel) pair over a
// slice of npq: per K-tile of 64 output pixels it DMAs the 64 x 64 dy tile (8 KiB) and
// only the 64 NEW activation rows of a 256-row LDS ring (8 KiB: the 9 taps of
// consecutive pixels read overlapping row windows, flattened pixel npq + (r-1) W +
// (s-1)) -- 16 KiB per 4.7 MFLOP instead of 120 KiB.  Both operands are read k-major
// (k = npq) with ds_read_b64_tr_b16 from 128-B rows (16-B chunks XOR-swizzled by row);
// a tap that leaves the image (row / column edge) zeroes its activation element by a
// per-lane mask (dy rows past the end read as zeros, so they need none).  Wave w owns
// channels 16w.. of the block for all 9 taps (taps unrolled: every mask / offset choice
// is compile-time): 9 x 4 MFMA accumulator tiles per wave; partial blocks go to fp32
// slabs summed by slab_sum_kernel.  The tiles of one npq slice run on one XCD.
namespace wr {
constexpr int kRingRows = 256, kRingBytes = kRingRows * 128, kDyBytes = 64 * 128;
}

struct WRArgs {
  int N, H, W, C, K, M;  // M = N*H*W output pixels (stride 1: = input pixels)
  int nk, nk_split;      // K-tiles of 64 pixels, per slice
  int kbn, cbn;          // 64-filter / 64-channel blocks
  int HE;                // halo rows beyond a K-tile's 64: (2W + 2) rounded up to 8 (<= 128)
  FastDiv f_w, f_h;
  float* out;            // [slices][K][9C] fp32 slabs, or dw itself with one slice
  float beta;            // one slice: out = acc + beta * out
};

__global__ __launch_bounds__(256, 2) void wgrad_ring_kernel(WRArgs a, const bf16_t* pdy, uint32_t bytes_dy,
                                                            const bf16_t* px, uint32_t bytes_x) {
  using namespace wr;
  __shared__ __attribute__((aligned(1024))) char smem[2 * kDyBytes + kRingBytes];  // 48 KiB
  char* const dyst = smem;
  char* const ring = smem + 2 * kDyBytes;
  typedef __attribute__((address_space(3))) bf16x4 lds_b4;
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = lane >> 4, r16 = lane & 15, qq = r16 >> 2, pp = r16 & 3;
  const int ntiles = a.kbn * a.cbn;
  const int id = xcd_remap(blockIdx.x, gridDim.x);  // the tiles of one slice on one XCD
  const int slice = id / ntiles, tile = id - (id / ntiles) * ntiles;
  const int kb = tile / a.cbn, cb = tile - (tile / a.cbn) * a.cbn;
  const int kt0 = slice * a.nk_split;
  const int nk = min(a.nk - kt0, a.nk_split);

  floatx4 acc[9][4];
#pragma unroll
  for (int j = 0; j < 9; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    Rsrc rdy, rx;
    rdy.r = __builtin_amdgcn_make_buffer_rsrc((void*)pdy, (short)0, (int)bytes_dy, 0x00020000);
    rx.r = __builtin_amdgcn_make_buffer_rsrc((void*)px, (short)0, (int)bytes_x, 0x00020000);
    const int hb = kt0 * 64 - (a.W + 1);  // pixel of ring slot 0
    const int jrow = lane >> 3, jslot = lane & 7;
    // dy K-tile kt into stage `st`: 8 pieces of 8 rows, pieces wid and wid + 4
    auto load_dy = [&](int kt, int st) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int pc = wid + 4 * h;
        const int j = pc * 8 + jrow;
        const int k = jslot ^ (j & 7);
        const uint32_t o = ((uint32_t)(kt * 64 + j) * (uint32_t)a.K + (uint32_t)(kb * 64 + k * 8)) * 2u;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rdy.r, (lds_void*)(dyst + st * kDyBytes + pc * 1024), 16, (int)o, 0,
                                                 0, 0);
      }
    };
    // ring rows [p0, p0 + n): n % 8 == 0, (p0 - hb) % 8 == 0; piece i issued by wave i % 4
    auto load_rows = [&](int p0, int n) {
      for (int pc = wid; pc < (n >> 3); pc += 4) {
        const int pix0 = p0 + pc * 8;
        const int slot0 = (pix0 - hb) & (kRingRows - 1);
        const int pix = pix0 + jrow;
        const int k = jslot ^ jrow;
        const int o = pix >= 0 ? (int)(((uint32_t)pix * (uint32_t)a.C + (uint32_t)(cb * 64 + k * 8)) * 2u) : (int)kOOB;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rx.r, (lds_void*)(ring + slot0 * 128), 16, o, 0, 0, 0);
      }
    };
    load_dy(kt0, 0);
    load_rows(hb, 64 + a.HE);
    const int cc = 2 * wid + (pp >> 1);  // this wave's 16 channels cb*64 + 16 wid ..: 16-B chunk of the tr reads
    for (int t = 0; t < nk; ++t) {
      wait_vm<0>();
      lds_barrier();  // publishes K-tile t; every wave is done with K-tile t-1's dy stage
      if (t + 1 < nk) {
        load_dy(kt0 + t + 1, (t + 1) & 1);
        load_rows(hb + 64 * (t + 1) + a.HE, 64);
      }
      const char* dys = dyst + (t & 1) * kDyBytes;
      const int npq0 = (kt0 + t) * 64;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        // this lane's 8 pixels b + e (b = npq0 + 32kk + 8g) cross at most one image row (W >= 8):
        // elements e >= ew are in the next row.  Edge masks (bit e = tap element valid):
        const int b = npq0 + 32 * kk + 8 * g;
        const int t1 = fdiv(b, a.f_w), q0 = b - t1 * a.W;
        const int p0 = t1 - fdiv(t1, a.f_h) * a.H;
        const int ew = a.W - q0;                                  // >= 1
        const uint32_t low = ew >= 8 ? 0xffu : (1u << ew) - 1u;  // elements in row p0
        const uint32_t row0 = (p0 == 0 ? ~low : 0xffu) & (p0 + 1 == a.H ? low : 0xffu) & 0xffu;  // tap row r = 0
        const uint32_t row2 = (p0 + 1 == a.H ? ~low : 0xffu) & (p0 + 2 == a.H ? low : 0xffu) & 0xffu;  // r = 2
        const uint32_t col0 = 0xffu & ~(q0 == 0 ? 1u : 0u) & ~(ew < 8 ? 1u << ew : 0u);        // s = 0: q >= 1
        const uint32_t col2 = 0xffu & ~(ew - 1 < 8 ? 1u << (ew - 1) : 0u);                      // s = 2: q <= W-2
        auto words = [](uint32_t m, u32x4& w) {
#pragma unroll
          for (int h = 0; h < 4; ++h)
            w[h] = ((0u - ((m >> (2 * h)) & 1u)) & 0xffffu) | ((0u - ((m >> (2 * h + 1)) & 1u)) << 16);
        };
        u32x4 wr0, wr2, wc0, wc2;
        words(row0, wr0);
        words(row2, wr2);
        words(col0, wc0);
        words(col2, wc2);
        // dy fragments (A: rows = filters i*16 + r16, k = pixels)
        bf16x8 fa[4];
        const int rl = 32 * kk + 8 * g + qq;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int c = 2 * i + (pp >> 1);
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_b4*)(dys + rl * 128 + ((c ^ (rl & 7)) << 4) + 8 * (pp & 1)));
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_b4*)(dys + (rl + 4) * 128 + ((c ^ ((rl + 4) & 7)) << 4) + 8 * (pp & 1)));
          fa[i] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        }
        const int sb = npq0 + rl - hb;  // ring position of this lane's row at tap offset 0
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
          const int r = tap / 3, sc = tap % 3;  // compile-time
          const int s0 = (sb + (r - 1) * a.W + (sc - 1)) & (kRingRows - 1);
          const int s1 = (s0 + 4) & (kRingRows - 1);
          const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_b4*)(ring + s0 * 128 + ((cc ^ (s0 & 7)) << 4) + 8 * (pp & 1)));
          const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
              (lds_b4*)(ring + s1 * 128 + ((cc ^ (s1 & 7)) << 4) + 8 * (pp & 1)));
          u32x4 w = __builtin_bit_cast(u32x4, bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]});
          if (r == 0) w &= wr0;
          if (r == 2) w &= wr2;
          if (sc == 0) w &= wc0;
          if (sc == 2) w &= wc2;
          const bf16x8 fb = __builtin_bit_cast(bf16x8, w);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[tap][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb, fa[i], acc[tap][i], 0, 0, 0);
        }
      }
    }
  }
  // lane holds out[filter kb*64 + 16i + r16][tap * C + cb*64 + 16*wid + 4g + 0..3]
  float* outp = a.out + (gridDim.x > (unsigned)ntiles ? (size_t)slice * a.K * 9 * a.C : 0);
  const int ldo = 9 * a.C;
#pragma unroll
  for (int tap = 0; tap < 9; ++tap) {
    const int col = tap * a.C + cb * 64 + 16 * wid + 4 * g;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float* o = outp + (size_t)(kb * 64 + 16 * i + r16) * ldo + col;
      floatx4 v = acc[tap][i];
      if (gridDim.x == (unsigned)ntiles && a.beta != 0.f) v += a.beta * *reinterpret_cast<const floatx4*>(o);
      *reinterpret_cast<floatx4*>(o) = v;
    }
  }
}

// NT: the slabs are read for the last time -- streaming (nontemporal) loads (measured -0.8 %
// on EnhancedCNN, profiles/slab_nontemporal_ab_r2.jsonl; every launch uses NT = true)
template <bool NT>
__device__ __forceinline__ floatx4 slab_ld(const floatx4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// sum over `splits` slabs (stride4 floatx4 apart) of the two floatx4 at w: 4 slabs' loads in
// flight per step (a plain loop waits on every load before the next add)
template <bool NT>
__device__ __forceinline__ void slab_sum8(const floatx4* w, int64_t stride4, int splits, floatx4& v0, floatx4& v1) {
  v0 = slab_ld<NT>(w);
  v1 = slab_ld<NT>(w + 1);
  int sp = 1;
  for (; sp + 3 < splits; sp += 4) {
    floatx4 a[4], b[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      a[u] = slab_ld<NT>(w + (sp + u) * stride4);
      b[u] = slab_ld<NT>(w + (sp + u) * stride4 + 1);
    }
    v0 += (a[0] + a[1]) + (a[2] + a[3]);
    v1 += (b[0] + b[1]) + (b[2] + b[3]);
  }
  for (; sp < splits; ++sp) {
    v0 += slab_ld<NT>(w + sp * stride4);
    v1 += slab_ld<NT>(w + sp * stride4 + 1);
  }
}

// bf16 out[m][n] = epi(sum_s ws[s][m][n] (+ bias[n])): the split-K reduction of the
// small-M fwd / dgrad slabs, 8 consecutive outputs per thread (two float4 per slab,
// one 16-B store), all CUs.
template <int EPI, bool NT>
__device__ __forceinline__ void slab_epi_body(const float* __restrict__ ws, bf16_t* __restrict__ out, int64_t n8,
                                              int N, int splits, const float* __restrict__ bias, int bxi) {
  const int64_t i = (int64_t)bxi * 256 + threadIdx.x;
  if (i >= n8) return;
  const floatx4* w = reinterpret_cast<const floatx4*>(ws) + 2 * i;
  floatx4 v0, v1;
  slab_sum8<NT>(w, 2 * n8, splits, v0, v1);
  const int n = (int)((i * 8) % N);
  u16x8 o;
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const float b = (EPI == EPI_NONE) ? 0.f : bias[n + q];
    o[q] = f2bf(apply_epi<EPI>(q < 4 ? v0[q] : v1[q - 4], b, 0.f));
  }
  reinterpret_cast<u16x8*>(out)[i] = o;
}
template <int EPI, bool NT>
__global__ __launch_bounds__(256) void conv_slab_epilogue_kernel(const float* __restrict__ ws, bf16_t* __restrict__ out,
                                                                 int64_t n8, int N, int splits,
                                                                 const float* __restrict__ bias) {
  slab_epi_body<EPI, NT>(ws, out, n8, N, splits, bias, (int)blockIdx.x);
}

hipError_t conv_slab_epilogue(const float* ws, uint16_t* out, int M, int N, int splits, const float* bias, int epi,
                              hipStream_t st) {
  const int64_t n8 = (int64_t)M * N / 8;
  if (n8 <= 0) return hipSuccess;
  const unsigned g = (unsigned)((n8 + 255) / 256);
  switch (epi) {
    case EPI_NONE: conv_slab_epilogue_kernel<EPI_NONE, true><<<g, 256, 0, st>>>(ws, out, n8, N, splits, bias); break;
    case EPI_BIAS: conv_slab_epilogue_kernel<EPI_BIAS, true><<<g, 256, 0, st>>>(ws, out, n8, N, splits, bias); break;
    case EPI_BIAS_RELU:
      conv_slab_epilogue_kernel<EPI_BIAS_RELU, true><<<g, 256, 0, st>>>(ws, out, n8, N, splits, bias);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// The slab split-K sum of a small-M forward conv AND the following training BatchNorm's
// statistics in one pass (the slab epilogue + a separate statistics pass otherwise): the grouped
// geometry of bn_reduce_small_kernel -- workgroup = 64 channels x rpb rows, 8 channel lanes x 32
// row lanes, every slab's loads of a row in flight together -- summing the statistics of the
// bf16-rounded outputs, then the per-column ticket finalize (ldnn_bn_fin.h).  (A round-2 variant
// with 8-copy atomics and one finalizing block was slower than the pair, profiles/cnn_slab_bn_ab_r2.jsonl.)
// BWD: the slab sum of a small-M stride-1 dgrad AND the backward statistics of the BN whose
// output's gradient it is (x / mask: that BN's input and ReLU bits; see bn_stats_epilogue).
constexpr int kSlabBnJs = 256 + 8;
constexpr int kSlabBnRed = 2 * 8 * kSlabBnJs;   // the body's LDS floats (red[2][8 * kJs])
// (bxi, byi): the workgroup's (column group, row group) of the (G, gy) grid; red: kSlabBnRed LDS
// floats + one int after them
// SRC16 (BWD only): no slabs -- the statistics of the bf16 dgrad output already in `out` (an
// in-launch combine / direct dgrad's dx), read instead of written.
template <bool NT, bool BWD, bool SRC16 = false>
__device__ __forceinline__ void slab_bn_body(const float* __restrict__ ws, bf16_t* __restrict__ out, int M, int N,
                                             int splits, const BnFin& fin, int rpb, const bf16_t* __restrict__ bx,
                                             const uint8_t* __restrict__ bmask, int bxi, int byi, int gy,
                                             float* red_) {
  constexpr int kLanes = 8, kRl = 32, kJs = kSlabBnJs;
  float (*red)[8 * kJs] = reinterpret_cast<float (*)[8 * kJs]>(red_);
  int& last = *reinterpret_cast<int*>(red_ + kSlabBnRed);
  const int tid = threadIdx.x, lane = tid % kLanes, rlane = tid / kLanes;
  const int c0 = bxi * 64 + lane * 8;
  float s0[8], s1[8], mu[8], is[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s0[j] = s1[j] = mu[j] = is[j] = 0.f;
  if (c0 < N) {
    if constexpr (BWD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mu[j] = fin.save_mean[c0 + j];
        is[j] = fin.save_invstd[c0 + j];
      }
    }
    const int r_end = min(M, (byi + 1) * rpb);
    const size_t sstride = (size_t)M * N / 4;
    for (int r = byi * rpb + rlane; r < r_end; r += kRl) {
      const size_t o = (size_t)r * N + c0;
      u16x8 xv = {0, 0, 0, 0, 0, 0, 0, 0};
      uint32_t mb = 0xffu;
      if constexpr (BWD) {  // issued ahead of the slab loads
        xv = *reinterpret_cast<const u16x8*>(bx + o);
        if (bmask != nullptr) mb = bmask[o >> 3];
      }
      u16x8 ob;
      if constexpr (SRC16) {
        ob = *reinterpret_cast<const u16x8*>(out + o);
      } else {
        floatx4 v0, v1;
        slab_sum8<NT>(reinterpret_cast<const floatx4*>(ws + o), (int64_t)sstride, splits, v0, v1);
#pragma unroll
        for (int j = 0; j < 8; ++j) ob[j] = f2bf(j < 4 ? v0[j] : v1[j - 4]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float v = bf2f(ob[j]);
        if constexpr (BWD) {
          const float gv = ((mb >> j) & 1u) ? v : 0.f;
          s0[j] += gv;
          s1[j] += gv * (bf2f(xv[j]) - mu[j]) * is[j];
        } else {
          s0[j] += v;
          s1[j] += v * v;
        }
      }
      if constexpr (!SRC16) *reinterpret_cast<u16x8*>(out + o) = ob;
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][j * kJs + tid] = s0[j];
    red[1][j * kJs + tid] = s1[j];
  }
  __syncthreads();
  if (tid < 64) {
    const int j = tid / kLanes, ln = tid - j * kLanes;
    float t0 = 0.f, t1 = 0.f;
#pragma unroll 8
    for (int q = 0; q < kRl; ++q) {
      t0 += red[0][j * kJs + q * kLanes + ln];
      t1 += red[1][j * kJs + q * kLanes + ln];
    }
    const int c = bxi * 64 + ln * 8 + j;
    if (gy == 1) {
      if (c < N) bn_finalize_channel<BWD>(fin, M, N, c, t0, t1, 1.f / (float)M);
    } else if (c < N) {
      grp_store(fin.part + (size_t)byi * 2 * N + c, t0);
      grp_store(fin.part + ((size_t)byi * 2 + 1) * N + c, t1);
    }
  }
  if (!BWD && bxi == 0 && byi == 0 && tid == 0 && fin.num_batches) fin.num_batches[0] += 1;
  if (gy == 1) return;
  if (!grp_ticket(fin.tickets + bxi, gy, last)) return;
  float* tot = &red[0][0];
  const int cc = bxi * 64 + (tid & 63);
  grp_sum(fin.part, N, cc, 0, gy, tot);
  grp_sum(fin.part, N, cc, 1, gy, tot);
  __syncthreads();
  if (tid < 64 && cc < N) {
    const float S0 = tot[tid] + tot[64 + tid] + tot[128 + tid] + tot[192 + tid];
    const float S1 = tot[256 + tid] + tot[320 + tid] + tot[384 + tid] + tot[448 + tid];
    bn_finalize_channel<BWD>(fin, M, N, cc, S0, S1, 1.f / (float)M);
  }
}

template <bool NT, bool BWD = false>
__global__ __launch_bounds__(256) void conv_slab_bn_kernel(const float* __restrict__ ws, bf16_t* __restrict__ out,
                                                           int M, int N, int splits, BnFin fin, int rpb,
                                                           const bf16_t* __restrict__ bx,
                                                           const uint8_t* __restrict__ bmask) {
  __shared__ float red[kSlabBnRed + 1];
  slab_bn_body<NT, BWD>(ws, out, M, N, splits, fin, rpb, bx, bmask, (int)blockIdx.x, (int)blockIdx.y,
                        (int)gridDim.y, red);
}

int env_int(const char* name, int dflt);
// slab-split forward convs followed by a training BN take the BN statistics in
// conv_slab_bn_kernel (9 fewer launches per EnhancedCNN step, profiles/r5/conv_slab_bn_ab.txt)
constexpr int kSlabBnTarget = 512;   // conv_slab_bn workgroups aimed at
// LDNN_CONV_BN_BWD (documented fallback): stride-1 dgrads take the backward statistics of the BN
// whose output's gradient they produce (conv2d_dgrad with a BnBwdFuse): 1 (default) in the slab
// split-K sum, and for a dgrad without slabs that shares its launch with the wgrad, as a pass over
// dx in the shared post launch, and in the weight-stationary 64 -> 64 dgrad's persistent epilogue;
// 2 all but the weight-stationary one; 0 never (the BN runs its own reduce).  (The form inside the direct
// / in-launch-combine epilogue -- x and mask loads, 8-copy atomics and one finalizing workgroup
// behind the tile's own stores -- added 11-13 us to a 64 / 128-tile dgrad to save an 8-10 us reduce
// launch, profiles/r5/conv_bn_bwd_ab.txt, and was removed in round 6.)
int g_bn_bwd = -1;
int bn_bwd_env() {
  if (g_bn_bwd < 0) g_bn_bwd = env_int("LDNN_CONV_BN_BWD", 1);
  return g_bn_bwd;
}
hipError_t conv_slab_bn(const float* ws, uint16_t* out, int M, int N, int splits, const BnFin& fin, hipStream_t st,
                        const BnBwdFuse* bnb = nullptr) {
  if (M <= 0) return hipSuccess;
  constexpr int target = kSlabBnTarget;
  const int G = (N + 63) / 64;
  int ny = std::max(1, std::min({(target + G - 1) / G, (M + 31) / 32, kGrpMax}));
  const int rpb = (M + ny - 1) / ny;
  ny = (M + rpb - 1) / rpb;
  const dim3 g(G, ny);
  if (bnb != nullptr) {
    const bf16_t* bx = reinterpret_cast<const bf16_t*>(bnb->x);
    conv_slab_bn_kernel<true, true><<<g, 256, 0, st>>>(ws, out, M, N, splits, fin, rpb, bx, bnb->mask);
    return hipGetLastError();
  }
  conv_slab_bn_kernel<true><<<g, 256, 0, st>>>(ws, out, M, N, splits, fin, rpb, nullptr, nullptr);
  return hipGetLastError();
}

// out[i] = sum_s ws[s][i] (+ beta * out[i]): the cross-CU reduction of wgrad slabs.
// A block is 32 float4 columns x 8 split lanes (each lane sums every 8th slab,
// 4 loads in flight), reduced through LDS: enough blocks to cover the chip even
// for a 64 x 576 weight, and a fixed summation order (deterministic).
template <bool NT>
__device__ __forceinline__ void slab_sum_body(const float* __restrict__ ws, float* __restrict__ out, int64_t n4,
                                              int splits, float beta, int bxi, floatx4 (*part)[32]) {
  const int col = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int64_t i = (int64_t)bxi * 32 + col;
  floatx4 v = {0.f, 0.f, 0.f, 0.f};
  if (i < n4) {
    const floatx4* w = reinterpret_cast<const floatx4*>(ws) + i;
    int sp = sl;
    for (; sp + 24 < splits; sp += 32) {
      const floatx4 a = slab_ld<NT>(w + (int64_t)sp * n4), b = slab_ld<NT>(w + (int64_t)(sp + 8) * n4);
      const floatx4 c = slab_ld<NT>(w + (int64_t)(sp + 16) * n4), d = slab_ld<NT>(w + (int64_t)(sp + 24) * n4);
      v += (a + b) + (c + d);
    }
    for (; sp < splits; sp += 8) v += slab_ld<NT>(w + (int64_t)sp * n4);
  }
  part[sl][col] = v;
  __syncthreads();
  if (sl == 0 && i < n4) {
#pragma unroll
    for (int q = 1; q < 8; ++q) v += part[q][col];
    if (beta != 0.f) v += beta * reinterpret_cast<const floatx4*>(out)[i];
    reinterpret_cast<floatx4*>(out)[i] = v;
  }
}
template <bool NT>
__global__ __launch_bounds__(256) void slab_sum_kernel(const float* __restrict__ ws, float* __restrict__ out,
                                                       int64_t n4, int splits, float beta) {
  __shared__ floatx4 part[8][32];
  slab_sum_body<NT>(ws, out, n4, splits, beta, (int)blockIdx.x, part);
}

// The passes after a shared conv launch -- its GEMMs' slab sums (plain, with the next BN's
// statistics, with a BN's backward statistics) and wgrad slab sums -- as ONE launch: task k owns
// workgroups [start, start + gx * gy).  They are independent (disjoint outputs, per-BN tickets).
enum PostKind { PK_EPI = 0, PK_BN_FWD, PK_BN_BWD, PK_SUM, PK_BN_BWD_RED };
struct PostTask {
  int kind, start, gx, gy;
  const float* ws;
  void* out;
  int M, N, splits, rpb;
  float beta;
  int64_t n;  // PK_EPI: outputs / 8; PK_SUM: floats / 4
  BnFin fin;
  const uint16_t* bx;
  const uint8_t* mask;
};
template <bool NT>
__device__ __forceinline__ void post_run(const PostTask& t, int b, float* lds) {
  switch (t.kind) {
    case PK_EPI:
      slab_epi_body<EPI_NONE, NT>(t.ws, reinterpret_cast<bf16_t*>(t.out), t.n, t.N, t.splits, nullptr, b);
      break;
    case PK_BN_FWD:
      slab_bn_body<NT, false>(t.ws, reinterpret_cast<bf16_t*>(t.out), t.M, t.N, t.splits, t.fin, t.rpb, nullptr,
                              nullptr, b % t.gx, b / t.gx, t.gy, lds);
      break;
    case PK_BN_BWD:
      slab_bn_body<NT, true>(t.ws, reinterpret_cast<bf16_t*>(t.out), t.M, t.N, t.splits, t.fin, t.rpb,
                             reinterpret_cast<const bf16_t*>(t.bx), t.mask, b % t.gx, b / t.gx, t.gy, lds);
      break;
    case PK_BN_BWD_RED:
      slab_bn_body<NT, true, true>(nullptr, reinterpret_cast<bf16_t*>(t.out), t.M, t.N, 0, t.fin, t.rpb,
                                   reinterpret_cast<const bf16_t*>(t.bx), t.mask, b % t.gx, b / t.gx, t.gy, lds);
      break;
    default:
      slab_sum_body<NT>(t.ws, reinterpret_cast<float*>(t.out), t.n, t.splits, t.beta, b,
                        reinterpret_cast<floatx4(*)[32]>(lds));
      break;
  }
}
template <bool NT>
__global__ __launch_bounds__(256) void conv_post_kernel(PostTask t0, PostTask t1, PostTask t2, PostTask t3) {
  __shared__ __attribute__((aligned(16))) float lds[kSlabBnRed + 4];
  const int b = (int)blockIdx.x;
  if (t3.gx && b >= t3.start) post_run<NT>(t3, b - t3.start, lds);
  else if (t2.gx && b >= t2.start) post_run<NT>(t2, b - t2.start, lds);
  else if (t1.gx && b >= t1.start) post_run<NT>(t1, b - t1.start, lds);
  else post_run<NT>(t0, b, lds);
}

bool fits(size_t bytes) { return bytes < kOOBLimit; }

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

struct WgradPlan {
  bool narrow;
  bool ring;  // wgrad_ring_kernel (3x3 s1 p1, C % 64 == K % 64 == 0, 8 <= W <= 63)
  int tiles, splits, nk_all, nk_split;
};

// LDNN_CONV_WGRAD_RING (A/B knob): 1 (default) the ring wgrad for the 64-filter x 64-channel
// 3x3 stride-1 convs (ResNet-18 layer 1: 56 -> 43 us at b64, 178 -> 117 us at b256, where the
// split-K kernel's 64x256 tiles re-read dy 3x and waste a quarter of their MFMAs); 2 also
// for wider layers (measured equal at ResNet-18 28x28 / 14x14, slower at EnhancedCNN's 16x16
// / 8x8 b64, whose ~20 K-tiles per block leave too few workgroups:
// profiles/r3/wgrad_ring_ab_r3.txt); 0 off
int g_wgrad_ring = -2;  // -2: not read yet
int wgrad_ring_env() {
  if (g_wgrad_ring == -2) g_wgrad_ring = env_int("LDNN_CONV_WGRAD_RING", 1);
  return g_wgrad_ring;
}
bool wgrad_ring_ok(const ConvShape& s) {
  const int m = wgrad_ring_env();
  return m != 0 && s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.P == s.H && s.Q == s.W &&
         s.C % 64 == 0 && s.K % 64 == 0 && s.W >= 8 && s.W <= 63 && (m == 2 || (s.C == 64 && s.K == 64));
}

WgradPlan plan_wgrad(const ConvShape& s, bool allow_ring = true) {
  WgradPlan p;
  p.ring = allow_ring && wgrad_ring_ok(s);
  if (p.ring) {  // (64 filters x 576 tap-channels) blocks x npq slices of >= 12 K-tiles, ~512 workgroups
    // (two per CU: ResNet-18 b256 7.652 vs 7.705-7.711 ms at 384, 7.70 at 256, 7.78 at 1024; b64 capped by
    // the 12-K-tile floor either way, profiles/r4/ring_wgrad_target_ab.jsonl)
    constexpr int target = 512;
    p.narrow = false;
    p.tiles = (s.K / 64) * (s.C / 64);
    p.nk_all = (s.N * s.P * s.Q + 63) / 64;
    int splits = std::max(1, std::min(target / p.tiles, p.nk_all / 12));
    p.nk_split = (p.nk_all + splits - 1) / splits;
    p.splits = (p.nk_all + p.nk_split - 1) / p.nk_split;
    return p;
  }
  p.narrow = s.K <= 64;
  const int BM = p.narrow ? 64 : 128, BN = p.narrow ? 256 : 128;
  const int M = s.K, N = s.R * s.S * s.C;
  p.tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  p.nk_all = (s.N * s.P * s.Q + 63) / 64;
  // split the npq reduction over ~1.5 workgroups per CU, >= min_kt K-tiles per slice
  int splits = 1;
  // (512 since dgrad and wgrad share launches: ResNet-18 b256 7.332 -> 7.256 ms, b64 -0.2 %, EnhancedCNN
  // neutral, 6 alternated samples each, profiles/r5/conv_wgrad_target_ab.txt)
  constexpr int target = 512;  // workgroups to aim for
  constexpr int min_kt1 = 8;   // K-tiles per slice, 1x1 filters
  // larger filters: >= 16 K-tiles per slice since dgrad and wgrad share a launch (EnhancedCNN b64
  // 1.642 -> 1.573 ms with the slab target at 256, ResNet-18 b64 / b256 -0.3 / -0.2 %; the 1x1
  // shortcut wgrads stay at 8: 16 there cost ResNet-18 b64 +0.6 %, profiles/r5/conv_split_knobs_ab.txt)
  constexpr int min_kt3 = 16;
  // (C = 8 / K <= 16 -- LeNet-5 -- : one 64x256 tile, the slices' K loops are the whole pass)
  const int min_kt = (s.C <= 8 && s.K <= 16) ? 4 : s.R * s.S > 1 ? min_kt3 : min_kt1;
  if (p.tiles < 256) splits = std::max(1, std::min((target + p.tiles - 1) / p.tiles, p.nk_all / min_kt));
  p.nk_split = (p.nk_all + splits - 1) / splits;
  p.splits = (p.nk_all + p.nk_split - 1) / p.nk_split;
  return p;
}

uint64_t* g_conv_trace = nullptr;  // phase-trace buffer of LDNN_CONV_XF=32 builds (set_conv_trace)

// the in-launch split-K combine's summer is the tile's last K slice (splitk_combine_last, round 5)
// instead of the last workgroup to arrive; set_conv_combine_last(0) (tests) selects the latter
int g_combine_last = 1;

// Fixed choices of earlier A/Bs (round 2, profiles/*_ab_r2.jsonl): filter taps fastest in the
// fwd / dgrad K-tile order (consecutive K-tiles re-read shifted rows of one channel block, which
// L2 / L1 serve warm: ResNet-18 b64 3.89 -> 3.85 ms); fp32 outputs, bf16 outputs (also in two
// 32-row halves where a wave has only 8 KiB of LDS) and the stride-2 dgrad row remap all staged
// through LDS for full-row stores.
LArgs base_args(const ConvShape& s) {
  LArgs a{};
  a.trace = g_conv_trace;
  a.combine_last = g_combine_last;
  a.tap_major = 1;
  a.f32_rows = 1;
  a.bf16_rows = 2;
  a.remap_rows = 1;
  a.s = s;
  a.rsc = s.R * s.S * s.C;
  a.pq = s.P * s.Q;
  a.classes = 1;
  a.f_p = make_fastdiv(s.P);
  a.f_q = make_fastdiv(s.Q);
  a.f_h = make_fastdiv(s.H);
  a.f_w = make_fastdiv(s.W);
  for (int c = 0; c < 2; ++c) {
    a.f_cw[c] = make_fastdiv((s.W - c + 1) >> 1);
    a.f_ch[c] = make_fastdiv((s.H - c + 1) >> 1);
  }
  return a;
}

bool shape_ok(const ConvShape& s) {
  return s.N > 0 && s.stride >= 1 && s.stride <= 2 && fits((size_t)s.N * s.H * s.W * s.C * 2) &&
         fits((size_t)s.K * s.R * s.S * s.C * 2) && fits((size_t)s.N * s.P * s.Q * s.K * 2);
}

// LDS ring depth NS = 2 (two workgroups = 8 waves per CU).  (A deep ring, NS 3 / 4 at one
// workgroup per CU with 2-3 K-tiles in flight, measured SLOWER on every ResNet-18 @224 shape --
// fwd+dgrad+wgrad 922 vs 710 us, profiles/conv_ring_depth_r1.txt; r4: 10.05 vs 7.71 ms -- and was
// removed in round 6: the second workgroup's waves hide the per-wave ds_read / barrier latency
// better than deeper DMA prefetch does.)

// OA / OB = Policy<rows, DMA pieces per wave (= rows / 8 / 4 waves), 4 waves>.
int conv_xf_env() {
  static const int v = env_int("LDNN_CONV_XF", 0);
  return v;
}

template <int WM, int WN, class OA, class OB, bool OUT_F32, bool DGRAD, int NS>
hipError_t launch_ns(LArgs a, int epi, int splits, const bf16_t* pa, size_t ba, const bf16_t* pb, size_t bb,
                     hipStream_t st) {
  constexpr int NW = WM * WN;
  dim3 grid(a.tiles_x, splits, a.classes), block(NW * 64);
  if constexpr ((std::is_same_v<OA, FwdA<128, 4, 4>> || std::is_same_v<OA, WgradA<64, 2, 4>> ||
                 std::is_same_v<OA, WgradA<128, 4, 4>> || std::is_same_v<OA, DgradA<128, 4, 4>>) && NS == 2) {
    const int xf = conv_xf_env();
    if (xf != 0 && epi == EPI_NONE) {
      switch (xf) {
        case 1: conv_lds_kernel<WM, WN, OA, OB, EPI_NONE, OUT_F32, DGRAD, NS, 1><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb); break;
        case 2:
          if constexpr (!std::is_same_v<OA, FwdA<128, 4, 4>>) return hipErrorInvalidValue;
          else conv_lds_kernel<WM, WN, OA, OB, EPI_NONE, OUT_F32, DGRAD, NS, 2><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb);
          break;
        case 4: conv_lds_kernel<WM, WN, OA, OB, EPI_NONE, OUT_F32, DGRAD, NS, 4><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb); break;
        case 6:
          if constexpr (!std::is_same_v<OA, FwdA<128, 4, 4>>) return hipErrorInvalidValue;
          else conv_lds_kernel<WM, WN, OA, OB, EPI_NONE, OUT_F32, DGRAD, NS, 6><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb);
          break;
        case 8: conv_lds_kernel<WM, WN, OA, OB, EPI_NONE, OUT_F32, DGRAD, NS, 8><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb); break;
        case 16: conv_lds_kernel<WM, WN, OA, OB, EPI_NONE, OUT_F32, DGRAD, NS, 16><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb); break;
        case 32: conv_lds_kernel<WM, WN, OA, OB, EPI_NONE, OUT_F32, DGRAD, NS, 32><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
#define CONV_LDS_CASE(E)                                                                                      \
  conv_lds_kernel<WM, WN, OA, OB, E, OUT_F32, DGRAD, NS><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, \
                                                                                  (uint32_t)bb)
  switch (epi) {
    case EPI_NONE:
      CONV_LDS_CASE(EPI_NONE);
      break;
    case EPI_BIAS:
      if constexpr (OUT_F32) return hipErrorInvalidValue;
      else CONV_LDS_CASE(EPI_BIAS);
      break;
    case EPI_BIAS_RELU:
      if constexpr (OUT_F32) return hipErrorInvalidValue;
      else CONV_LDS_CASE(EPI_BIAS_RELU);
      break;
    default:
      return hipErrorInvalidValue;
  }
#undef CONV_LDS_CASE
  return hipGetLastError();
}

template <int WM, int WN, class OA, class OB, bool OUT_F32, bool DGRAD>
hipError_t launch(LArgs a, int epi, int splits, const bf16_t* pa, size_t ba, const bf16_t* pb, size_t bb,
                  hipStream_t st) {
  return launch_ns<WM, WN, OA, OB, OUT_F32, DGRAD, 2>(a, epi, splits, pa, ba, pb, bb, st);
}

// Halo path (conv_halo_kernel) for 3x3 stride-1 pad-1 fwd / dgrad.  LDNN_CONV_HALO
// (A/B knob): 0 off; 1 (default) the 256x64 tiles of 64-channel layers only (there the
// activation tile is 4/5 of the gather kernel's fill and one channel block is loaded
// once); 2 the 128x128 tiles too (slower: there the weight tile dominates the fill and
// the per-block halo reload stalls, profiles/conv_halo_micro_r2.txt).
int g_conv_halo = -2;  // -2: not read yet
int halo_env() {
  if (g_conv_halo == -2) g_conv_halo = env_int("LDNN_CONV_HALO", 1);
  return g_conv_halo;
}
bool halo_ok(const ConvShape& s) {
  return halo_env() != 0 && s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.P == s.H && s.Q == s.W &&
         ((2 * s.W + 2 + 7) & ~7) <= kHaloExtra;
}
// the halo path takes this plan (wm: its wave rows, 4 = 256x64 tiles, 2 = 128x128)
bool halo_takes(const ConvShape& s, int wm) {
  if (!halo_ok(s)) return false;
  const int m = halo_env();
  if (wm == 4) return m != 0;
  return m == 2;
}

// Weight-stationary path (conv_ws64_kernel) for 64 -> 64 channel 3x3 stride-1 pad-1 fwd
// (no bias) and dgrad, and conv_patch_ws_kernel for the 64-filter 7x7 / 2 stem.  LDNN_CONV_WS=0
// (A/B knob) turns both off (conv_halo_kernel / conv_patch_kernel).
int g_conv_ws = -2;  // -2: not read yet
int ws_env() {
  if (g_conv_ws == -2) g_conv_ws = env_int("LDNN_CONV_WS", 1);
  return g_conv_ws;
}
bool ws64_takes(const ConvShape& s, int epi) {
  return ws_env() != 0 && epi == EPI_NONE && s.C == 64 && s.K == 64 && s.R == 3 && s.S == 3 && s.stride == 1 &&
         s.pad == 1 && s.P == s.H && s.Q == s.W && s.W <= 63;
}
int cu_count() {
  static int n[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (n[dev] == 0) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
    n[dev] = v;
  }
  return n[dev];
}
template <int RT, bool DGRAD>
hipError_t launch_ws64_m(LArgs a, int grid, const bf16_t* pa, size_t ba, const bf16_t* pw, hipStream_t st) {
  a.tiles_x = grid;
  const int xf = conv_xf_env();
  if (xf == 32) {
    conv_ws64_kernel<RT, DGRAD, 32><<<grid, 256, 0, st>>>(a, pa, (uint32_t)ba, pw);
  } else
    conv_ws64_kernel<RT, DGRAD><<<grid, 256, 0, st>>>(a, pa, (uint32_t)ba, pw);
  return hipGetLastError();
}
// 128-row tiles (RT 4).  (256-row tiles, RT 8, need ~290 live registers per lane; hipcc spilled
// them and the dgrad variant read corrupted B fragments -- removed.)
template <bool DGRAD>
hipError_t launch_ws64(const LArgs& a, const bf16_t* pa, size_t ba, const bf16_t* pw, hipStream_t st) {
  const int64_t tiles = (a.M + 127) / 128;
  return launch_ws64_m<4, DGRAD>(a, (int)std::min<int64_t>(tiles, cu_count()), pa, ba, pw, st);
}

template <int WM, int WN, class OB, bool DGRAD>
hipError_t launch_halo(LArgs a, int epi, int splits, const bf16_t* pa, size_t ba, const bf16_t* pb, size_t bb,
                       hipStream_t st) {
  a.tap_major = 1;  // taps fastest inside a channel block: one halo per block
  dim3 grid(a.tiles_x, splits, 1), block(256);
  if (conv_xf_env() == 32 && epi == EPI_NONE) {
    conv_halo_kernel<WM, WN, OB, EPI_NONE, DGRAD, 32><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb);
    return hipGetLastError();
  }
#define HALO_CASE(E) \
  conv_halo_kernel<WM, WN, OB, E, DGRAD><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb)
  switch (epi) {
    case EPI_NONE: HALO_CASE(EPI_NONE); break;
    case EPI_BIAS: HALO_CASE(EPI_BIAS); break;
    case EPI_BIAS_RELU: HALO_CASE(EPI_BIAS_RELU); break;
    default: return hipErrorInvalidValue;
  }
#undef HALO_CASE
  return hipGetLastError();
}

// Big-tile halo path (conv_hb_kernel) for 3x3 stride-1 pad-1 fwd / dgrad with 64-multiple input
// and 128-multiple output channels, W <= 32 (ResNet-18 layers 2-4, EnhancedCNN's stages).
// LDNN_CONV_HB (documented fallback): 0 off; 1 (default) dgrad grids of >= 96 tiles.  (Test hooks
// only, set_conv_hb: 2 fwd too; 3 every eligible shape.)  Measured (scripts/conv_micro.py, profiles/r5/conv_hb_micro.jsonl): the dgrad
// wins at ResNet-18 b256 (C128 H28 108 -> 102 us, C256 H14 100 -> 93, C512 H7 104 -> 94) and
// b64 C128 H28 (28.6 -> 26.5); the fwd loses to the gather kernel (C128 H28 b256 79 -> 94 us) and
// the small split-K grids (EnhancedCNN b64) lose both ways.
int g_conv_hb = -2;  // -2: not read yet
int hb_env() {
  if (g_conv_hb == -2) g_conv_hb = env_int("LDNN_CONV_HB", 1) != 0 ? 1 : 0;
  return g_conv_hb;
}
bool hb_takes(const ConvShape& s, bool dgrad) {
  const int m = hb_env();
  const int cin = dgrad ? s.K : s.C, cout = dgrad ? s.C : s.K;
  if (m == 0 || (m == 1 && !dgrad)) return false;
  if (!(s.R == 3 && s.S == 3 && s.stride == 1 && s.pad == 1 && s.P == s.H && s.Q == s.W && s.W <= hb::kMaxW &&
        cin % 64 == 0 && cout % 128 == 0))
    return false;
  const int64_t tiles = ((int64_t)s.N * s.H * s.W + hb::kBM - 1) / hb::kBM * (cout / hb::kBN);
  return m == 3 || tiles >= 96;
}

template <class OB, bool DGRAD>
hipError_t launch_hb(LArgs a, int epi, int splits, const bf16_t* pa, size_t ba, const bf16_t* pb, size_t bb,
                     hipStream_t st) {
  a.tap_major = 1;  // taps fastest inside a channel block: one halo per block
  dim3 grid(a.tiles_x, splits, 1), block(hb::kNT);
#define HB_CASE(E) conv_hb_kernel<OB, E, DGRAD><<<grid, block, 0, st>>>(a, pa, (uint32_t)ba, pb, (uint32_t)bb)
  switch (epi) {
    case EPI_NONE: HB_CASE(EPI_NONE); break;
    case EPI_BIAS:
      if constexpr (DGRAD) return hipErrorInvalidValue;
      else HB_CASE(EPI_BIAS);
      break;
    case EPI_BIAS_RELU:
      if constexpr (DGRAD) return hipErrorInvalidValue;
      else HB_CASE(EPI_BIAS_RELU);
      break;
    default: return hipErrorInvalidValue;
  }
#undef HB_CASE
  return hipGetLastError();
}

// LDNN_CONV_SLAB=0 (documented fallback): small-M fwd / dgrad use the in-launch combine
bool slab_env_off() {
  static const bool v = env_int("LDNN_CONV_SLAB", 1) == 0;
  return v;
}

// In-launch split-K for small-M fwd / dgrad (below 256 tiles: ResNet-18's 14x14
// stage, 196 tiles, A/B 3.76 -> 3.68 ms at b64, profiles/cnn_split_tiles_ab_r2.jsonl):
// enough slices for ~1.5 workgroups per CU, >= 8 K-tiles each, at most 8.
int small_m_splits(int tiles, int nk) {
  if (tiles >= 256 || nk < 16) return 1;
  constexpr int target = 384;  // workgroups to aim for
  int sp = (target + tiles - 1) / tiles;
  sp = std::min(sp, nk / 8);
  sp = std::min(sp, 8);
  return sp < 2 ? 1 : sp;
}

// Slab split-K for small-M fwd / stride-1 dgrad: the splits write fp32 slabs and a
// chip-wide kernel sums them, so a deep split costs no per-tile serial combine:
// ~2 workgroups per CU (the weights of a 2x2 / 4x4 tail stage stream from HBM at
// the per-CU rate, so the more CUs read them the sooner they land), >= 3 K-tiles
// per slice, at most 32 slices.
int slab_splits(int tiles, int nk) {
  if (tiles >= 160 || nk < 8) return 1;
  // (256 since conv GEMMs share launches: EnhancedCNN b64 -1.2 %, ResNet-18 neutral,
  // profiles/r5/conv_split_knobs_ab.txt)
  constexpr int target = 256;  // workgroups to aim for
  constexpr int min_kt = 3;    // K-tiles per slice at least
  int sp = (target + tiles - 1) / tiles;
  sp = std::min(sp, nk / std::max(1, min_kt));
  sp = std::min(sp, 32);
  return sp < 2 ? 1 : sp;
}

struct Plan {
  int wm, wn;  // wave grid (tile = 64*wm x 64*wn)
  int tiles_x, classes, splits, nk_all, nk_split;
  bool slab;   // split-K via fp32 slabs + conv_slab_epilogue (else the in-launch combine)
  int M, N;    // GEMM output (slab size)
};

void finish_plan(Plan& p) {
  // slabs only for the deep tails (< 48 output tiles): measured on MI355X at 64 - 160
  // tiles (EnhancedCNN 8x8 / 16x16 stages, ResNet-18 7x7) the slab traffic cost what
  // the in-launch combine does (ResNet-18 b64 3.94 vs 3.89 ms), at 16 / 32 tiles the
  // slabs win (EnhancedCNN 4x4 / 2x2 convs 28 / 38 -> 25 / 28 us)
  constexpr int slab_tiles = 48;
  p.slab = p.classes == 1 && p.tiles_x < slab_tiles && !slab_env_off();
  p.splits = p.slab ? slab_splits(p.tiles_x, p.nk_all) : small_m_splits(p.tiles_x * p.classes, p.nk_all);
  p.nk_split = (p.nk_all + p.splits - 1) / p.splits;
  p.splits = (p.nk_all + p.nk_split - 1) / p.nk_split;
  if (p.splits < 2) p.slab = false;
}

Plan plan_fwd(const ConvShape& s) {
  Plan p{};
  p.classes = 1;
  if (s.K <= 64) { p.wm = 4; p.wn = 1; } else { p.wm = 2; p.wn = 2; }
  const int M = s.N * s.P * s.Q;
  p.tiles_x = ((M + p.wm * 64 - 1) / (p.wm * 64)) * ((s.K + p.wn * 64 - 1) / (p.wn * 64));
  p.nk_all = s.R * s.S * s.C / 64;
  p.M = M;
  p.N = s.K;
  finish_plan(p);
  return p;
}

Plan plan_dgrad(const ConvShape& s) {
  Plan p{};
  if (s.C <= 64) { p.wm = 4; p.wn = 1; } else { p.wm = 2; p.wn = 2; }
  const int tn = (s.C + p.wn * 64 - 1) / (p.wn * 64);
  const int nb = s.K / 64;
  if (s.stride == 2) {
    p.classes = 4;  // class (0, 0) has the most rows, a class with r0 = s0 = 0 the most taps
    const int h0 = (s.H + 1) >> 1, w0 = (s.W + 1) >> 1;
    p.tiles_x = ((s.N * h0 * w0 + p.wm * 64 - 1) / (p.wm * 64)) * tn;
    p.nk_all = ((s.R + 1) >> 1) * ((s.S + 1) >> 1) * nb;
  } else {
    p.classes = 1;
    p.tiles_x = ((s.N * s.H * s.W + p.wm * 64 - 1) / (p.wm * 64)) * tn;
    p.nk_all = s.R * s.S * nb;
  }
  p.M = s.N * s.H * s.W;
  p.N = s.C;
  finish_plan(p);
  return p;
}

// conv_hb_kernel: 256 x 128 tiles (4 x 2 waves); a split-K slice holds whole channel blocks.
// Split only grids below ~3/4 of a workgroup per CU, to ~one workgroup per CU.
Plan plan_hb(const ConvShape& s, bool dgrad) {
  Plan p{};
  p.wm = 4;
  p.wn = 2;
  p.classes = 1;
  const int cin = dgrad ? s.K : s.C, cout = dgrad ? s.C : s.K;
  p.M = s.N * s.H * s.W;
  p.N = cout;
  p.tiles_x = ((p.M + hb::kBM - 1) / hb::kBM) * (cout / hb::kBN);
  const int nblk = cin / 64;
  p.nk_all = 9 * nblk;
  constexpr int target = 256;  // workgroups to aim for
  int sp = 1;
  if (p.tiles_x < 192) sp = std::min(nblk, std::max(1, (target + p.tiles_x - 1) / p.tiles_x));
  const int bps = (nblk + sp - 1) / sp;  // channel blocks per slice
  p.nk_split = 9 * bps;
  p.splits = (nblk + bps - 1) / bps;
  p.slab = p.splits > 1 && p.tiles_x < 48 && !slab_env_off();
  return p;
}

constexpr int kSlabBytes8 = 16 * 512 * 16;  // one 8-wave workgroup's fp32 accumulators

ConvWorkspace ws_of(const Plan& p) {
  ConvWorkspace w{};
  if (p.splits > 1 && p.slab) {
    w.slab_bytes = (size_t)p.splits * p.M * p.N * 4;
  } else if (p.splits > 1) {
    w.slab_bytes = (size_t)p.tiles_x * p.classes * p.splits * (p.wm * p.wn == 8 ? kSlabBytes8 : kSlabBytes4);
    w.counters = p.tiles_x * p.classes;
  }
  return w;
}

}  // namespace convlds

using namespace convlds;

void set_conv_halo(int mode) { g_conv_halo = mode; }
void set_conv_hb(int mode) { g_conv_hb = mode; }
int get_conv_hb() { return hb_env(); }
void set_conv_ws(int mode) { g_conv_ws = mode; }
int get_conv_ws() { return ws_env(); }
void set_conv_trace(uint64_t* buf) { g_conv_trace = buf; }
void set_conv_bn_bwd(int mode) { g_bn_bwd = mode; }
int get_conv_bn_bwd() { return bn_bwd_env(); }

void set_conv_combine_last(int on) { g_combine_last = on; }
int get_conv_combine_last() { return g_combine_last; }
void set_conv_wgrad_ring(int mode) { g_wgrad_ring = mode; }
int get_conv_halo() { return halo_env(); }

ConvWorkspace conv2d_lds_workspace(const ConvShape& s, int op) {
  if (!shape_ok(s)) return ConvWorkspace{};
  if (op == 2 && stem_s2d_ok(s)) {
    ConvWorkspace w{};
    w.slab_bytes = stem_s2d_ws_bytes(s);
    return w;
  }
  if (op == 0 && s.C % 64 == 0) return ws_of(hb_takes(s, false) ? plan_hb(s, false) : plan_fwd(s));
  // dgrad / wgrad: the larger of the layer's own plan and the generic one a paired launch may
  // take instead (conv2d_bwd_lds with LDNN_CONV_PAIR=2)
  if (op == 1 && s.K % 64 == 0) {
    ConvWorkspace w = ws_of(plan_dgrad(s));
    if (hb_takes(s, true)) {
      const ConvWorkspace h = ws_of(plan_hb(s, true));
      w.slab_bytes = std::max(w.slab_bytes, h.slab_bytes);
      w.counters = std::max(w.counters, h.counters);
    }
    return w;
  }
  if (op == 2 && s.C % 8 == 0 && s.K % 8 == 0) {
    ConvWorkspace w{};
    for (int ring = 0; ring < 2; ++ring) {
      const WgradPlan p = plan_wgrad(s, ring != 0);
      if (p.splits > 1) w.slab_bytes = std::max(w.slab_bytes, (size_t)p.splits * s.K * s.R * s.S * s.C * 4);
    }
    return w;
  }
  return ConvWorkspace{};
}

hipError_t slab_sum(const float* ws, float* out, int64_t n4, int splits, float beta, hipStream_t st) {
  if (n4 <= 0) return hipSuccess;
  slab_sum_kernel<true><<<(unsigned)((n4 + 31) / 32), 256, 0, st>>>(ws, out, n4, splits, beta);
  return hipGetLastError();
}

// Each returns hipErrorNotSupported when the shape is outside the fast path
// (conv.hip then runs its generic register-staged kernel).
// Stems and other small-C convolutions (C in {8, 16, 32}, e.g. the 7x7 ResNet stem
// on 3 -> 8 padded channels): K-tiles span several taps, one 256x64 / 128x128 tile.
hipError_t conv2d_fwd_lds_small_c(const ConvShape& s, const uint16_t* x, const uint16_t* w, uint16_t* y,
                                  const float* bias, int epi, hipStream_t st, const BnFin* bn, uint16_t* s2d_xs) {
  LArgs a = base_args(s);
  if (bn != nullptr && epi == EPI_NONE) {
    a.bn_stats = 1;
    a.bn = *bn;
  }
  a.out = y;
  a.bias = bias;
  a.M = s.N * s.P * s.Q;
  a.N = s.K;
  a.nb = 0;
  a.taps_per_tile = 64 / s.C;
  a.f_s = make_fastdiv(s.S);
  a.nk_all = (a.rsc + 63) / 64;
  a.nk_split = a.nk_all;
  const bool narrow = s.K <= 64;
  a.tiles_x = ((a.M + (narrow ? 255 : 127)) / (narrow ? 256 : 128)) * ((s.K + (narrow ? 63 : 127)) / (narrow ? 64 : 128));
  const size_t bx = (size_t)s.N * s.H * s.W * s.C * 2, bw = (size_t)s.K * a.rsc * 2;
  if (s2d_xs != nullptr) {   // the caller keeps the packed image for the weight gradient (conv_stem.hip)
    if (epi != EPI_NONE || !stem_s2d_fwd_ok(s)) return hipErrorInvalidValue;
    return stem_s2d_fwd(a, x, w, s2d_xs, st);
  }
  if (patch_ok(s)) return launch_patch(a, epi, x, bx, w, st);
  if (narrow) return launch<4, 1, FwdASmallC<256, 8, 4>, WeightKC<64, 2, 4>, false, false>(a, epi, 1, x, bx, w, bw, st);
  return launch<2, 2, FwdASmallC<128, 4, 4>, WeightKC<128, 4, 4>, false, false>(a, epi, 1, x, bx, w, bw, st);
}

namespace {
// Post passes gathered for one conv_post_kernel launch (post_flush).
struct PostBatch {
  PostTask t[4] = {};
  int n = 0, blocks = 0;
  void push(PostTask task) {
    task.start = blocks;
    blocks += task.gx * task.gy;
    t[n++] = task;
  }
};
PostTask slab_bn_task(const float* ws, uint16_t* out, int M, int N, int splits, const BnFin& fin,
                      const BnBwdFuse* bnb) {
  constexpr int target = kSlabBnTarget;
  const int G = (N + 63) / 64;
  int ny = std::max(1, std::min({(target + G - 1) / G, (M + 31) / 32, kGrpMax}));
  const int rpb = (M + ny - 1) / ny;
  ny = (M + rpb - 1) / rpb;
  PostTask t{};
  t.kind = bnb != nullptr ? PK_BN_BWD : PK_BN_FWD;
  t.gx = G;
  t.gy = ny;
  t.ws = ws;
  t.out = out;
  t.M = M;
  t.N = N;
  t.splits = splits;
  t.rpb = rpb;
  t.fin = fin;
  if (bnb != nullptr) {
    t.bx = bnb->x;
    t.mask = bnb->mask;
  }
  return t;
}
PostTask slab_epi_task(const float* ws, uint16_t* out, int M, int N, int splits) {
  PostTask t{};
  t.kind = PK_EPI;
  t.n = (int64_t)M * N / 8;
  t.gx = (int)((t.n + 255) / 256);
  t.gy = 1;
  t.ws = ws;
  t.out = out;
  t.N = N;
  t.splits = splits;
  return t;
}
PostTask slab_sum_task(const float* ws, float* out, int64_t n4, int splits, float beta) {
  PostTask t{};
  t.kind = PK_SUM;
  t.n = n4;
  t.gx = (int)((n4 + 31) / 32);
  t.gy = 1;
  t.ws = ws;
  t.out = out;
  t.splits = splits;
  t.beta = beta;
  return t;
}
// every post task of a conv step in ONE launch (measured 1-2 % faster than a launch per task,
// profiles/r5/conv_post_merge_ab.txt)
hipError_t post_flush(const PostBatch& pb, hipStream_t st) {
  if (pb.n == 0 || pb.blocks == 0) return hipSuccess;
  conv_post_kernel<true><<<(unsigned)pb.blocks, 256, 0, st>>>(pb.t[0], pb.t[1], pb.t[2], pb.t[3]);
  return hipGetLastError();
}
}  // namespace

namespace {
// What conv2d_fwd_lds launches for a C % 64 == 0 shape, planned without launching it.
struct FwdPrep {
  LArgs a;
  Plan pl;
  bool slab, hb, halo, ws64;
  const BnFin* slab_fin;
  bool bn_used;
  size_t bx, bw;
};

FwdPrep fwd_prep(const ConvShape& s, uint16_t* y, const float* bias, int epi, float* ws, int* cnt, const BnFin* bn) {
  FwdPrep f{};
  f.bn_used = bn != nullptr;
  f.hb = hb_takes(s, false);
  Plan& pl = f.pl;
  pl = f.hb ? plan_hb(s, false) : plan_fwd(s);
  LArgs& a = f.a;
  a = base_args(s);
  // the weight-stationary 64 -> 64 kernel runs unsplit on a persistent grid and takes the BN
  // statistics in its own epilogue, whatever the plan says for the gather kernels (with the slab
  // hand-off below its small-M launches -- ResNet-18 at 64 x 64 inputs -- took them nowhere)
  f.ws64 = ws64_takes(s, epi);
  // slab split-K: the slab pass takes the next BN's statistics (conv_slab_bn), or with
  if (bn != nullptr && pl.slab && pl.splits > 1 && ws != nullptr && !f.ws64) {   // (the slab pass will run)
    if (bn->part != nullptr && bn->tickets != nullptr && s.K % 8 == 0) f.slab_fin = bn;
    else f.bn_used = false;
    bn = nullptr;
  }
  if (bn != nullptr) {
    a.bn_stats = 1;
    a.bn = *bn;
  }
  a.out = y;
  a.bias = bias;
  a.M = s.N * s.P * s.Q;
  a.N = s.K;
  a.nb = s.C / 64;
  a.tiles_x = pl.tiles_x;
  a.nk_all = pl.nk_all;
  f.slab = pl.splits > 1 && pl.slab && ws != nullptr;
  if (f.slab) {
    a.ws = ws;
    a.nk_split = pl.nk_split;
  } else if (pl.splits > 1 && !pl.slab && ws != nullptr && cnt != nullptr) {
    a.ws = ws;
    a.cnt = cnt;
    a.nk_split = pl.nk_split;
  } else {
    pl.splits = 1;
    a.nk_split = pl.nk_all;
  }
  f.bx = (size_t)s.N * s.H * s.W * s.C * 2;
  f.bw = (size_t)s.K * a.rsc * 2;
  if (f.ws64) {  // persistent grid, no split-K: the plan's slab / combine is not used
    f.slab = false;
    a.ws = nullptr;
    a.cnt = nullptr;
    a.nk_split = a.nk_all;
  }
  f.halo = !f.ws64 && !f.hb && halo_takes(s, pl.wm);
  return f;
}

// the same as a post task (bias-free EPI_NONE convs; conv2d_fwd2_lds)
void fwd_post_task(const FwdPrep& f, uint16_t* y, float* ws, PostBatch& pb) {
  if (!f.slab) return;
  if (f.slab_fin != nullptr) pb.push(slab_bn_task(ws, y, f.a.M, f.a.N, f.pl.splits, *f.slab_fin, nullptr));
  else pb.push(slab_epi_task(ws, y, f.a.M, f.a.N, f.pl.splits));
}

// after the main kernel: the slab split-K sum (with the next BN's statistics when taken)
hipError_t fwd_post(const FwdPrep& f, uint16_t* y, const float* bias, int epi, float* ws, hipStream_t st) {
  if (!f.slab) return hipSuccess;
  if (f.slab_fin != nullptr) return conv_slab_bn(ws, y, f.a.M, f.a.N, f.pl.splits, *f.slab_fin, st);
  return conv_slab_epilogue(ws, y, f.a.M, f.a.N, f.pl.splits, bias, epi, st);
}
}  // namespace

hipError_t conv2d_fwd_lds(const ConvShape& s, const uint16_t* x, const uint16_t* w, uint16_t* y, const float* bias,
                          int epi, hipStream_t st, float* ws, int* cnt, const BnFin* bn, bool* bn_used,
                          uint16_t* s2d_xs) {
  if (bn_used) *bn_used = bn != nullptr;
  if (!shape_ok(s)) return s2d_xs ? hipErrorInvalidValue : hipErrorNotSupported;
  if (bn != nullptr && epi != EPI_NONE) return hipErrorInvalidValue;
  if (s.C == 8 || s.C == 16 || s.C == 32) {
    if (s.N * s.P * s.Q <= 0) return s2d_xs ? hipErrorInvalidValue : hipErrorNotSupported;
    return conv2d_fwd_lds_small_c(s, x, w, y, bias, epi, st, bn, s2d_xs);
  }
  if (s2d_xs != nullptr) return hipErrorInvalidValue;
  if (s.C % 64 != 0) return hipErrorNotSupported;
  if (s.N * s.P * s.Q <= 0) return bn != nullptr ? hipErrorNotSupported : hipSuccess;
  const FwdPrep f = fwd_prep(s, y, bias, epi, ws, cnt, bn);
  if (bn_used) *bn_used = f.bn_used;
  const LArgs& a = f.a;
  const int splits = f.pl.splits;
  if (f.ws64) return launch_ws64<false>(a, x, f.bx, w, st);
  hipError_t e;
  if (f.hb) {
    e = launch_hb<WeightKC<128, 2, 8>, false>(a, epi, splits, x, f.bx, w, f.bw, st);
  } else if (f.halo) {
    // fwd: the halo wins on the 256x64 tiles of 64-filter layers (C64 H56: 53.7 -> 35-37 us) and
    // loses on 128x128 ones (C128 H28 25.8 -> 27.7, C512 H7 34.9 -> 40.0 us; double-buffered too)
    if (f.pl.wm == 4) e = launch_halo<4, 1, WeightKC<64, 2, 4>, false>(a, epi, splits, x, f.bx, w, f.bw, st);
    else e = launch_halo<2, 2, WeightKC<128, 4, 4>, false>(a, epi, splits, x, f.bx, w, f.bw, st);
  } else if (f.pl.wm == 4) {
    e = launch<4, 1, FwdA<256, 8, 4>, WeightKC<64, 2, 4>, false, false>(a, epi, splits, x, f.bx, w, f.bw, st);
  } else {
    e = launch<2, 2, FwdA<128, 4, 4>, WeightKC<128, 4, 4>, false, false>(a, epi, splits, x, f.bx, w, f.bw, st);
  }
  if (e != hipSuccess) return e;
  return fwd_post(f, y, bias, epi, ws, st);
}

namespace {
// What conv2d_dgrad_lds launches, planned without launching it (conv2d_bwd_lds can then
// issue the main kernel together with the wgrad's).
struct DgradPrep {
  LArgs a;
  Plan pl;
  bool slab, hb, halo, ws64;
  bool ws64_bnb;              // the weight-stationary dgrad's epilogue takes the BN backward statistics
  const BnBwdFuse* slab_bnb;
  const BnBwdFuse* red_bnb;   // no slabs: the BN statistics as a post task over dx (paired launches)
  size_t bdy, bw;
};

// generic: 1 = no big-tile halo kernel, 2 = the 4-wave gather kernel only (no big-tile / halo /
// weight-stationary variant)
DgradPrep dgrad_prep(const ConvShape& s, uint16_t* dx, float* ws, int* cnt, const BnBwdFuse* bnb,
                     int generic = 0) {
  DgradPrep d{};
  d.hb = !generic && hb_takes(s, true);
  Plan& pl = d.pl;
  pl = d.hb ? plan_hb(s, true) : plan_dgrad(s);
  LArgs& a = d.a;
  a = base_args(s);
  a.out = dx;
  a.M = s.N * s.H * s.W;
  a.N = s.C;
  a.nb = s.K / 64;
  a.classes = pl.classes;
  a.tiles_x = pl.tiles_x;
  a.nk_all = pl.nk_all;
  d.slab = pl.splits > 1 && pl.slab && ws != nullptr;
  if (d.slab) {
    a.ws = ws;
    a.nk_split = pl.nk_split;
  } else if (pl.splits > 1 && !pl.slab && ws != nullptr && cnt != nullptr) {
    a.ws = ws;
    a.cnt = cnt;
    a.nk_split = pl.nk_split;
  } else {
    pl.splits = 1;
    a.nk_split = pl.nk_all;
  }
  d.bdy = (size_t)s.N * s.P * s.Q * s.K * 2;
  d.bw = (size_t)s.K * a.rsc * 2;
  d.ws64 = generic < 2 && ws64_takes(s, EPI_NONE);
  if (d.ws64) {
    d.slab = false;
    a.ws = nullptr;
    a.cnt = nullptr;
    a.nk_split = a.nk_all;
    // the BN backward statistics in the persistent epilogue (per-lane sums over all of the
    // workgroup's tiles, one atomic pair per channel per workgroup, as its forward does)
    if (bnb != nullptr && bn_bwd_env() == 1 && bnb->fin.acc != nullptr && bnb->fin.ticket != nullptr &&
        bnb->fin.save_mean != nullptr && bnb->fin.save_invstd != nullptr && bnb->x != nullptr) {
      a.bn_stats = 1;
      a.bn = bnb->fin;
      a.bnb_x = reinterpret_cast<const bf16_t*>(bnb->x);
      a.bnb_mask = bnb->mask;
      d.ws64_bnb = true;
    }
    return d;
  }
  d.halo = generic < 2 && !d.hb && halo_takes(s, pl.wm);
  // the BN backward statistics of the BN whose output's gradient dx is: stride-1 dgrads (no
  // class row remap) in the direct / in-launch combine epilogue, or in the slab sum
  if (bnb != nullptr && bn_bwd_env() && s.stride == 1 && pl.classes == 1 && s.C % 8 == 0 &&
      bnb->fin.part != nullptr && bnb->fin.tickets != nullptr) {
    if (d.slab) d.slab_bnb = bnb;
    else d.red_bnb = bnb;
  }
  return d;
}

// the same as a post task (conv2d_bwd_lds / conv2d_bwd2_lds)
void dgrad_post_task(const DgradPrep& d, uint16_t* dx, float* ws, PostBatch& pb, bool* bn_used) {
  if (!d.slab) {
    if (d.red_bnb != nullptr) {   // the BN's backward statistics over dx, beside the other post passes
      PostTask t = slab_bn_task(nullptr, dx, d.a.M, d.a.N, 0, d.red_bnb->fin, d.red_bnb);
      t.kind = PK_BN_BWD_RED;
      // the BN reduce's own row grouping (bn_pool.hip grp_geo): >= 256 rows per group, ~512 workgroups
      const int M = d.a.M, G = t.gx;
      int ny = std::max(1, std::min({(512 + G - 1) / G, M / 256, kGrpMax}));
      t.rpb = (M + ny - 1) / ny;
      t.gy = (M + t.rpb - 1) / t.rpb;
      pb.push(t);
      if (bn_used) *bn_used = true;
      return;
    }
    return;
  }
  if (d.slab_bnb != nullptr) {
    if (bn_used) *bn_used = true;
    pb.push(slab_bn_task(ws, dx, d.a.M, d.a.N, d.pl.splits, d.slab_bnb->fin, d.slab_bnb));
    return;
  }
  pb.push(slab_epi_task(ws, dx, d.a.M, d.a.N, d.pl.splits));
}

// after the main kernel: the slab split-K sum (with the BN statistics when taken)
hipError_t dgrad_post(const DgradPrep& d, uint16_t* dx, float* ws, hipStream_t st, bool* bn_used) {
  if (!d.slab) {   // (the BN backward statistics, when taken: one pass over dx)
    if (d.red_bnb == nullptr) return hipSuccess;
    PostBatch pb;
    dgrad_post_task(d, dx, ws, pb, bn_used);
    return post_flush(pb, st);
  }
  if (d.slab_bnb != nullptr) {
    if (bn_used) *bn_used = true;
    return conv_slab_bn(ws, dx, d.a.M, d.a.N, d.pl.splits, d.slab_bnb->fin, st, d.slab_bnb);
  }
  return conv_slab_epilogue(ws, dx, d.a.M, d.a.N, d.pl.splits, nullptr, EPI_NONE, st);
}
}  // namespace

hipError_t conv2d_dgrad_lds(const ConvShape& s, const uint16_t* dy, const uint16_t* w, uint16_t* dx, hipStream_t st,
                            float* ws, int* cnt, const BnBwdFuse* bnb, bool* bn_used) {
  if (bn_used) *bn_used = false;
  if (s.K % 64 != 0 || !shape_ok(s)) return hipErrorNotSupported;
  if (s.N * s.H * s.W <= 0) return hipSuccess;
  const DgradPrep d = dgrad_prep(s, dx, ws, cnt, bnb);
  const LArgs& a = d.a;
  const int splits = d.pl.splits;
  if (d.ws64) {
    if (bn_used) *bn_used = d.ws64_bnb;
    return launch_ws64<true>(a, dy, d.bdy, w, st);
  }
  hipError_t e;
  if (d.hb) {
    e = launch_hb<DgradB<128, 2, 8>, true>(a, EPI_NONE, splits, dy, d.bdy, w, d.bw, st);
  } else if (d.halo) {
    // dgrad likewise: C64 H56 38.9 -> 36.5 us; single-buffered on 128x128 tiles neutral to 1 us
    // slower (ResNet-18 C128-C512), up to 2.6 us slower on the EnhancedCNN 16x16 .. 2x2 stages
    if (d.pl.wm == 4) e = launch_halo<4, 1, DgradB<64, 2, 4>, true>(a, EPI_NONE, splits, dy, d.bdy, w, d.bw, st);
    else e = launch_halo<2, 2, DgradB<128, 4, 4>, true>(a, EPI_NONE, splits, dy, d.bdy, w, d.bw, st);
  } else if (d.pl.wm == 4) {
    e = launch<4, 1, DgradA<256, 8, 4>, DgradB<64, 2, 4>, false, true>(a, EPI_NONE, splits, dy, d.bdy, w, d.bw, st);
  } else {
    e = launch<2, 2, DgradA<128, 4, 4>, DgradB<128, 4, 4>, false, true>(a, EPI_NONE, splits, dy, d.bdy, w, d.bw, st);
  }
  if (e != hipSuccess) return e;
  return dgrad_post(d, dx, ws, st, bn_used);
}

namespace {
// The 4-wave gather wgrad's launch (conv2d_wgrad_lds), planned without launching it.
struct WgradPrep {
  LArgs a;
  int splits;
  bool slab;
  size_t bdy, bx;
};

WgradPrep wgrad_prep(const ConvShape& s, const WgradPlan& pl, float* dw, float beta, float* ws) {
  WgradPrep w{};
  LArgs& a = w.a;
  a = base_args(s);
  a.out = dw;
  a.beta = beta;
  a.M = s.K;
  a.N = a.rsc;
  a.Kd = s.N * s.P * s.Q;
  a.nk_all = pl.nk_all;
  a.nk_split = pl.nk_split;
  a.tiles_x = pl.tiles;
  a.nb = 0;
  const int pq = s.P * s.Q;
  a.dn = 64 / pq;
  a.dp = (64 % pq) / s.Q;
  a.dq = (64 % pq) % s.Q;
  a.f_pq = make_fastdiv(pq);
  a.f_q = make_fastdiv(s.Q);
  a.f_c = make_fastdiv(s.C);
  a.f_s = make_fastdiv(s.S);
  w.splits = pl.splits;
  a.xcd_split = w.splits > 1 ? 1 : 0;   // a slice's tiles on one XCD (split_coords)
  w.slab = w.splits > 1 && ws != nullptr;
  if (w.slab) a.ws = ws;  // partial slabs + slab_sum_kernel (else fp32 atomics into a cleared output)
  w.bdy = (size_t)s.N * s.P * s.Q * s.K * 2;
  w.bx = (size_t)s.N * s.H * s.W * s.C * 2;
  return w;
}

void wgrad_post_task(const WgradPrep& w, float* dw, float beta, float* ws, PostBatch& pb) {
  if (w.slab) pb.push(slab_sum_task(ws, dw, (int64_t)w.a.M * w.a.N / 4, w.splits, beta));
}

hipError_t wgrad_post(const WgradPrep& w, float* dw, float beta, float* ws, hipStream_t st) {
  if (!w.slab) return hipSuccess;
  const int64_t n4 = (int64_t)w.a.M * w.a.N / 4;
  slab_sum_kernel<true><<<(unsigned)((n4 + 31) / 32), 256, 0, st>>>(ws, dw, n4, w.splits, beta);
  return hipGetLastError();
}
}  // namespace

hipError_t conv2d_wgrad_lds(const ConvShape& s, const uint16_t* dy, const uint16_t* x, float* dw, float beta,
                            hipStream_t st, float* ws, const uint16_t* s2d_xs) {
  if (!shape_ok(s) || s.C % 8 != 0 || s.K % 8 != 0) return s2d_xs ? hipErrorInvalidValue : hipErrorNotSupported;
  if (beta != 0.f && beta != 1.f) return s2d_xs ? hipErrorInvalidValue : hipErrorNotSupported;
  if (s2d_xs != nullptr && !(stem_s2d_ok(s) && ws != nullptr)) return hipErrorInvalidValue;
  if (stem_s2d_ok(s) && ws != nullptr) return stem_s2d_wgrad(s, dy, x, dw, beta, st, ws, s2d_xs);   // conv_stem.hip
  const WgradPlan pl = plan_wgrad(s);
  if (pl.ring) {
    WRArgs r{};
    r.N = s.N; r.H = s.H; r.W = s.W; r.C = s.C; r.K = s.K;
    r.M = s.N * s.H * s.W;
    r.nk = pl.nk_all;
    r.nk_split = pl.nk_split;
    r.kbn = s.K / 64;
    r.cbn = s.C / 64;
    r.HE = (2 * s.W + 2 + 7) & ~7;
    r.f_w = make_fastdiv(s.W);
    r.f_h = make_fastdiv(s.H);
    r.beta = beta;
    const bool slab = pl.splits > 1;
    if (slab && ws == nullptr) return hipErrorNotSupported;  // (conv2d_lds_workspace sizes the slabs)
    r.out = slab ? ws : dw;
    const size_t bdy = (size_t)s.N * s.P * s.Q * s.K * 2, bx = (size_t)s.N * s.H * s.W * s.C * 2;
    wgrad_ring_kernel<<<pl.splits * pl.tiles, 256, 0, st>>>(r, dy, (uint32_t)bdy, x, (uint32_t)bx);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess || !slab) return e;
    const int64_t n4 = (int64_t)s.K * 9 * s.C / 4;
    slab_sum_kernel<true><<<(unsigned)((n4 + 31) / 32), 256, 0, st>>>(ws, dw, n4, pl.splits, beta);
    return hipGetLastError();
  }
  const WgradPrep wp = wgrad_prep(s, pl, dw, beta, ws);
  if (pl.splits > 1 && ws == nullptr && beta == 0.f) {  // no workspace: fp32 atomics into a cleared output
    hipError_t e = zero2d_f32(dw, wp.a.M, wp.a.N, wp.a.N, st);
    if (e != hipSuccess) return e;
  }
  hipError_t e;
  if (pl.narrow)
    e = launch<1, 4, WgradA<64, 2, 4>, WgradB<256, 8, 4>, true, false>(wp.a, EPI_NONE, pl.splits, dy, wp.bdy, x, wp.bx,
                                                                       st);
  else
    e = launch<2, 2, WgradA<128, 4, 4>, WgradB<128, 4, 4>, true, false>(wp.a, EPI_NONE, pl.splits, dy, wp.bdy, x,
                                                                         wp.bx, st);
  if (e != hipSuccess) return e;
  return wgrad_post(wp, dw, beta, ws, st);
}

// A layer's dgrad and wgrad (both reading dy) as ONE launch (conv_pair_kernel) when both take
// the 4-wave gather kernels; hipErrorNotSupported otherwise (the caller runs them one by one).
// LDNN_CONV_PAIR (A/B knob): 0 off; 1 pair where both GEMMs take the gather kernels anyway;
// 3 (default) also where the dgrad alone would take the big-tile halo kernel (ResNet-18 b64
// 2.697 -> 2.675 ms, b256 7.343 -> 7.315: profiles/r5/conv_pair_hb_ab.txt); 2 also instead of
// the weight-stationary dgrad and the ring wgrad (slower: profiles/r5/conv_pair_fwd_ab.txt)
int g_conv_pair = -1;
int pair_env() {
  if (g_conv_pair < 0) g_conv_pair = env_int("LDNN_CONV_PAIR", 3);
  return g_conv_pair;
}
void set_conv_pair(int on) { g_conv_pair = on; }
int get_conv_pair() { return pair_env(); }

template <int WM0, int WN0, class OA0, class OB0, bool F0, bool D0, int WM1, int WN1, class OA1, class OB1, bool F1,
          bool D1>
hipError_t launch_pair(const PairArgs& p, hipStream_t st) {
  const int n1 = p.gx[1] * p.gy[1] * p.gz[1];
  conv_pair_kernel<WM0, WN0, OA0, OB0, F0, D0, WM1, WN1, OA1, OB1, F1, D1><<<(unsigned)(p.n0 + n1), 256, 0, st>>>(p);
  return hipGetLastError();
}
#define DG128 2, 2, DgradA<128, 4, 4>, DgradB<128, 4, 4>, false, true
#define DG256 4, 1, DgradA<256, 8, 4>, DgradB<64, 2, 4>, false, true
#define WG128 2, 2, WgradA<128, 4, 4>, WgradB<128, 4, 4>, true, false
#define WGN 1, 4, WgradA<64, 2, 4>, WgradB<256, 8, 4>, true, false
#define FW128 2, 2, FwdA<128, 4, 4>, WeightKC<128, 4, 4>, false, false
#define FW256 4, 1, FwdA<256, 8, 4>, WeightKC<64, 2, 4>, false, false

hipError_t conv2d_bwd_lds(const ConvShape& sd, const uint16_t* dy, const uint16_t* w, uint16_t* dx, float* ws_d,
                          int* cnt_d, const BnBwdFuse* bnb, bool* bn_used, const ConvShape& sw, const uint16_t* x,
                          float* dw, float beta, float* ws_w, hipStream_t st) {
  if (bn_used) *bn_used = false;
  if (!pair_env() || conv_xf_env() != 0) return hipErrorNotSupported;
  if (sd.K % 64 != 0 || !shape_ok(sd) || sd.N * sd.H * sd.W <= 0) return hipErrorNotSupported;
  if (!shape_ok(sw) || sw.C % 8 != 0 || sw.K % 8 != 0 || (beta != 0.f && beta != 1.f)) return hipErrorNotSupported;
  if (stem_s2d_ok(sw)) return hipErrorNotSupported;
  // LDNN_CONV_PAIR=2: pair on the generic kernels even where a layer alone takes the big-tile /
  // weight-stationary dgrad or the ring wgrad; =3: instead of the big-tile dgrad only
  const int generic = pair_env() == 2 ? 2 : pair_env() == 3 ? 1 : 0;
  const WgradPlan pw = plan_wgrad(sw, generic < 2);
  if (pw.ring || (pw.splits > 1 && ws_w == nullptr)) return hipErrorNotSupported;
  const DgradPrep d = dgrad_prep(sd, dx, ws_d, cnt_d, bnb, generic);
  if (d.ws64 || d.hb || d.halo) return hipErrorNotSupported;
  const WgradPrep wp = wgrad_prep(sw, pw, dw, beta, ws_w);
  PairArgs p{};
  p.a[0] = d.a;
  p.a[1] = wp.a;
  p.pa[0] = reinterpret_cast<const bf16_t*>(dy);
  p.pb[0] = reinterpret_cast<const bf16_t*>(w);
  p.ba[0] = (uint32_t)d.bdy;
  p.bb[0] = (uint32_t)d.bw;
  p.pa[1] = reinterpret_cast<const bf16_t*>(dy);
  p.pb[1] = reinterpret_cast<const bf16_t*>(x);
  p.ba[1] = (uint32_t)wp.bdy;
  p.bb[1] = (uint32_t)wp.bx;
  p.gx[0] = d.a.tiles_x; p.gy[0] = d.pl.splits; p.gz[0] = d.a.classes;
  p.gx[1] = wp.a.tiles_x; p.gy[1] = pw.splits; p.gz[1] = 1;
  p.n0 = (p.gx[0] * p.gy[0] * p.gz[0] + 7) / 8 * 8;
  hipError_t e;
  if (d.pl.wm == 4) {
    if (pw.narrow) e = launch_pair<DG256, WGN>(p, st);
    else e = launch_pair<DG256, WG128>(p, st);
  } else {
    if (pw.narrow) e = launch_pair<DG128, WGN>(p, st);
    else e = launch_pair<DG128, WG128>(p, st);
  }
  if (e != hipSuccess) return e;
  // the dgrad's slab pass and the wgrad's slab sum in one launch
  PostBatch pb;
  dgrad_post_task(d, dx, ws_d, pb, bn_used);
  wgrad_post_task(wp, dw, beta, ws_w, pb);
  return post_flush(pb, st);
}

// A downsampling block's two forward convs of one input x (the 3x3 and the 1x1 shortcut) as ONE
// launch when both take the 4-wave gather kernel (EPI_NONE, each with its BN's statistics);
// hipErrorNotSupported otherwise (the caller runs them one by one).
hipError_t conv2d_fwd2_lds(const ConvShape& s0, const uint16_t* x, const uint16_t* w0, uint16_t* y0, float* ws0,
                           int* cnt0, const BnFin* bn0, bool* used0, const ConvShape& s1, const uint16_t* w1,
                           uint16_t* y1, float* ws1, int* cnt1, const BnFin* bn1, bool* used1, hipStream_t st) {
  if (used0) *used0 = false;
  if (used1) *used1 = false;
  if (!pair_env() || conv_xf_env() != 0) return hipErrorNotSupported;
  for (const ConvShape* s : {&s0, &s1})
    if (!shape_ok(*s) || s->C % 64 != 0 || s->N * s->P * s->Q <= 0) return hipErrorNotSupported;
  const FwdPrep f0 = fwd_prep(s0, y0, nullptr, EPI_NONE, ws0, cnt0, bn0);
  const FwdPrep f1 = fwd_prep(s1, y1, nullptr, EPI_NONE, ws1, cnt1, bn1);
  for (const FwdPrep* f : {&f0, &f1})
    if (f->ws64 || f->hb || f->halo) return hipErrorNotSupported;
  PairArgs p{};
  const FwdPrep* fs[2] = {&f0, &f1};
  const uint16_t* wk[2] = {w0, w1};
  for (int k = 0; k < 2; ++k) {
    p.a[k] = fs[k]->a;
    p.pa[k] = reinterpret_cast<const bf16_t*>(x);
    p.pb[k] = reinterpret_cast<const bf16_t*>(wk[k]);
    p.ba[k] = (uint32_t)fs[k]->bx;
    p.bb[k] = (uint32_t)fs[k]->bw;
    p.gx[k] = fs[k]->a.tiles_x;
    p.gy[k] = fs[k]->pl.splits;
    p.gz[k] = 1;
  }
  p.n0 = (p.gx[0] * p.gy[0] + 7) / 8 * 8;
  hipError_t e;
  if (f0.pl.wm == 4) {
    if (f1.pl.wm == 4) e = launch_pair<FW256, FW256>(p, st);
    else e = launch_pair<FW256, FW128>(p, st);
  } else {
    if (f1.pl.wm == 4) e = launch_pair<FW128, FW256>(p, st);
    else e = launch_pair<FW128, FW128>(p, st);
  }
  if (e != hipSuccess) return e;
  if (used0) *used0 = f0.bn_used;
  if (used1) *used1 = f1.bn_used;
  PostBatch pb;
  fwd_post_task(f0, y0, ws0, pb);
  fwd_post_task(f1, y1, ws1, pb);
  return post_flush(pb, st);
}

// A downsampling block's two convs of one input x, backward: both dgrads and both wgrads in ONE
// launch (conv_multi_kernel), then the dgrads' slab passes and both wgrads' slab sums in one
// (conv_post_kernel); hipErrorNotSupported where a GEMM takes another kernel.
hipError_t conv2d_bwd2_lds(const BwdJob& j0, const BwdJob& j1, const uint16_t* x, hipStream_t st) {
  if (!pair_env() || conv_xf_env() != 0) return hipErrorNotSupported;
  const BwdJob* js[2] = {&j0, &j1};
  DgradPrep d[2];
  WgradPrep w[2];
  WgradPlan pw[2];
  for (int c = 0; c < 2; ++c) {
    const BwdJob& j = *js[c];
    const ConvShape &sd = j.sd, &sw = j.sw;
    if (sd.K % 64 != 0 || !shape_ok(sd) || sd.N * sd.H * sd.W <= 0) return hipErrorNotSupported;
    if (!shape_ok(sw) || sw.C % 8 != 0 || sw.K % 8 != 0 || (j.beta != 0.f && j.beta != 1.f) || stem_s2d_ok(sw))
      return hipErrorNotSupported;
    pw[c] = plan_wgrad(sw);
    if (pw[c].ring || (pw[c].splits > 1 && j.ws_w == nullptr)) return hipErrorNotSupported;
    d[c] = dgrad_prep(sd, j.dx, j.ws_d, j.cnt_d, nullptr);
    if (d[c].ws64 || d[c].hb || d[c].halo) return hipErrorNotSupported;
    w[c] = wgrad_prep(sw, pw[c], j.dw, j.beta, j.ws_w);
  }
  MultiSlot q[4] = {};
  int at = 0;
  for (int c = 0; c < 2; ++c) {
    for (int g = 0; g < 2; ++g) {
      MultiSlot& m = q[2 * c + g];
      const bool dg = g == 0;
      m.a = dg ? d[c].a : w[c].a;
      m.pa = reinterpret_cast<const bf16_t*>(js[c]->dy);
      m.pb = reinterpret_cast<const bf16_t*>(dg ? js[c]->w : x);
      m.ba = (uint32_t)(dg ? d[c].bdy : w[c].bdy);
      m.bb = (uint32_t)(dg ? d[c].bw : w[c].bx);
      m.gx = m.a.tiles_x;
      m.gy = dg ? d[c].pl.splits : pw[c].splits;
      m.gz = dg ? d[c].a.classes : 1;
      m.kind = dg ? (d[c].pl.wm == 4 ? MK_DG256 : MK_DG128) : (pw[c].narrow ? MK_WGN : MK_WG128);
      m.start = at;
      at += (m.gx * m.gy * m.gz + 7) / 8 * 8;
    }
  }
  conv_multi_kernel<<<(unsigned)at, 256, 0, st>>>(q[0], q[1], q[2], q[3]);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  PostBatch pb;
  for (int c = 0; c < 2; ++c) dgrad_post_task(d[c], js[c]->dx, js[c]->ws_d, pb, nullptr);
  for (int c = 0; c < 2; ++c) wgrad_post_task(w[c], js[c]->dw, js[c]->beta, js[c]->ws_w, pb);
  return post_flush(pb, st);
}

}  // namespace ldnn
