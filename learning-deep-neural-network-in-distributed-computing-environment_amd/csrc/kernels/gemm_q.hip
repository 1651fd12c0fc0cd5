// Four-wave 256x256 bf16 MFMA GEMM for gfx950: the big GEMMs of the MLP step.
//
//   C[m][n] = epi( sum_k A(m,k) * B(k,n) )   fp32 accumulation; same operand
//   layouts / epilogues / GemmParams contract as gemm.hip (A_KC, B_KC, EPI_*).
//
// Design (measured on MI355X against gemm.hip's 8-wave k256 and gemm_pp.hip,
// profiles/gemm_q_r2.txt):
//  * ONE wave per SIMD, each owning a 128 x 128 block of C: 8 x 8 accumulator
//    tiles of v_mfma_f32_16x16x32_bf16 = 256 accumulator registers (AGPR half of
//    the unified 512-entry file at 1 wave/SIMD), 128 VGPRs of operand fragments.
//    Per K-tile a wave reads (128 + 128) x 64 x 2 B = 32 KiB from LDS for 2 MFLOP,
//    two thirds of the LDS traffic per FLOP of a 128x64-per-wave layout; the
//    8-wave kernels were LDS-read bound (SQ_WAIT_INST_LDS, profiles/).
//  * Software pipeline inside the wave: the K-tile is two 32-deep sub-steps; the
//    fragments of sub-step s+1 are read while the 64 MFMAs of sub-step s run
//    (two fragment register sets), so the MFMA pipe never waits on LDS.
//  * Operands HBM/L2 -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds): 2 K-tile
//    stages x (A + B) x 32 KiB = 128 KiB.  Tile t+2's DMA is issued right after
//    the one per-tile barrier (which certifies every wave finished reading the
//    stage tile t used), so a DMA has one full K-tile (~128 MFMAs per SIMD) to land.
//  * Per-tile buffer resource rebased to the K-tile (scalar), per-lane offsets
//    precomputed once: the loop issues 16 DMA instructions per wave with no
//    address VALU.  Range checking of the resource zero-fills rows past the
//    operand; a K tail (K % 64 != 0) of a k-contiguous operand is masked per slot.
//  * LDS images, fragment reads, XCD-aware tile order and the fused epilogues are
//    shared with gemm.hip (ldnn_gemm_tile.h).
#include <type_traits>

#include "ldnn_common.h"
#include "ldnn_gemm_tile.h"
#include "ldnn_kernels.h"

namespace ldnn {
namespace {
namespace kq {

constexpr int BM = 256, BN = 256;
constexpr int kThreads = 256;
constexpr int kTile = 256 * BK * 2;      // 32 KiB: one operand's K-tile
constexpr int kStage = 2 * kTile;        // A + B
constexpr int kPieces = kTile / 1024 / 4;  // 1-KiB DMA pieces per wave per operand = 8
constexpr uint32_t kOOB = 0x80000000u;

struct Op {
  const char* base;
  uint32_t bytes;            // extent of the operand (range check)
  uint32_t voff[kPieces];    // this lane's slot offset relative to the K-tile base
  int kslot;                 // k-contiguous operand: k of this lane's slot (K-tail mask)
  uint32_t kstep;            // bytes per unit of k
};

template <bool KC>
__device__ __forceinline__ void init_op(Op& op, const bf16_t* X, int ld, int rows, int K, int r0, int wid,
                                        int lane) {
  op.base = reinterpret_cast<const char*>(X);
  op.bytes = KC ? (uint32_t)((size_t)rows * ld * 2) : (uint32_t)((size_t)K * ld * 2);
  op.kstep = KC ? 2u : (uint32_t)ld * 2u;
  op.kslot = 0;
#pragma unroll
  for (int i = 0; i < kPieces; ++i) {
    int row, k;
    lds_slot_to_rk<KC, BM>((i * 4 + wid) * 1024 + lane * 16, row, k);
    const uint32_t r = (uint32_t)(r0 + row);
    op.voff[i] = KC ? (r * (uint32_t)ld + (uint32_t)k) * 2u : ((uint32_t)k * (uint32_t)ld + r) * 2u;
    if (KC) op.kslot = k;  // the same for every piece of a lane
  }
}

// DMA the K-tile at k0 of one operand into `dst` (8 x buffer_load_dwordx4 ... lds per lane).
// k0 >= kend (a prefetch past this workgroup's K range) zero-fills without reading.
template <bool KC>
__device__ __forceinline__ void issue(const Op& op, char* dst, int k0, int K, int kend, int wid) {
  const bool past = k0 >= kend;
  const uint32_t shift = past ? 0u : (uint32_t)k0 * op.kstep;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(op.base + shift), (short)0, past ? 0 : (int)(op.bytes - shift), 0x00020000);
  const bool kill = KC && (k0 + op.kslot >= K);
#pragma unroll
  for (int i = 0; i < kPieces; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + (i * 4 + wid) * 1024), 16,
                                             kill ? kOOB : op.voff[i], 0, 0, 0);
}

template <bool KC>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_at(const Op& op, int k0, int kend) {
  const bool past = k0 >= kend;
  const uint32_t shift = past ? 0u : (uint32_t)k0 * op.kstep;
  return __builtin_amdgcn_make_buffer_rsrc((void*)(op.base + shift), (short)0, past ? 0 : (int)(op.bytes - shift),
                                           0x00020000);
}
template <int XF = 0>
__device__ __forceinline__ void dma1(__amdgpu_buffer_rsrc_t rs, char* dst, const Op& op, int i, bool kill, int wid) {
  if constexpr (XF & 32) kill = true;  // experiment: issue the DMA, read nothing (out of range)
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (lds_void*)(dst + (i * 4 + wid) * 1024), 16, kill ? kOOB : op.voff[i],
                                           0, 0, 0);
}

// Fragment read (same image / lane map as read_frag in ldnn_gemm_tile.h), issued
// as inline asm: hipcc cannot tell the builtin ds_read_b64_tr_b16 from an alias of
// the in-flight LDS-DMA writes and would drain the DMA (vmcnt(0)) before every
// one, and its own counted lgkm waits (which do not see asm reads) over-wait once
// the two kinds mix.  The compiler counts none of these reads: each consuming
// sub-step starts with an explicit lgkmcnt(0) (lgkm_all; the barrier does it for
// sub-step 1) -- the reads were issued a whole sub-step earlier.
__device__ __forceinline__ uint32_t lds_addr(const char* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
template <bool KC, bool ASM = true>
__device__ __forceinline__ bf16x8 frag(const char* lds, int rt, int kk, int lane) {
  if constexpr (KC && !ASM) {
    return read_frag<true, BM>(lds, rt, kk, lane);
  } else if constexpr (KC) {
    const int row = rt * 16 + (lane & 15);
    const int chunk = kk * 4 + (lane >> 4);
    bf16x8 v;
    asm volatile("ds_read_b128 %0, %1" : "=v"(v) : "v"(lds_addr(lds) + (uint32_t)(row * 128 + ((chunk ^ (row & 7)) << 4)))
                 : "memory");
    return v;
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int kb = kk * 4 + g;
    const int sw = (kb & 1) << 2;
    const uint32_t blk = lds_addr(lds) + (uint32_t)((kb * (BM / 16) + rt) * 256);
    bf16x4 lo, hi;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(blk + ((q ^ sw) * 32) + pp * 8) : "memory");
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(hi) : "v"(blk + (((4 + q) ^ sw) * 32) + pp * 8) : "memory");
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}
__device__ __forceinline__ void lgkm_all() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

template <bool KC, bool ASM>
__device__ __forceinline__ void read8(bf16x8 (&f)[8], const char* lds, int rt0, int kk, int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) f[i] = frag<KC, ASM>(lds, rt0 + i, kk, lane);
}

// 64 MFMAs: acc[n-tile j][m-tile i] += B_j^T A_i (MFMA-A <- B fragment: lanes own 4 consecutive columns)
// The accumulators are pinned to AGPRs ("+a"): with 256 of them the register
// allocator otherwise splits their live ranges across the two register halves and
// shuffles them with hundreds of v_accvgpr moves per K-tile.  Operands come from
// ds_reads (the compiler waits lgkmcnt before each asm); MFMA -> MFMA accumulate
// chains need no padding, and the AGPR <-> VALU hand-offs around the loop are
// padded explicitly (mma_fence).
__device__ __forceinline__ void mfma1(floatx4& acc, const bf16x8& b, const bf16x8& a) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(b), "v"(a) : "memory");
}
// 64 MFMAs of one 32-deep sub-step with `extra(q)` issued before MFMA q (q = 0..63):
// the LDS reads / DMA of the pipeline trickle out between the MFMAs instead of
// stalling the wave's issue in one burst (the texture path accepts a 1-KiB DMA
// instruction only every few tens of cycles per CU).  The "memory" clobber pins
// that order.
template <typename F>
__device__ __forceinline__ void mma(floatx4 (&acc)[8][8], const bf16x8 (&fa)[8], const bf16x8 (&fb)[8], F&& extra) {
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      extra(i * 8 + j);
      mfma1(acc[j][i], fb[j], fa[i]);
    }
}
// wait states between an MFMA that wrote an accumulator and a VALU / v_accvgpr_read of it
// (and between v_accvgpr_write initialisation and the first MFMA)
__device__ __forceinline__ void mma_fence() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 3" ::: "memory"); }

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Row-coalesced epilogue of a wave's 128 x 128 tile (bf16 or fp32 output): the
// fp32 accumulators are parked in the wave's 32 KiB LDS slice one 64-row half at
// a time ([64][128] fp32, 512-B rows, 16-B chunks XOR-swizzled by row), then
// re-read ROW-wise -- 16 lanes cover one 128-column row, 4 rows per instruction
// -- so the saved-activation (aux) loads and the output stores are full 256-B
// (bf16) / 512-B (fp32) row runs.  All 16 aux rows of a half are loaded before
// the staging writes, so their latency overlaps it instead of serialising.
// Bias-gradient column sums stay per lane (8 fixed columns) and are reduced
// across the 4 row lanes once, then one atomic per column per wave.
template <int EPI, bool OUT_F32, int XF = 0>
__device__ __forceinline__ void epilogue_q(const GemmParams& p, floatx4 (&acc)[8][8], char* smem, int wid, int mbase,
                                           int nbase, int lane) {
  char* wbuf = smem + wid * 32768;
  uint32_t xsum = 0;  // XF bit 7 (experiment): no global stores, a checksum keeps the work live
  const int c8 = lane & 15;  // this lane's 8 columns
  const int n = nbase + c8 * 8;
  const bool nok = n < p.N;  // N % 8 == 0
  constexpr bool kAux = EPI == EPI_DRELU || EPI == EPI_DSIGMOID;
  constexpr bool kMaskIn = EPI == EPI_DRELU_MASK, kMaskOut = EPI == EPI_BIAS_RELU_MASK;
  constexpr bool kBias = EPI == EPI_BIAS || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_SIGMOID || kMaskOut;
  float bias[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (kBias) {
    if (nok) {
      const floatx4 b0 = *reinterpret_cast<const floatx4*>(p.bias + n);
      const floatx4 b1 = *reinterpret_cast<const floatx4*>(p.bias + n + 4);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        bias[q] = b0[q];
        bias[q + 4] = b1[q];
      }
    }
  }
  // fused optimizer (weight-gradient GEMMs): the 8-column row runs update master / state /
  // shadow in place of storing the gradient -- 512-B fp32 runs per row, like the stores
  constexpr bool kOpt = EPI == EPI_OPT_SGD || EPI == EPI_OPT_ADAM;
  // bias-gradient column sums: dgrad / plain epilogues only (a forward never has a dbias)
  constexpr bool kSums = !kBias && !kOpt && EPI != EPI_BIAS_RELU_HEAD;
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  OptConst okc{};
  if constexpr (kOpt) okc = opt_const<EPI>(p.opt);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if constexpr (kOpt) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int row = i * 16 + (lane & 15);
          const int chunk = j * 4 + (lane >> 4);
          *reinterpret_cast<floatx4*>(wbuf + row * 512 + ((chunk ^ (row & 31)) << 4)) = acc[j][h * 4 + i];
        }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own staging writes landed (wave-private slice)
      __builtin_amdgcn_wave_barrier();
      constexpr int U = EPI == EPI_OPT_SGD ? 8 : 4;  // row runs per batch: all their state loads in flight
      // together (SGD 2 state arrays: 8 x 2 x (g, p, m) floatx4 = 192 VGPRs; Adam 3 arrays: 4)
#pragma unroll
      for (int it0 = 0; it0 < 16; it0 += U) {
        size_t off[U];
        bool ok[U];
        floatx4 g[U][2];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int row = (it0 + u) * 4 + (lane >> 4);
          const int m = mbase + h * 64 + row;
          const char* rb = wbuf + row * 512;
          g[u][0] = *reinterpret_cast<const floatx4*>(rb + (((2 * c8) ^ (row & 31)) << 4));
          g[u][1] = *reinterpret_cast<const floatx4*>(rb + (((2 * c8 + 1) ^ (row & 31)) << 4));
          ok[u] = nok && m < p.M;
          off[u] = (size_t)m * p.ldc + n;
        }
        opt_update8_batch<EPI, U>(p.opt, okc, off, ok, g);
      }
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    u16x8 a8[16];
    uint32_t mk[16];
    if constexpr (kAux) {
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int m = mbase + h * 64 + it * 4 + (lane >> 4);
        a8[it] = (nok && m < p.M) ? *reinterpret_cast<const u16x8*>(p.aux + (size_t)m * p.ldaux + n) : u16x8{};
      }
    }
    if constexpr (kMaskIn) {  // one byte per row and 8 columns: 1/16 of the aux bytes
#pragma unroll
      for (int it = 0; it < 16; ++it) {
        const int m = mbase + h * 64 + it * 4 + (lane >> 4);
        mk[it] = (nok && m < p.M) ? (uint32_t)p.mask_in[(size_t)m * p.ldmask + (n >> 3)] : 0u;
      }
    }
    // lane holds C[m = i*16 + (l&15)][n = j*16 + 4*(l>>4) + r]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int row = i * 16 + (lane & 15);
        const int chunk = j * 4 + (lane >> 4);
        *reinterpret_cast<floatx4*>(wbuf + row * 512 + ((chunk ^ (row & 31)) << 4)) = acc[j][h * 4 + i];
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own staging writes landed (wave-private slice)
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int row = it * 4 + (lane >> 4);
      const int m = mbase + h * 64 + row;
      const char* rb = wbuf + row * 512;
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(rb + (((2 * c8) ^ (row & 31)) << 4));
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(rb + (((2 * c8 + 1) ^ (row & 31)) << 4));
      if (!(nok && m < p.M)) continue;
      float o[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float aux = kAux ? bf2f(a8[it][q]) : (kMaskIn ? (float)((mk[it] >> q) & 1u) : 0.f);
        o[q] = apply_epi<EPI>(q < 4 ? v0[q] : v1[q - 4], bias[q], aux);
      }
      if constexpr (OUT_F32) {
        float* c = reinterpret_cast<float*>(p.C) + (size_t)m * p.ldc + n;
        floatx4 w0{o[0], o[1], o[2], o[3]}, w1{o[4], o[5], o[6], o[7]};
        if (p.beta != 0.f) {
          w0 += p.beta * *reinterpret_cast<const floatx4*>(c);
          w1 += p.beta * *reinterpret_cast<const floatx4*>(c + 4);
        }
        *reinterpret_cast<floatx4*>(c) = w0;
        *reinterpret_cast<floatx4*>(c + 4) = w1;
        if constexpr (kSums) {
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            cs[q] += w0[q];
            cs[q + 4] += w1[q];
          }
        }
      } else {
        u16x8 ob;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          ob[q] = f2bf(o[q]);
          if constexpr (kSums) cs[q] += bf2f(ob[q]);
        }
        u16x8* dst = reinterpret_cast<u16x8*>(reinterpret_cast<bf16_t*>(p.C) + (size_t)m * p.ldc + n);
        if constexpr ((XF & 128) != 0) {
          xsum ^= (uint32_t)ob[0] | ((uint32_t)ob[7] << 16);
        } else if (p.variant & 4096) {
          __builtin_nontemporal_store(ob, dst);
        } else {
          *dst = ob;
        }
        if constexpr (kMaskOut) {
          uint32_t bits = 0;
#pragma unroll
          for (int q = 0; q < 8; ++q) bits |= (bf2f(ob[q]) > 0.f ? 1u : 0u) << q;
          p.mask_out[(size_t)m * p.ldmask + (n >> 3)] = (uint8_t)bits;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if constexpr ((XF & 128) != 0) reinterpret_cast<uint32_t*>(p.C)[(size_t)blockIdx.x * kThreads + wid * 64 + lane] = xsum;
  if (kSums && p.dbias != nullptr) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float t = cs[q];
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      cs[q] = t;
    }
    if (lane < 16 && nok) {
#pragma unroll
      for (int q = 0; q < 8; ++q) atomicAdd(p.dbias + n + q, cs[q]);
    }
  }
}

// bf16-output epilogue with the activation finished in the MFMA accumulator layout
// (EPI_NONE / EPI_BIAS / EPI_BIAS_RELU / EPI_BIAS_RELU_MASK / EPI_BIAS_RELU_HEAD /
// EPI_DRELU_MASK).  Measured on MI355X (scripts/bench_epi_share.py): the fp32-staged
// row epilogue (epilogue_q) costs ~20 us of VALU + LDS work per 16384 x 4096 output
// on top of its ~10 us of stores; this one moves half the LDS bytes and leaves the
// store phase almost free of VALU work.
//  * bias (+ ReLU) + bf16 in registers: one packed add per 2 values, one
//    v_cvt_pk_bf16_f32 per 2, ReLU as a packed int16 max on the bf16 bits (negative
//    bf16 <=> negative int16; rounding is monotone, so max(bf16(v), 0) == bf16(max(v, 0))).
//  * EPI_BIAS_RELU_HEAD: the wave's 128 x 128 block of the activation times the
//    classifier head's weight on the MFMA pipe (32 MFMAs: 16 classes x 128 rows).  The
//    accumulator layout is fed to the MFMA as is: lane (g = l >> 4, r16 = l & 15) of
//    m-tile i holds row i*16 + r16 at columns 32t + 4g + {0..3} (n-tile 2t) and
//    32t + 16 + 4g + {0..3} (n-tile 2t+1), so k-slot 8g + e of k-step t means exactly
//    those columns, and the head weight fragment is loaded with the same permutation
//    (two 8-B pieces per class row).  The two column halves of the workgroup
//    (wn = 0, 1) combine their partial logits in the wn = 0 wave's LDS slice; wn = 0
//    stores head_part[n0 / 256][m][c].
//  * The bf16 tile is staged in the wave's own 32 KiB slice (all 128 rows at once,
//    16-B chunks XOR-swizzled by row) and re-read row-wise -- 16 lanes per 256-B row,
//    4 rows per instruction -- for full-row stores; the ReLU bit masks (read for the
//    dgrad, written by the forward) and the bias-gradient column sums work on those
//    8-column row pieces.
template <int EPI>
__device__ __forceinline__ void epilogue_bf16(const GemmParams& p, floatx4 (&acc)[8][8], char* smem, int wid, int mbase,
                                              int nbase, int lane) {
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
  constexpr bool kHead = EPI == EPI_BIAS_RELU_HEAD;
  constexpr bool kRelu = EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_RELU_MASK || kHead;
  constexpr bool kBias = kRelu || EPI == EPI_BIAS;
  constexpr bool kMaskIn = EPI == EPI_DRELU_MASK, kMaskOut = EPI == EPI_BIAS_RELU_MASK;
  constexpr bool kSums = EPI == EPI_NONE || kMaskIn;
  const int g = lane >> 4, r16 = lane & 15;
  floatx4 bias[8];
  if constexpr (kBias) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = nbase + j * 16 + 4 * g;
      bias[j] = n < p.N ? *reinterpret_cast<const floatx4*>(p.bias + n) : floatx4{0.f, 0.f, 0.f, 0.f};
    }
  }
  bf16x8 wf[4];
  if constexpr (kHead) {
    const bf16_t* wrow = p.head_w + (size_t)r16 * p.ldhw;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int nlo = nbase + 32 * t + 4 * g, nhi = nlo + 16;
      const bf16x4 zero = {};
      const bf16x4 lo = nlo < p.N ? *reinterpret_cast<const bf16x4*>(wrow + nlo) : zero;
      const bf16x4 hi = nhi < p.N ? *reinterpret_cast<const bf16x4*>(wrow + nhi) : zero;
      wf[t] = bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    }
  }
  // packed bf16 results, [n-tile j][m-tile i]: 4 values = 2 dwords
  uint32_t hq[8][8][2];
  const s16x2 zero2 = {0, 0};
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      floatx4 v = acc[j][i];
      if constexpr (kBias) v += bias[j];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const bf16x2 pb = {(__bf16)v[2 * h], (__bf16)v[2 * h + 1]};
        s16x2 r = __builtin_bit_cast(s16x2, pb);
        if constexpr (kRelu) r = __builtin_elementwise_max(r, zero2);
        hq[j][i][h] = __builtin_bit_cast(uint32_t, r);
      }
    }
  if constexpr (kHead) {
    floatx4 d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      d[i] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const u32x4 q = {hq[2 * t][i][0], hq[2 * t][i][1], hq[2 * t + 1][i][0], hq[2 * t + 1][i][1]};
        d[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t], __builtin_bit_cast(bf16x8, q), d[i], 0, 0, 0);
      }
    }
    const int wm = wid >> 1, wn = wid & 1;
    floatx4* xch = reinterpret_cast<floatx4*>(smem + (2 * wm) * 32768);  // the wn = 0 wave's slice
    if (wn == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) xch[i * 64 + lane] = d[i];
    }
    barrier();
    if (wn == 0) {
      float* part = p.head_part + (size_t)(nbase / 256) * p.M * 16;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int m = mbase + i * 16 + r16;
        const floatx4 v = d[i] + xch[i * 64 + lane];
        if (m < p.M) *reinterpret_cast<floatx4*>(part + (size_t)m * 16 + 4 * g) = v;
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // reads of the slice done before this wave stages into it
    }
  }
  // stage: row i*16 + r16 (256 B), 8-B piece (j*16 + 4g) * 2 B within 16-B chunk 2j + (g >> 1)
  char* wbuf = smem + wid * 32768;
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int row = i * 16 + r16;
      const int chunk = 2 * j + (g >> 1);
      *reinterpret_cast<uint2*>(wbuf + row * 256 + ((chunk ^ (row & 15)) << 4) + (g & 1) * 8) =
          uint2{hq[j][i][0], hq[j][i][1]};
    }
  const int c8 = lane & 15;
  const int n = nbase + c8 * 8;
  const bool nok = n < p.N;  // N % 8 == 0
  uint32_t mk[32];
  if constexpr (kMaskIn) {  // one byte per row and 8 columns, all 32 in flight during the staging
#pragma unroll
    for (int it = 0; it < 32; ++it) {
      const int m = mbase + it * 4 + (lane >> 4);
      mk[it] = (nok && m < p.M) ? (uint32_t)p.mask_in[(size_t)m * p.ldmask + (n >> 3)] : 0u;
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own staging writes landed (wave-private slice)
  __builtin_amdgcn_wave_barrier();
  auto rows = [&](auto sums) {
    constexpr bool kS = decltype(sums)::value;
    float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int it = 0; it < 32; ++it) {
      const int row = it * 4 + (lane >> 4);
      const int m = mbase + row;
      u32x4 v = *reinterpret_cast<const u32x4*>(wbuf + row * 256 + ((c8 ^ (row & 15)) << 4));
      if (!(nok && m < p.M)) continue;
      if constexpr (kMaskIn) {  // relu'(h) from the bit mask: zero the 16-bit halves whose bit is 0
        const uint32_t b = mk[it];
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] &= (((b >> (2 * k)) & 1u) ? 0x0000ffffu : 0u) | (((b >> (2 * k + 1)) & 1u) ? 0xffff0000u : 0u);
      }
      if constexpr (kS) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          cs[2 * k] += __uint_as_float(v[k] << 16);
          cs[2 * k + 1] += __uint_as_float(v[k] & 0xffff0000u);
        }
      }
      u32x4* dst = reinterpret_cast<u32x4*>(reinterpret_cast<bf16_t*>(p.C) + (size_t)m * p.ldc + n);
      if (p.variant & 4096) __builtin_nontemporal_store(v, dst);
      else *dst = v;
      if constexpr (kMaskOut) {  // bit q = output (m, n + q) > 0 (ReLU output: sign clear, nonzero)
        uint32_t bits = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          bits |= ((v[k] & 0xffffu) != 0u ? 1u : 0u) << (2 * k);
          bits |= ((v[k] >> 16) != 0u ? 1u : 0u) << (2 * k + 1);
        }
        p.mask_out[(size_t)m * p.ldmask + (n >> 3)] = (uint8_t)bits;
      }
    }
    if constexpr (kS) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        float t = cs[q];
        t += __shfl_xor(t, 16, 64);
        t += __shfl_xor(t, 32, 64);
        cs[q] = t;
      }
      if (lane < 16 && nok) {
#pragma unroll
        for (int q = 0; q < 8; ++q) atomicAdd(p.dbias + n + q, cs[q]);
      }
    }
  };
  if constexpr (kSums) {
    if (p.dbias != nullptr) rows(std::true_type{});
    else rows(std::false_type{});
  } else {
    rows(std::false_type{});
  }
}

// XF: experiment flags (0 in production): bit0 no in-loop DMA, bit1 no DMA wait, bit2 no in-loop ds_reads,
// bits 3 / 4: alternative DMA / read placements in sub-step 1 (see there), bit5 in-loop DMAs read nothing,
// bit6 no epilogue (measures the epilogue's share of the kernel), bit7 epilogue without its global stores
template <bool A_KC, bool B_KC, int EPI, bool OUT_F32, int XF = 0>
__global__ __launch_bounds__(kThreads, 1) void gemm_kernel(GemmParams p) {
  constexpr bool kDma = !(XF & 1), kWait = !(XF & 2), kRead = !(XF & 4);
  // all-k-contiguous kernels let the compiler track their ds_read_b128s (measured faster);
  // any k-strided operand switches every fragment read to asm (see frag)
  constexpr bool kAsm = !(A_KC && B_KC);
  __shared__ __attribute__((aligned(1024))) char smem[2 * kStage];  // 128 KiB, the only LDS object

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;
  int m0, n0;
  {
    // XCD remap, then groups of G tile-rows (G from variant bits 8..11 in experiments; default 4:
    // measured on MI355X equal to 8 on the forward, +7 % on the dgrad, profiles/gemm_q_r2.txt)
    const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
    const int gsel = (p.variant >> 8) & 15;
    const int G = gsel ? (1 << (gsel - 1)) : 4;
    const int id = xcd_remap(blockIdx.x, tiles_m * tiles_n);
    const int per_group = G * tiles_n;
    const int first_m = (id / per_group) * G;
    const int gsize = min(tiles_m - first_m, G);
    m0 = (first_m + (id % per_group) % gsize) * BM;
    n0 = ((id % per_group) / gsize) * BN;
  }

  const int nk_all = (p.K + BK - 1) / BK;
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
  const int kbase = kt0 * BK;

  Op oa, ob;
  init_op<A_KC>(oa, p.A, p.lda, p.M, p.K, m0, wid, lane);
  init_op<B_KC>(ob, p.B, p.ldb, p.N, p.K, n0, wid, lane);

  floatx4 acc[8][8];
#pragma unroll
  for (int j = 0; j < 8; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int kend = kbase + nk * BK;
  auto stage = [&](int t, char* dst) {
    const int k0 = kbase + t * BK;
    issue<A_KC>(oa, dst, k0, p.K, kend, wid);
    issue<B_KC>(ob, dst + kTile, k0, p.K, kend, wid);
  };

  bf16x8 fa0[8], fb0[8], fa1[8], fb1[8];
  mma_fence();
  if (nk > 0) {
    stage(0, smem);
    stage(1, smem + kStage);
    asm volatile("s_waitcnt vmcnt(16)" ::: "memory");  // tile 0 landed, tile 1 in flight
    barrier();
    read8<A_KC, kAsm>(fa0, smem, wm * 8, 0, lane);
    read8<B_KC, kAsm>(fb0, smem + kTile, wn * 8, 0, lane);
  }
  for (int t = 0; t < nk; ++t) {
    char* const cur = smem + (t & 1) * kStage;
    char* const nxt = smem + ((t + 1) & 1) * kStage;
    // sub-step 0: fragments of sub-step 1 stream in between the MFMAs
    lgkm_all();  // the fragment reads of F0
    // (reads every 2nd MFMA: all issued by MFMA 30, so the barrier's lgkmcnt(0) finds them done)
    mma(acc, fa0, fb0, [&](int q) {
      const int r = q >> 1;
      if ((kRead || t == 0) && !(q & 1) && r < 16) {
        if (r < 8) fa1[r] = frag<A_KC, kAsm>(cur, wm * 8 + r, 1, lane);
        else fb1[r - 8] = frag<B_KC, kAsm>(cur + kTile, wn * 8 + r - 8, 1, lane);
      }
    });
    // one barrier per K-tile: every wave finished reading `cur`, tile t+1 (own DMA waited) published
    if (kWait) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    barrier();
    // sub-step 1: tile t+2's DMA into `cur` and tile t+1's first fragments, between the MFMAs
    const int k2 = kbase + (t + 2) * BK;
    const __amdgpu_buffer_rsrc_t ra = rsrc_at<A_KC>(oa, k2, kend), rb = rsrc_at<B_KC>(ob, k2, kend);
    const bool killa = A_KC && (k2 + oa.kslot >= p.K), killb = B_KC && (k2 + ob.kslot >= p.K);
    // (DMA every 4th MFMA, reads every 2nd from MFMA 1 on; experiment schedules:
    // XF bit3 = reads in MFMA gaps 0..31, DMAs in gaps 32..63 every 2nd;
    // XF bit4 = DMAs in gaps 0..31 every 2nd, reads in gaps 32..63)
    mma(acc, fa1, fb1, [&](int q) {
      if constexpr (XF & 8) {
        const int rr = q >> 1, r = (q - 32) >> 1;
        if (kRead && q < 32 && (q & 1)) {
          if (rr < 8) fa0[rr] = frag<A_KC, kAsm>(nxt, wm * 8 + rr, 0, lane);
          else fb0[rr - 8] = frag<B_KC, kAsm>(nxt + kTile, wn * 8 + rr - 8, 0, lane);
        }
        if (kDma && q >= 32 && !(q & 1)) {
          if (r < 8) dma1<XF>(ra, cur, oa, r, killa, wid);
          else dma1<XF>(rb, cur + kTile, ob, r - 8, killb, wid);
        }
      } else if constexpr (XF & 16) {
        const int r = q >> 1, rr = (q - 32) >> 1;
        if (kDma && q < 32 && !(q & 1)) {
          if (r < 8) dma1<XF>(ra, cur, oa, r, killa, wid);
          else dma1<XF>(rb, cur + kTile, ob, r - 8, killb, wid);
        }
        if (kRead && q >= 32 && (q & 1)) {
          if (rr < 8) fa0[rr] = frag<A_KC, kAsm>(nxt, wm * 8 + rr, 0, lane);
          else fb0[rr - 8] = frag<B_KC, kAsm>(nxt + kTile, wn * 8 + rr - 8, 0, lane);
        }
      } else {
        const int r = q >> 2;
        if (kDma && !(q & 3)) {
          if (r < 8) dma1<XF>(ra, cur, oa, r, killa, wid);
          else dma1<XF>(rb, cur + kTile, ob, r - 8, killb, wid);
        }
        const int rr = q >> 1;
        if (kRead && (q & 1) && rr < 16) {
          if (rr < 8) fa0[rr] = frag<A_KC, kAsm>(nxt, wm * 8 + rr, 0, lane);
          else fb0[rr - 8] = frag<B_KC, kAsm>(nxt + kTile, wn * 8 + rr - 8, 0, lane);
        }
      }
    });
  }
  mma_fence();

  GemmParams pe = p;
  if (gridDim.y > 1) {
    if (p.c_split_stride > 0) {  // partial products to separate slabs (summed by slab_sum)
      pe.C = reinterpret_cast<char*>(p.C) + (size_t)blockIdx.y * (size_t)p.c_split_stride * (OUT_F32 ? 4u : 2u);
    } else if (!splitk_combine<8, 8, kThreads>(acc, p.ws, p.cnt, blockIdx.x, gridDim.y, blockIdx.y, smem)) {
      return;
    }
  }
  if constexpr ((XF & 64) != 0) {  // experiment: no epilogue (one float per lane keeps the MFMAs live)
    float t = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) t += acc[j][i][0] + acc[j][i][3];
    reinterpret_cast<float*>(p.C)[(size_t)blockIdx.x * kThreads + tid] = t;
    return;
  }
  if constexpr (EPI != EPI_OPT_SGD && EPI != EPI_OPT_ADAM) {
    barrier();  // every wave is done with the operand stages: LDS belongs to the epilogue
    // bf16 outputs whose activation is exact on the bf16 value: the register-side epilogue
    // (variant bit 13 selects the fp32-staged one, an A/B knob)
    constexpr bool kBf16Epi = !OUT_F32 && (EPI == EPI_NONE || EPI == EPI_BIAS || EPI == EPI_BIAS_RELU ||
                                           EPI == EPI_BIAS_RELU_MASK || EPI == EPI_BIAS_RELU_HEAD ||
                                           EPI == EPI_DRELU_MASK) && (XF & 128) == 0;
    if constexpr (EPI == EPI_BIAS_RELU_HEAD) {
      epilogue_bf16<EPI>(pe, acc, smem, wid, m0 + wm * 128, n0 + wn * 128, lane);
    } else if constexpr (kBf16Epi) {
      if (p.variant & 8192) epilogue_q<EPI, OUT_F32, XF>(pe, acc, smem, wid, m0 + wm * 128, n0 + wn * 128, lane);
      else epilogue_bf16<EPI>(pe, acc, smem, wid, m0 + wm * 128, n0 + wn * 128, lane);
    } else {
      epilogue_q<EPI, OUT_F32, XF>(pe, acc, smem, wid, m0 + wm * 128, n0 + wn * 128, lane);
    }
  } else {
    barrier();  // every wave is done with the operand stages: LDS belongs to the epilogue
    epilogue_q<EPI, OUT_F32, XF>(pe, acc, smem, wid, m0 + wm * 128, n0 + wn * 128, lane);
  }
}

template <bool A_KC, bool B_KC, bool OUT_F32>
hipError_t dispatch_epi(const GemmParams& p, int epi, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const dim3 grid(tiles, max(1, p.splitk)), block(kThreads);
  if ((p.variant & 255) > 32) {  // experiment builds (fwd layout, bias+ReLU only)
    if constexpr (A_KC && B_KC && !OUT_F32) {
      if (epi != EPI_BIAS_RELU) return hipErrorInvalidValue;
      switch ((p.variant & 255) - 32) {
        case 1: gemm_kernel<true, true, EPI_BIAS_RELU, false, 1><<<grid, block, 0, s>>>(p); break;
        case 2: gemm_kernel<true, true, EPI_BIAS_RELU, false, 2><<<grid, block, 0, s>>>(p); break;
        case 4: gemm_kernel<true, true, EPI_BIAS_RELU, false, 4><<<grid, block, 0, s>>>(p); break;
        case 5: gemm_kernel<true, true, EPI_BIAS_RELU, false, 5><<<grid, block, 0, s>>>(p); break;
        case 8: gemm_kernel<true, true, EPI_BIAS_RELU, false, 8><<<grid, block, 0, s>>>(p); break;
        case 16: gemm_kernel<true, true, EPI_BIAS_RELU, false, 16><<<grid, block, 0, s>>>(p); break;
        case 32: gemm_kernel<true, true, EPI_BIAS_RELU, false, 32><<<grid, block, 0, s>>>(p); break;
        case 64: gemm_kernel<true, true, EPI_BIAS_RELU, false, 64><<<grid, block, 0, s>>>(p); break;
        case 128: gemm_kernel<true, true, EPI_BIAS_RELU, false, 128><<<grid, block, 0, s>>>(p); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  switch (epi) {
#define Q_EPI_CASE(E) \
  case E: gemm_kernel<A_KC, B_KC, E, OUT_F32><<<grid, block, 0, s>>>(p); break;
    Q_EPI_CASE(EPI_NONE)
    Q_EPI_CASE(EPI_BIAS)
    Q_EPI_CASE(EPI_BIAS_RELU)
    Q_EPI_CASE(EPI_BIAS_SIGMOID)
    Q_EPI_CASE(EPI_DRELU)
    Q_EPI_CASE(EPI_DSIGMOID)
#undef Q_EPI_CASE
    case EPI_BIAS_RELU_MASK:
      if constexpr (!OUT_F32) {
        gemm_kernel<A_KC, B_KC, EPI_BIAS_RELU_MASK, false><<<grid, block, 0, s>>>(p);
        break;
      }
      return hipErrorInvalidValue;
    case EPI_DRELU_MASK:
      if constexpr (!OUT_F32) {
        gemm_kernel<A_KC, B_KC, EPI_DRELU_MASK, false><<<grid, block, 0, s>>>(p);
        break;
      }
      return hipErrorInvalidValue;
    case EPI_BIAS_RELU_HEAD:
      if constexpr (A_KC && B_KC && !OUT_F32) {
        gemm_kernel<true, true, EPI_BIAS_RELU_HEAD, false><<<grid, block, 0, s>>>(p);
        break;
      }
      return hipErrorInvalidValue;
    case EPI_OPT_SGD:
      if constexpr (OUT_F32) {
        gemm_kernel<A_KC, B_KC, EPI_OPT_SGD, true><<<grid, block, 0, s>>>(p);
        break;
      }
      return hipErrorInvalidValue;
    case EPI_OPT_ADAM:
      if constexpr (OUT_F32) {
        gemm_kernel<A_KC, B_KC, EPI_OPT_ADAM, true><<<grid, block, 0, s>>>(p);
        break;
      }
      return hipErrorInvalidValue;
    default:
      return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace kq
}  // namespace

size_t gemm_q_ws_bytes(int M, int N, int splitk) {
  const size_t tiles = (size_t)((M + kq::BM - 1) / kq::BM) * ((N + kq::BN - 1) / kq::BN);
  return tiles * (size_t)splitk * (size_t)(64 * kq::kThreads * 16);
}
int gemm_q_tiles(int M, int N) { return ((M + kq::BM - 1) / kq::BM) * ((N + kq::BN - 1) / kq::BN); }

hipError_t gemm_q(const GemmParams& p, bool a_kc, bool b_kc, int epi, bool out_f32, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  const size_t abytes = (size_t)(a_kc ? p.M : p.K) * p.lda * 2;
  const size_t bbytes = (size_t)(b_kc ? p.N : p.K) * p.ldb * 2;
  if (abytes >= kOOBLimit || bbytes >= kOOBLimit) return hipErrorInvalidValue;
  if (p.splitk > 1 && p.c_split_stride == 0 && (p.ws == nullptr || p.cnt == nullptr)) return hipErrorInvalidValue;
  if ((epi == EPI_BIAS_RELU_MASK && p.mask_out == nullptr) || (epi == EPI_DRELU_MASK && p.mask_in == nullptr) ||
      ((epi == EPI_BIAS_RELU_MASK || epi == EPI_DRELU_MASK) && (p.ldmask * 8 < p.N || p.N % 8 != 0)))
    return hipErrorInvalidValue;
  if (epi == EPI_BIAS_RELU_HEAD &&
      (p.head_w == nullptr || p.head_part == nullptr || p.bias == nullptr || p.splitk > 1 || p.ldhw < p.N ||
       p.ldhw % 4 != 0 || p.N % 8 != 0 || ((uintptr_t)p.head_w & 7) != 0 || ((uintptr_t)p.head_part & 15) != 0))
    return hipErrorInvalidValue;
  if (a_kc) {
    if (b_kc) return out_f32 ? kq::dispatch_epi<true, true, true>(p, epi, s) : kq::dispatch_epi<true, true, false>(p, epi, s);
    return out_f32 ? kq::dispatch_epi<true, false, true>(p, epi, s) : kq::dispatch_epi<true, false, false>(p, epi, s);
  }
  if (b_kc) return out_f32 ? kq::dispatch_epi<false, true, true>(p, epi, s) : kq::dispatch_epi<false, true, false>(p, epi, s);
  return out_f32 ? kq::dispatch_epi<false, false, true>(p, epi, s) : kq::dispatch_epi<false, false, false>(p, epi, s);
}

}  // namespace ldnn
