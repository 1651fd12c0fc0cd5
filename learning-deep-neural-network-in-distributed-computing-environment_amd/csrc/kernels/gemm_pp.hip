// Ping-pong 256x256 bf16 MFMA GEMM for gfx950 (the hot GEMM of the MLP step).
//
//   C[m][n] = epi( sum_k A(m,k) * B(k,n) )     fp32 accumulation, same operand
//   layouts / epilogues / GemmParams contract as gemm.hip (A_KC, B_KC, EPI_*).
//
// Why a second 256^2 kernel: gemm.hip's k256 runs one barrier per K-tile and
// drains its DMA (vmcnt(0)) at the end of every tile, so all 8 waves hit the
// LDS together at the top of each tile while the MFMA pipes idle, and the next
// tile's DMA has only one tile of compute to land in.  Measured on MI355X that
// caps it at ~1.1-1.25 PF where hipBLASLt reaches 1.33-1.41 PF on the MLP shapes
// (profiles/mlp_gemm_library_r1.jsonl).  This kernel is structured for the
// CDNA4 pipe mix (cdna_hip_programming.md §5 "8-phase", T3-T5):
//
//  * Two wave groups (wr = 0: waves 0-3, wr = 1: waves 4-7; waves w and w+4
//    share a SIMD) run the same 4-phase-per-K-tile schedule ONE BARRIER APART:
//    each phase is  [R] issue DMA + ds_read fragments | barrier | [M] 16 MFMAs
//    | barrier,  and group 1 executes one extra barrier up front, so while one
//    group's wave is in its MFMA cluster its SIMD partner is in its LDS-read /
//    DMA-issue section.  The MFMA pipe sees back-to-back clusters.
//  * Per wave: 128x64 of C as 4 quadrants of 64x32 (16 x v_mfma_f32_16x16x32_bf16
//    per quadrant per K-tile); quadrant order (0,0) (0,1) (1,1) (1,0) re-uses
//    operand fragments so a K-tile reads A once and B once (24 ds_read_b128-
//    equivalents per wave, 12/4/8/0 per phase).
//  * LDS = 2 K-tile buffers x {A, B} x 2 halves x 16 KiB = 128 KiB.  A half is
//    the 128 tile rows ONE quadrant row of every wave reads (A: 64-row blocks,
//    B: 32-row blocks, interleaved), so each half is consumed in one phase and
//    refilled (LDS-DMA, buffer_load ... lds) >= 2 phases after its last read:
//        phase q0 of tile t: DMA B.half1(t+1)   read A.half0, B.half0 (t)
//        phase q1          : DMA A.half1(t+1)   read B.half1 (t)
//        phase q2          : DMA A.half0(t+2)   read A.half1 (t)
//        phase q3          : DMA B.half0(t+2)   (no reads)
//    Every phase waits `vmcnt(8)` (= 4 phases of DMA still in flight, never 0
//    in the loop) before its first barrier, which retires exactly the halves
//    the NEXT phase reads; the barrier publishes them.  A DMA therefore has ~4
//    phases (~2000 cycles) to land.  Past the K end the DMAs read out of range
//    (zero fill, no memory traffic), so the counts never change.
//  * Raw s_barrier only (a __syncthreads would drain the in-flight DMA), all LDS
//    in one __shared__ array, no VGPR-destination global loads in the loop
//    (cdna_hip_programming.md §5 "Projection GEMM" item 4 traps).
//  * Split-K over gridDim.y with the in-launch deterministic combine
//    (splitk_combine) for grids that cannot fill 256 CUs (784-wide wgrad).
#include "ldnn_common.h"
#include "ldnn_gemm_tile.h"
#include "ldnn_kernels.h"

namespace ldnn {
namespace {
namespace kpp {

constexpr int BM = 256, BN = 256;
constexpr int kThreads = 512;
constexpr int kHalf = 128 * BK * 2;  // 16 KiB: 128 rows x 64 k
constexpr int kStage = 4 * kHalf;    // A.half0 A.half1 B.half0 B.half1
constexpr uint32_t kOOB = 0x80000000u;

// Tile row of in-half row `hr` of half `h`: halves interleave SPAN-row blocks
// (A: SPAN 64 -> a wave's two 64-row quadrant rows; B: SPAN 32).
template <int SPAN>
__device__ __forceinline__ int tile_row(int h, int hr) {
  return (hr / SPAN) * (2 * SPAN) + h * SPAN + (hr % SPAN);
}

struct Op {
  __amdgpu_buffer_rsrc_t rsrc;
  uint32_t base[2][2];  // [half][piece] byte offset of this lane's 16-B slot at k0 = 0
  int klim[2][2];       // the slot is in range iff k0 < klim (INT_MIN: rows outside the operand)
  uint32_t kstep;       // bytes per unit of k0
};

template <bool KC, int SPAN>
__device__ __forceinline__ void init_op(Op& op, const bf16_t* X, int ld, int rows, int K, int kend, int r0,
                                        int wid, int lane) {
  const uint32_t bytes = KC ? (uint32_t)((size_t)rows * ld * 2) : (uint32_t)((size_t)K * ld * 2);
  op.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)bytes, 0x00020000);
  op.kstep = KC ? 2u : (uint32_t)ld * 2u;
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int hr, k;
      lds_slot_to_rk<KC, 128>((i * 8 + wid) * 1024 + lane * 16, hr, k);
      const int r = r0 + tile_row<SPAN>(h, hr);
      const bool ok = r < rows;
      op.klim[h][i] = ok ? kend - k : INT_MIN;
      op.base[h][i] = ok ? (KC ? (uint32_t)(((size_t)r * ld + k) * 2) : (uint32_t)(((size_t)k * ld + r) * 2)) : 0u;
    }
}

// DMA one operand half (16 KiB = 2 x 1-KiB wave pieces per wave) of K-tile k0 into `dst`.
__device__ __forceinline__ void issue(const Op& op, char* dst, int h, int k0, int wid) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const bool ok = k0 < op.klim[h][i];
    const uint32_t off = ok ? op.base[h][i] + (uint32_t)k0 * op.kstep : kOOB;
    __builtin_amdgcn_raw_ptr_buffer_load_lds(op.rsrc, (lds_void*)(dst + (i * 8 + wid) * 1024), 16, off, 0, 0, 0);
  }
}

__device__ __forceinline__ void bar_r() {  // end of a read section: own ds_reads done, then the barrier
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void bar_m() {  // end of an MFMA section
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void wait_dma() { asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); }

template <bool KC>
__device__ __forceinline__ void read_a(bf16x8 (&fa)[4][2], const char* half, int wr, int lane) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int i = 0; i < 4; ++i) fa[i][kk] = read_frag<KC, 128>(half, wr * 4 + i, kk, lane);
}
template <bool KC>
__device__ __forceinline__ void read_b(bf16x8 (&fb)[2][2], const char* half, int wc, int lane) {
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < 2; ++j) fb[j][kk] = read_frag<KC, 128>(half, wc * 2 + j, kk, lane);
}

// One quadrant (mh, nh) x K = 64: 16 MFMAs.  MFMA-A <- B fragment, MFMA-B <- A
// fragment: each lane then owns 4 consecutive output columns (gemm.hip header).
template <int MH, int NH>
__device__ __forceinline__ void mma(floatx4 (&acc)[4][8], const bf16x8 (&fa)[4][2], const bf16x8 (&fb)[2][2]) {
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        acc[NH * 2 + j][MH * 4 + i] =
            __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j][kk], fa[i][kk], acc[NH * 2 + j][MH * 4 + i], 0, 0, 0);
  __builtin_amdgcn_s_setprio(0);
}

// XF: experiment flags (0 in production).  bit0: no stagger, bit1: no in-loop DMA,
// bit2: no in-loop ds_reads (fragments stay stale), bit3: one barrier per phase
template <bool A_KC, bool B_KC, int EPI, bool OUT_F32, int XF = 0>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmParams p) {
  constexpr bool kStagger = !(XF & 1), kDma = !(XF & 2), kRead = !(XF & 4), kBarM = !(XF & 8), kWait = !(XF & 16);
  __shared__ __attribute__((aligned(1024))) char smem[2 * kStage];  // 128 KiB, the only LDS object

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid >> 2, wc = wid & 3;
  int m0, n0;
  tile_coords(p.M, p.N, BM, BN, m0, n0);

  // split-K: this workgroup covers K-tiles [kt0, kt0 + nk)
  const int nk_all = (p.K + BK - 1) / BK;
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
  const int kbase = kt0 * BK;
  const int kend = min(p.K, kbase + nk * BK);

  Op oa, ob;
  init_op<A_KC, 64>(oa, p.A, p.lda, p.M, p.K, kend, m0, wid, lane);
  init_op<B_KC, 32>(ob, p.B, p.ldb, p.N, p.K, kend, n0, wid, lane);

  floatx4 acc[4][8];  // [n-tile j][m-tile i] of the wave's 128 x 64
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  char* const s0 = smem;
  char* const s1 = smem + kStage;
  // prologue: tile 0 complete, tile 1's phase-q2/q3 halves (as if issued by tile -1)
  issue(oa, s0, 0, kbase, wid);
  issue(ob, s0 + 2 * kHalf, 0, kbase, wid);
  issue(ob, s0 + 3 * kHalf, 1, kbase, wid);
  issue(oa, s0 + kHalf, 1, kbase, wid);
  issue(oa, s1, 0, kbase + BK, wid);
  issue(ob, s1 + 2 * kHalf, 0, kbase + BK, wid);
  wait_dma();  // tile 0's A.half0 / B.half0 landed
  __builtin_amdgcn_s_barrier();
  if (kStagger && wr == 1) __builtin_amdgcn_s_barrier();  // stagger: group 1 runs one barrier behind

  bf16x8 fa[4][2], fb0[2][2], fb1[2][2];
  if (!kRead) {
    read_a<A_KC>(fa, s0, wr, lane);
    read_b<B_KC>(fb0, s0 + 2 * kHalf, wc, lane);
    read_b<B_KC>(fb1, s0 + 3 * kHalf, wc, lane);
  }
  for (int t = 0; t < nk; ++t) {
    char* const sc = (t & 1) ? s1 : s0;
    char* const sn = (t & 1) ? s0 : s1;
    const int k1 = kbase + (t + 1) * BK, k2 = kbase + (t + 2) * BK;
    // q0
    if (kDma) issue(ob, sn + 3 * kHalf, 1, k1, wid);
    if (kRead) {
      read_a<A_KC>(fa, sc, wr, lane);
      read_b<B_KC>(fb0, sc + 2 * kHalf, wc, lane);
    }
    if (kDma && kWait) wait_dma();
    bar_r();
    mma<0, 0>(acc, fa, fb0);
    if (kBarM) bar_m();
    // q1
    if (kDma) issue(oa, sn + kHalf, 1, k1, wid);
    if (kRead) read_b<B_KC>(fb1, sc + 3 * kHalf, wc, lane);
    if (kDma && kWait) wait_dma();
    bar_r();
    mma<0, 1>(acc, fa, fb1);
    if (kBarM) bar_m();
    // q2
    if (kDma) issue(oa, sc, 0, k2, wid);
    if (kRead) read_a<A_KC>(fa, sc + kHalf, wr, lane);
    if (kDma && kWait) wait_dma();
    bar_r();
    mma<1, 1>(acc, fa, fb1);
    if (kBarM) bar_m();
    // q3
    if (kDma) issue(ob, sc + 2 * kHalf, 0, k2, wid);
    if (kDma && kWait) wait_dma();
    bar_r();
    mma<1, 0>(acc, fa, fb0);
    if (kBarM) bar_m();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the out-of-range tail DMAs
  if (kStagger && wr == 0) __builtin_amdgcn_s_barrier();  // un-stagger: equal barrier counts

  if (gridDim.y > 1) {
    if (!splitk_combine<4, 8, kThreads>(acc, p.ws, p.cnt, blockIdx.x, gridDim.y, blockIdx.y, smem)) return;
  }
  if constexpr (!OUT_F32 && EPI != EPI_OPT_SGD && EPI != EPI_OPT_ADAM) {
    __builtin_amdgcn_s_barrier();  // every wave is done with the operand stages: LDS is the epilogue's
    epilogue_lds_bf16<EPI>(p, acc, smem, wid, m0 + wr * 128, n0 + wc * 64, lane);
  } else {
    epilogue<EPI, OUT_F32, 8, 4>(p, acc, m0 + wr * 128, n0 + wc * 64, lane);
  }
}

template <bool A_KC, bool B_KC, bool OUT_F32>
hipError_t dispatch_epi(const GemmParams& p, int epi, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  const dim3 grid(tiles, max(1, p.splitk)), block(kThreads);
  if (p.variant > 4) {  // experiment builds (fwd layout, bias+ReLU only)
    if constexpr (A_KC && B_KC && !OUT_F32) {
      if (epi != EPI_BIAS_RELU) return hipErrorInvalidValue;
      switch (p.variant - 4) {
        case 1: gemm_kernel<true, true, EPI_BIAS_RELU, false, 1><<<grid, block, 0, s>>>(p); break;
        case 2: gemm_kernel<true, true, EPI_BIAS_RELU, false, 2><<<grid, block, 0, s>>>(p); break;
        case 4: gemm_kernel<true, true, EPI_BIAS_RELU, false, 4><<<grid, block, 0, s>>>(p); break;
        case 6: gemm_kernel<true, true, EPI_BIAS_RELU, false, 6><<<grid, block, 0, s>>>(p); break;
        case 8: gemm_kernel<true, true, EPI_BIAS_RELU, false, 8><<<grid, block, 0, s>>>(p); break;
        case 9: gemm_kernel<true, true, EPI_BIAS_RELU, false, 9><<<grid, block, 0, s>>>(p); break;
        case 14: gemm_kernel<true, true, EPI_BIAS_RELU, false, 14><<<grid, block, 0, s>>>(p); break;
        case 16: gemm_kernel<true, true, EPI_BIAS_RELU, false, 16><<<grid, block, 0, s>>>(p); break;
        case 20: gemm_kernel<true, true, EPI_BIAS_RELU, false, 20><<<grid, block, 0, s>>>(p); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
    return hipErrorInvalidValue;
  }
  switch (epi) {
#define LDNN_PP_CASE(E) \
  case E: gemm_kernel<A_KC, B_KC, E, OUT_F32><<<grid, block, 0, s>>>(p); break;
    LDNN_PP_CASE(EPI_NONE)
    LDNN_PP_CASE(EPI_BIAS)
    LDNN_PP_CASE(EPI_BIAS_RELU)
    LDNN_PP_CASE(EPI_BIAS_SIGMOID)
    LDNN_PP_CASE(EPI_DRELU)
    LDNN_PP_CASE(EPI_DSIGMOID)
#undef LDNN_PP_CASE
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

}  // namespace kpp
}  // namespace

size_t gemm_pp_ws_bytes(int M, int N, int splitk) {
  const size_t tiles = (size_t)((M + kpp::BM - 1) / kpp::BM) * ((N + kpp::BN - 1) / kpp::BN);
  return tiles * (size_t)splitk * (size_t)(32 * kpp::kThreads * 16);
}
int gemm_pp_tiles(int M, int N) { return ((M + kpp::BM - 1) / kpp::BM) * ((N + kpp::BN - 1) / kpp::BN); }

hipError_t gemm_pp(const GemmParams& p, bool a_kc, bool b_kc, int epi, bool out_f32, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  const size_t abytes = (size_t)(a_kc ? p.M : p.K) * p.lda * 2;
  const size_t bbytes = (size_t)(b_kc ? p.N : p.K) * p.ldb * 2;
  if (abytes >= kOOBLimit || bbytes >= kOOBLimit) return hipErrorInvalidValue;
  if (p.splitk > 1 && (p.ws == nullptr || p.cnt == nullptr)) return hipErrorInvalidValue;
  if (a_kc) {
    if (b_kc) return out_f32 ? kpp::dispatch_epi<true, true, true>(p, epi, s) : kpp::dispatch_epi<true, true, false>(p, epi, s);
    return out_f32 ? kpp::dispatch_epi<true, false, true>(p, epi, s) : kpp::dispatch_epi<true, false, false>(p, epi, s);
  }
  if (b_kc) return out_f32 ? kpp::dispatch_epi<false, true, true>(p, epi, s) : kpp::dispatch_epi<false, true, false>(p, epi, s);
  return out_f32 ? kpp::dispatch_epi<false, false, true>(p, epi, s) : kpp::dispatch_epi<false, false, false>(p, epi, s);
}

}  // namespace ldnn
