// bf16 MFMA GEMM for gfx950 with fused epilogues.
//
//   C[m][n] = epi( sum_k A(m,k) * B(k,n) )      fp32 accumulation
//
// Operand layouts (both chosen per call, so no transpose kernels are needed
// for the three GEMMs of a Linear layer):
//   A_KC (k-contiguous): A(m,k) = A[m*lda + k]     else A(m,k) = A[k*lda + m]
//   B_KC (k-contiguous): B(k,n) = B[n*ldb + k]     else B(k,n) = B[k*ldb + n]
//   fwd   Y  = X W^T  -> A_KC=1, B_KC=1   (W stored [N][K] like the reference's nn.Linear)
//   dgrad dX = dY W   -> A_KC=1, B_KC=0
//   wgrad dW = dY^T X -> A_KC=0, B_KC=0   (fp32 output straight into the flat grad buffer)
//
// Two tilings, picked per shape by gemm_bf16():
//
//  * gemm256 (large shapes): 256x256 output tile, BK = 64, 512 threads = 8 waves
//    (2 M x 4 N, 128x64 per wave, 8x4 accumulators of v_mfma_f32_16x16x32_bf16).
//    Operands are staged HBM/L2 -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds,
//    no VGPR round trip) into two 64 KiB stages; the next tile's DMA stays in
//    flight across the compute of the current one (counted vmcnt + raw
//    s_barrier, never __syncthreads while a DMA is outstanding).  Buffer
//    resource range checking zero-fills every out-of-range element, so ragged
//    M / N / K edges need no scalar tail.  One workgroup per CU.
//  * gemm128 (small / skinny shapes that cannot fill 256 CUs with 256^2 tiles):
//    128x128 tile, 4 waves (64x64 each), register-staged double buffer.
//
// Common to both (cdna_hip_programming.md §5, T1, T2, T10):
//   * MFMA roles swapped (MFMA-A <- our B tile, MFMA-B <- our A tile) so each lane
//     owns 4 consecutive output columns: bf16 epilogue stores are 8 B, fp32 16 B,
//     and a bias/activation needs 4 contiguous bias values.
//   * k-contiguous operands live in LDS as [rows][64 k] with a 16-B chunk XOR
//     swizzle (chunk ^ (row & 7)) -> conflict-free ds_read_b128 fragment reads.
//   * k-strided operands live in LDS as [k/8][rows/16][8][16] 256-B blocks read
//     with ds_read_b64_tr_b16 (hardware transpose); odd k-blocks store k-rows
//     0-3 <-> 4-7 swapped so the two 16-lane groups of a half-wave hit opposite
//     128-B halves of the bank row.
//   * With LDS-DMA the LDS image is lane-linear per wave instruction, so the
//     swizzle is applied on the per-lane SOURCE address (rule 21).
//   * XCD-aware bijective block remap + grouped tile order for L2 reuse.
//
// Epilogues fuse what the reference runs as separate ATen kernels
// (BAR/model.py Linear + F.relu; the autograd backward of both):
//   EPI_NONE, EPI_BIAS, EPI_BIAS_RELU, EPI_BIAS_SIGMOID (forward),
//   EPI_DRELU / EPI_DSIGMOID (dgrad multiplied by the activation derivative read
//   from the saved forward output `aux`), optional column-sum of the final
//   output into fp32 `dbias` (bias gradient of the previous layer, one atomic
//   per column per wave), optional beta-accumulate for fp32 outputs.
#include "ldnn_common.h"
#include "ldnn_gemm_tile.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

// =============================================================================
// gemm128: register-staged, 128x128x64, 4 waves
// =============================================================================
namespace k128 {

constexpr int BM = 128, BN = 128;
constexpr int kThreads = 256;
constexpr int kTileBytes = 128 * BK * 2;  // 16 KiB per operand tile

// 1024 16-B chunks per operand tile, 4 per thread.
template <bool KC>
__device__ __forceinline__ void load_tile(u32x4 (&r)[4], const bf16_t* __restrict__ X, int ld, int rows,
                                          int K, int r0, int k0, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + kThreads * i;
    int row, k;
    if constexpr (KC) {
      k = (c & 7) * 8;
      row = c >> 3;
    } else {
      // lanes 0..7 of a write group cover 4 k-rows x 2 halves -> conflict-free ds_write_b128,
      // and a wave reads 4 k-rows x 256 B of global memory
      const int half = c & 1, klo = (c >> 1) & 3, rb = (c >> 3) & 7, khi = c >> 6;
      k = khi * 4 + klo;
      row = rb * 16 + half * 8;
    }
    const int gr = r0 + row, gk = k0 + k;
    const bool ok = (gr < rows) && (gk < K);
    const bf16_t* p = KC ? (X + (size_t)gr * ld + gk) : (X + (size_t)gk * ld + gr);
    if (ok) {
      r[i] = *reinterpret_cast<const u32x4*>(p);
    } else {
      r[i] = u32x4{0u, 0u, 0u, 0u};
    }
  }
}

template <bool KC>
__device__ __forceinline__ void store_tile(const u32x4 (&r)[4], char* lds, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + kThreads * i;
    int row, k;
    if constexpr (KC) {
      k = (c & 7) * 8;
      row = c >> 3;
    } else {
      const int half = c & 1, klo = (c >> 1) & 3, rb = (c >> 3) & 7, khi = c >> 6;
      k = khi * 4 + klo;
      row = rb * 16 + half * 8;
    }
    *reinterpret_cast<u32x4*>(lds + lds_offset<KC, 128>(row, k)) = r[i];
  }
}

template <bool A_KC, bool B_KC, int EPI, bool OUT_F32>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * kTileBytes];  // [buf][A|B]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  int m0, n0;
  tile_coords(p.M, p.N, BM, BN, m0, n0);

  floatx4 acc[4][4];  // [n-tile j][m-tile i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  // split-K: this workgroup covers K-tiles [kt0, kt1)
  const int nk_all = (p.K + BK - 1) / BK;
  const int per = (nk_all + gridDim.y - 1) / gridDim.y;
  const int kt0 = blockIdx.y * per;
  const int nk = max(0, min(nk_all, kt0 + per) - kt0);
  const int kbase = kt0 * BK;
  u32x4 ra[4], rb[4];
  load_tile<A_KC>(ra, p.A, p.lda, p.M, p.K, m0, kbase, tid);
  load_tile<B_KC>(rb, p.B, p.ldb, p.N, p.K, n0, kbase, tid);
  store_tile<A_KC>(ra, smem, tid);
  store_tile<B_KC>(rb, smem + kTileBytes, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = (kt + 1) < nk;
    if (more) {
      load_tile<A_KC>(ra, p.A, p.lda, p.M, p.K, m0, kbase + (kt + 1) * BK, tid);
      load_tile<B_KC>(rb, p.B, p.ldb, p.N, p.K, n0, kbase + (kt + 1) * BK, tid);
    }
    const char* la = smem + cur * 2 * kTileBytes;
    const char* lb = la + kTileBytes;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag<A_KC, 128>(la, wm * 4 + i, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag<B_KC, 128>(lb, wn * 4 + j, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[j][i], 0, 0, 0);
    }
    if (more) {
      char* nb = smem + (cur ^ 1) * 2 * kTileBytes;
      store_tile<A_KC>(ra, nb, tid);
      store_tile<B_KC>(rb, nb + kTileBytes, tid);
    }
    __syncthreads();
  }
  if (gridDim.y > 1) {
    if (p.cnt != nullptr) {
      // in-launch deterministic combine: the last slice to arrive sums every slab
      // and runs the full epilogue (bias / activation / dbias / beta / bf16 out)
      if (!splitk_combine<4, 4, kThreads>(acc, p.ws, p.cnt, blockIdx.x, gridDim.y, blockIdx.y, smem)) return;
    } else {
      if constexpr (OUT_F32 && EPI == EPI_NONE) {  // fp32 atomics (C pre-zeroed or accumulated into)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int m = m0 + wm * 64 + i * 16 + (lane & 15);
            if (n < p.N && m < p.M) {
              float* c = reinterpret_cast<float*>(p.C) + (size_t)m * p.ldc + n;
#pragma unroll
              for (int r = 0; r < 4; ++r) atomicAdd(c + r, acc[j][i][r]);
            }
          }
        }
      }
      return;
    }
  }
  epilogue<EPI, OUT_F32, 4, 4>(p, acc, m0 + wm * 64, n0 + wn * 64, lane);
}

}  // namespace k128

// =============================================================================
// gemm256: LDS-DMA staged, 256x256x64, 8 waves, DMA of tile t+1 in flight
// across the compute of tile t
// =============================================================================
namespace k256 {

constexpr int BM = 256, BN = 256;
constexpr int kThreads = 512;
constexpr int kTileBytes = 256 * BK * 2;       // 32 KiB per operand tile
constexpr int kStageBytes = 2 * kTileBytes;    // A + B
constexpr int kPiecesPerWave = kTileBytes / 1024 / 8;  // 1-KiB DMA pieces per wave per operand = 4
constexpr uint32_t kOOB = 0x80000000u;         // any offset >= num_records reads as zero

struct Operand {
  __amdgpu_buffer_rsrc_t rsrc;
  int ld, rows, K, r0;
  int row[kPiecesPerWave];  // tile-relative row of this lane's slot in each piece
  int k[kPiecesPerWave];    // tile-relative k
};

template <bool KC>
__device__ __forceinline__ void init_operand(Operand& op, const bf16_t* X, int ld, int rows, int K, int r0,
                                             int wid, int lane) {
  const uint32_t bytes = KC ? (uint32_t)((size_t)rows * ld * 2) : (uint32_t)((size_t)K * ld * 2);
  op.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)bytes, 0x00020000);
  op.ld = ld;
  op.rows = rows;
  op.K = K;
  op.r0 = r0;
#pragma unroll
  for (int i = 0; i < kPiecesPerWave; ++i) {
    const int piece = i * 8 + wid;
    lds_slot_to_rk<KC, BM>(piece * 1024 + lane * 16, op.row[i], op.k[i]);
  }
}

// Issue the DMA of one operand tile (k0) into LDS at `dst`: 4 x buffer_load_dwordx4 ... lds per lane.
template <bool KC>
__device__ __forceinline__ void issue_tile(const Operand& op, char* dst, int k0, int wid, int lane) {
#pragma unroll
  for (int i = 0; i < kPiecesPerWave; ++i) {
    const int gr = op.r0 + op.row[i], gk = k0 + op.k[i];
    const bool ok = (gr < op.rows) && (gk < op.K);
    const uint32_t off = KC ? (uint32_t)(((size_t)gr * op.ld + gk) * 2) : (uint32_t)(((size_t)gk * op.ld + gr) * 2);
    char* piece = dst + (i * 8 + wid) * 1024;  // wave-uniform LDS base (M0); lanes land at +16*lane
    __builtin_amdgcn_raw_ptr_buffer_load_lds(op.rsrc, (lds_void*)piece, 16, ok ? off : kOOB, 0, 0, 0);
  }
}

__device__ __forceinline__ void barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <bool A_KC, bool B_KC, int EPI, bool OUT_F32>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(1024))) char smem[2 * kStageBytes];  // [stage][A|B], 128 KiB

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  int m0, n0;
  tile_coords(p.M, p.N, BM, BN, m0, n0);

  Operand oa, ob;
  init_operand<A_KC>(oa, p.A, p.lda, p.M, p.K, m0, wid, lane);
  init_operand<B_KC>(ob, p.B, p.ldb, p.N, p.K, n0, wid, lane);

  floatx4 acc[4][8];  // [n-tile j][m-tile i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  issue_tile<A_KC>(oa, smem, 0, wid, lane);
  issue_tile<B_KC>(ob, smem + kTileBytes, 0, wid, lane);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // One barrier per K-tile: it publishes tile kt (every wave waited for its own
  // DMA of kt) AND certifies that every wave finished reading stage (kt+1)&1
  // (tile kt-1), which is then refilled with tile kt+1 while kt is multiplied.
  for (int kt = 0; kt < nk; ++kt) {
    char* stage = smem + (kt & 1) * kStageBytes;
    barrier();
    if (kt + 1 < nk) {
      char* nxt = smem + ((kt + 1) & 1) * kStageBytes;
      issue_tile<A_KC>(oa, nxt, (kt + 1) * BK, wid, lane);
      issue_tile<B_KC>(ob, nxt + kTileBytes, (kt + 1) * BK, wid, lane);
    }
    const char* la = stage;
    const char* lb = stage + kTileBytes;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fb[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag<B_KC, BN>(lb, wn * 4 + j, kk, lane);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        bf16x8 fa[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) fa[i] = read_frag<A_KC, BM>(la, wm * 8 + h * 4 + i, kk, lane);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[j][h * 4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[j][h * 4 + i], 0, 0, 0);
      }
    }
    __builtin_amdgcn_s_setprio(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // own DMA of tile kt+1 landed
  }
  if constexpr (!OUT_F32) {
    if (!p.direct_epi) {
      barrier();  // every wave is done with the operand stages: reuse LDS for the epilogue
      epilogue_lds_bf16<EPI>(p, acc, smem, wid, m0 + wm * 128, n0 + wn * 64, lane);
    } else {
      epilogue<EPI, OUT_F32, 8, 4>(p, acc, m0 + wm * 128, n0 + wn * 64, lane);
    }
  } else {
    epilogue<EPI, OUT_F32, 8, 4>(p, acc, m0 + wm * 128, n0 + wn * 64, lane);
  }
}

}  // namespace k256

// =============================================================================
// gemm256 ring variant (GemmParams::variant 2 / 3, experimental): 256x256
// output tile, BK = 32 slots in an NS-deep LDS ring (NS x 32 KiB), so the DMA
// of K-step t+NS-1 is issued while step t is multiplied -- NS-1 K-steps of
// latency cover instead of one.  One barrier per K-step both publishes step t
// and frees the slot of step t-1 for refilling.  Measured on MI355X at 4096^3
// it is SLOWER than the 2-stage BK 64 loop (fwd 1168 vs 1254 TF, dgrad 855 vs
// 1091, wgrad 782 vs 942): twice the barriers per FLOP cost more than the
// deeper prefetch buys (profiles/gemm_variants_r1.jsonl).
// =============================================================================
namespace k256r {

using k256::barrier;
constexpr int BM = 256, BN = 256, BKr = 32;
constexpr int kThreads = 512;
constexpr int kTileBytes = 256 * BKr * 2;             // 16 KiB per operand per slot
constexpr int kSlotBytes = 2 * kTileBytes;            // A + B
constexpr int kPiecesPerWave = kTileBytes / 1024 / 8;  // 2
constexpr uint32_t kOOB = 0x80000000u;

struct Operand {
  __amdgpu_buffer_rsrc_t rsrc;
  int ld, rows, K, r0;
  int row[kPiecesPerWave];
  int k[kPiecesPerWave];
};

template <bool KC>
__device__ __forceinline__ void init_operand(Operand& op, const bf16_t* X, int ld, int rows, int K, int r0,
                                             int wid, int lane) {
  const uint32_t bytes = KC ? (uint32_t)((size_t)rows * ld * 2) : (uint32_t)((size_t)K * ld * 2);
  op.rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)bytes, 0x00020000);
  op.ld = ld;
  op.rows = rows;
  op.K = K;
  op.r0 = r0;
#pragma unroll
  for (int i = 0; i < kPiecesPerWave; ++i) lds_slot_to_rk<KC, BM, BKr>((i * 8 + wid) * 1024 + lane * 16, op.row[i], op.k[i]);
}

template <bool KC>
__device__ __forceinline__ void issue_tile(const Operand& op, char* dst, int k0, int wid) {
#pragma unroll
  for (int i = 0; i < kPiecesPerWave; ++i) {
    const int gr = op.r0 + op.row[i], gk = k0 + op.k[i];
    const bool ok = (gr < op.rows) && (gk < op.K);
    const uint32_t off = KC ? (uint32_t)(((size_t)gr * op.ld + gk) * 2) : (uint32_t)(((size_t)gk * op.ld + gr) * 2);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(op.rsrc, (lds_void*)(dst + (i * 8 + wid) * 1024), 16, ok ? off : kOOB,
                                             0, 0, 0);
  }
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// own DMAs of step t landed, with `ahead` later steps (4 instructions each) allowed in flight
template <int NS>
__device__ __forceinline__ void wait_step(int ahead) {
  if constexpr (NS >= 5) {
    if (ahead >= 3) { wait_vm<12>(); return; }
  }
  if constexpr (NS >= 4) {
    if (ahead >= 2) { wait_vm<8>(); return; }
  }
  if (ahead >= 1) { wait_vm<4>(); return; }
  wait_vm<0>();
}

template <bool A_KC, bool B_KC, int EPI, bool OUT_F32, int NS>
__global__ __launch_bounds__(kThreads, 1) void gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(1024))) char smem[NS * kSlotBytes];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;
  int m0, n0;
  tile_coords(p.M, p.N, BM, BN, m0, n0);

  Operand oa, ob;
  init_operand<A_KC>(oa, p.A, p.lda, p.M, p.K, m0, wid, lane);
  init_operand<B_KC>(ob, p.B, p.ldb, p.N, p.K, n0, wid, lane);

  floatx4 acc[4][8];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BKr - 1) / BKr;
#pragma unroll
  for (int t = 0; t < NS - 1; ++t) {
    if (t < nk) {
      char* slot = smem + t * kSlotBytes;
      issue_tile<A_KC>(oa, slot, t * BKr, wid);
      issue_tile<B_KC>(ob, slot + kTileBytes, t * BKr, wid);
    }
  }

  int cur = 0;  // slot of step t
  for (int t = 0; t < nk; ++t) {
    // steps t+1 .. min(t+NS-2, nk-1) may stay in flight
    const int ahead = min(NS - 2, nk - 1 - t);
    wait_step<NS>(ahead);
    barrier();  // step t visible to all waves; every wave is done with step t-1
    {
      const int tn = t + NS - 1;
      if (tn < nk) {
        const int sl = cur == 0 ? NS - 1 : cur - 1;  // slot of step t-1
        char* slot = smem + sl * kSlotBytes;
        issue_tile<A_KC>(oa, slot, tn * BKr, wid);
        issue_tile<B_KC>(ob, slot + kTileBytes, tn * BKr, wid);
      }
    }
    const char* la = smem + cur * kSlotBytes;
    const char* lb = la + kTileBytes;
    __builtin_amdgcn_s_setprio(1);
    bf16x8 fb[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) fb[j] = read_frag<B_KC, BN, BKr>(lb, wn * 4 + j, 0, lane);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bf16x8 fa[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag<A_KC, BM, BKr>(la, wm * 8 + h * 4 + i, 0, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][h * 4 + i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb[j], fa[i], acc[j][h * 4 + i], 0, 0, 0);
    }
    __builtin_amdgcn_s_setprio(0);
    cur = cur == NS - 1 ? 0 : cur + 1;
  }
  if constexpr (!OUT_F32) {
    barrier();
    epilogue_lds_bf16<EPI>(p, acc, smem, wid, m0 + wm * 128, n0 + wn * 64, lane);
  } else {
    epilogue<EPI, OUT_F32, 8, 4>(p, acc, m0 + wm * 128, n0 + wn * 64, lane);
  }
}

}  // namespace k256r



// =============================================================================
// skinny-N forward GEMM (classifier heads: N <= 64, e.g. 10 classes padded to 16)
// With N this small a 128x128 tile wastes 7/8 of every MFMA and a 4096x16
// output has only 32 tiles, so the K loop runs on 32 CUs (latency-bound).
// Here a workgroup owns a 16-row strip of C; its 4 waves split K in interleaved
// 32-deep steps, load their fragments straight from global/L2 into registers
// (operands are read once: no LDS staging pays), and reduce their partial
// accumulators through LDS before the shared fused epilogue.
// =============================================================================
namespace skinny {

constexpr int kW = 8;  // waves per workgroup (K split 8 ways: more loads in flight per strip)

template <int NT, int EPI>
__global__ __launch_bounds__(kW * 64) void kernel(GemmParams p) {
  __shared__ floatx4 red[kW - 1][NT][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int m0 = blockIdx.x * 16;
  const int row = m0 + (lane & 15);
  const int kq = 8 * (lane >> 4);
  floatx4 acc[NT][1];
#pragma unroll
  for (int j = 0; j < NT; ++j) acc[j][0] = floatx4{0.f, 0.f, 0.f, 0.f};
  const int nsteps = (p.K + 31) / 32;
  const bf16x8 zero = {};
#pragma unroll 8
  for (int st = w; st < nsteps; st += kW) {
    const int k = st * 32 + kq;
    const bool kok = k < p.K;
    const bf16x8 a = (row < p.M && kok) ? *reinterpret_cast<const bf16x8*>(p.A + (size_t)row * p.lda + k) : zero;
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = j * 16 + (lane & 15);
      const bf16x8 b = (n < p.N && kok) ? *reinterpret_cast<const bf16x8*>(p.B + (size_t)n * p.ldb + k) : zero;
      acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(b, a, acc[j][0], 0, 0, 0);
    }
  }
  if (w > 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j) red[w - 1][j][lane] = acc[j][0];
  }
  __syncthreads();
  if (w == 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int q = 0; q < kW - 1; ++q) acc[j][0] += red[q][j][lane];
    epilogue<EPI, false, 1, NT>(p, acc, m0, 0, lane);
  }
}

template <int NT>
hipError_t launch_nt(const GemmParams& p, int epi, hipStream_t s) {
  dim3 grid((p.M + 15) / 16), block(kW * 64);
  switch (epi) {
    case EPI_NONE: kernel<NT, EPI_NONE><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS: kernel<NT, EPI_BIAS><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS_RELU: kernel<NT, EPI_BIAS_RELU><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS_SIGMOID: kernel<NT, EPI_BIAS_SIGMOID><<<grid, block, 0, s>>>(p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace skinny

template <int TILE, bool A_KC, bool B_KC, bool OUT_F32>
hipError_t dispatch_epi(const GemmParams& p, int epi, hipStream_t s) {
  constexpr int T = TILE == 128 ? 128 : 256;
  const int tiles = ((p.M + T - 1) / T) * ((p.N + T - 1) / T);
  dim3 grid(tiles, TILE == 128 ? max(1, p.splitk) : 1);
#define GEMM_EPI_CASE(E)                                                                          \
  case E:                                                                                          \
    if constexpr (TILE == 256) {                                                                   \
      if (p.variant == 2)                                                                          \
        k256r::gemm_kernel<A_KC, B_KC, E, OUT_F32, 4><<<grid, dim3(k256r::kThreads), 0, s>>>(p);  \
      else if (p.variant == 3)                                                                     \
        k256r::gemm_kernel<A_KC, B_KC, E, OUT_F32, 5><<<grid, dim3(k256r::kThreads), 0, s>>>(p);  \
      else                                                                                         \
        k256::gemm_kernel<A_KC, B_KC, E, OUT_F32><<<grid, dim3(k256::kThreads), 0, s>>>(p);       \
    } else {                                                                                       \
      k128::gemm_kernel<A_KC, B_KC, E, OUT_F32><<<grid, dim3(k128::kThreads), 0, s>>>(p);         \
    }                                                                                              \
    break;
  switch (epi) {
    GEMM_EPI_CASE(EPI_NONE)
    GEMM_EPI_CASE(EPI_BIAS)
    GEMM_EPI_CASE(EPI_BIAS_RELU)
    GEMM_EPI_CASE(EPI_BIAS_SIGMOID)
    GEMM_EPI_CASE(EPI_DRELU)
    GEMM_EPI_CASE(EPI_DSIGMOID)
    case EPI_OPT_SGD:
    case EPI_OPT_ADAM:
      if constexpr (OUT_F32 && TILE == 256) {  // the big weight gradients (plain 2-stage main loop)
        if (epi == EPI_OPT_SGD)
          k256::gemm_kernel<A_KC, B_KC, EPI_OPT_SGD, true><<<grid, dim3(k256::kThreads), 0, s>>>(p);
        else
          k256::gemm_kernel<A_KC, B_KC, EPI_OPT_ADAM, true><<<grid, dim3(k256::kThreads), 0, s>>>(p);
      } else if constexpr (OUT_F32) {
        if (epi == EPI_OPT_SGD)
          k128::gemm_kernel<A_KC, B_KC, EPI_OPT_SGD, true><<<grid, dim3(k128::kThreads), 0, s>>>(p);
        else
          k128::gemm_kernel<A_KC, B_KC, EPI_OPT_ADAM, true><<<grid, dim3(k128::kThreads), 0, s>>>(p);
      } else {
        return hipErrorInvalidValue;
      }
      break;
    default:
      return hipErrorInvalidValue;
  }
#undef GEMM_EPI_CASE
  return hipGetLastError();
}

template <int TILE>
hipError_t dispatch_layout(const GemmParams& p, bool a_kc, bool b_kc, int epi, bool f32, hipStream_t s) {
  if (a_kc) {
    if (b_kc) return f32 ? dispatch_epi<TILE, true, true, true>(p, epi, s) : dispatch_epi<TILE, true, true, false>(p, epi, s);
    return f32 ? dispatch_epi<TILE, true, false, true>(p, epi, s) : dispatch_epi<TILE, true, false, false>(p, epi, s);
  }
  if (b_kc) return f32 ? dispatch_epi<TILE, false, true, true>(p, epi, s) : dispatch_epi<TILE, false, true, false>(p, epi, s);
  return f32 ? dispatch_epi<TILE, false, false, true>(p, epi, s) : dispatch_epi<TILE, false, false, false>(p, epi, s);
}

}  // namespace

int gemm_pick_tile(int M, int N, int K, bool out_f32) {
  const int t256 = ((M + 255) / 256) * ((N + 255) / 256);
  // a 256^2 tile needs the grid to cover most of the 256 CUs and a K loop long
  // enough to amortise its 2-tile prologue -- or a bf16 output whose LDS-staged
  // epilogue (row-coalesced stores) is the bottleneck at tiny K
  if (t256 >= 192 && (K >= 256 || !out_f32)) return 256;
  return 128;
}

int gemm_pick_splitk(int M, int N, int K) {
  const int tiles = ((M + 127) / 128) * ((N + 127) / 128);
  // fp32 atomics run at ~1.3 TB/s chip-wide: only worth it when the grid is tiny
  if (tiles >= 128) return 1;
  int sk = (512 + tiles - 1) / tiles;  // aim at ~2 workgroups per CU
  const int max_by_k = K / 512;        // keep >= 8 K-tiles per split
  if (sk > max_by_k) sk = max_by_k;
  return sk < 2 ? 1 : (sk > 32 ? 32 : sk);
}

int gemm_tiles128(int M, int N) { return ((M + 127) / 128) * ((N + 127) / 128); }

size_t gemm_splitk_ws_bytes(int M, int N, int splitk) {
  return (size_t)gemm_tiles128(M, N) * (size_t)splitk * (size_t)(16 * k128::kThreads * 16);
}

hipError_t gemm_bf16(const GemmParams& p, bool a_kcontig, bool b_kcontig, int epi, bool out_f32,
                     hipStream_t s) {
  return gemm_bf16_tile(p, a_kcontig, b_kcontig, epi, out_f32, gemm_pick_tile(p.M, p.N, p.K, out_f32), s);
}

hipError_t gemm_bf16_tile(const GemmParams& p, bool a_kcontig, bool b_kcontig, int epi, bool out_f32, int tile,
                          hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (tile >= 256) {
    // buffer resources address at most 2 GiB per operand
    const size_t abytes = (size_t)(a_kcontig ? p.M : p.K) * p.lda * 2;
    const size_t bbytes = (size_t)(b_kcontig ? p.N : p.K) * p.ldb * 2;
    if (abytes >= kOOBLimit || bbytes >= kOOBLimit) tile = 128;
  }
  if (tile == 256) return dispatch_layout<256>(p, a_kcontig, b_kcontig, epi, out_f32, s);
  GemmParams q = p;
  if (q.splitk > 1 && q.cnt == nullptr) {
    if (!(out_f32 && epi == EPI_NONE && q.dbias == nullptr)) return hipErrorInvalidValue;
    if (q.beta == 0.f) {
      hipError_t e = zero2d_f32(reinterpret_cast<float*>(q.C), q.M, q.N, q.ldc, s);
      if (e != hipSuccess) return e;
    } else if (q.beta != 1.f) {
      return hipErrorInvalidValue;  // split-K accumulates: beta must be 0 or 1
    }
  }
  return dispatch_layout<128>(q, a_kcontig, b_kcontig, epi, out_f32, s);
}

}  // namespace ldnn

namespace ldnn {

hipError_t gemm_skinny_n(const GemmParams& p, int epi, hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (p.N > 64) return hipErrorInvalidValue;
  switch ((p.N + 15) / 16) {
    case 1: return skinny::launch_nt<1>(p, epi, s);
    case 2: return skinny::launch_nt<2>(p, epi, s);
    case 3: return skinny::launch_nt<3>(p, epi, s);
    default: return skinny::launch_nt<4>(p, epi, s);
  }
}

}  // namespace ldnn
