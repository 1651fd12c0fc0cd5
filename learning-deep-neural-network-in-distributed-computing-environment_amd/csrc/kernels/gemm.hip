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
// Tiling (CDNA4-first, see /opt/skills/guides/cdna_hip_programming.md §5):
//   * 128x128 output tile, BK = 64, 256 threads = 4 waves (2x2), 64x64 per wave,
//     v_mfma_f32_16x16x32_bf16 (4x4 accumulators of 16x16 per wave).
//   * MFMA roles swapped (MFMA-A <- our B tile, MFMA-B <- our A tile) so each lane
//     ends up owning 4 consecutive output columns: bf16 epilogue stores are 8 B,
//     fp32 are 16 B, and a bias/activation needs 4 contiguous bias values.
//   * k-contiguous operands are staged as [128 rows][64 k] with a 16-B chunk XOR
//     swizzle (chunk ^ (row & 7)) -> conflict-free ds_read_b128 fragment reads.
//   * k-strided operands are staged as [k/8][rows/16][8][16] 256-B blocks and
//     read with ds_read_b64_tr_b16 (hardware transpose); odd k-blocks store
//     k-rows 0-3 <-> 4-7 swapped so the two 16-lane groups of a half-wave read
//     opposite 128-B halves of the bank row (conflict-free).
//   * Register-staged double-buffered LDS: issue tile t+1's global loads before
//     computing tile t, write them to the other LDS buffer after, one barrier
//     per K-step (T3 minimum / T14).  All LDS in ONE __shared__ array.
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
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

constexpr int BM = 128, BN = 128, BK = 64;
constexpr int kThreads = 256;
constexpr int kTileBytes = 128 * BK * 2;  // 16 KiB per operand tile
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// ---- staging: global -> registers -------------------------------------------
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

// ---- staging: registers -> LDS image --------------------------------------
template <bool KC>
__device__ __forceinline__ void store_tile(const u32x4 (&r)[4], char* lds, int tid) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = tid + kThreads * i;
    int off;
    if constexpr (KC) {
      const int kc = c & 7, row = c >> 3;
      off = row * 128 + ((kc ^ (row & 7)) << 4);
    } else {
      const int half = c & 1, klo = (c >> 1) & 3, rb = (c >> 3) & 7, khi = c >> 6;
      const int k = khi * 4 + klo;
      const int kb = k >> 3;
      const int rowp = (k & 7) ^ ((kb & 1) << 2);
      off = (kb * 8 + rb) * 256 + rowp * 32 + half * 16;
    }
    *reinterpret_cast<u32x4*>(lds + off) = r[i];
  }
}

// ---- fragment read: 16 rows (row tile rt) x 8 consecutive k (k-sub kk) ------
// Lane l gets row (l & 15), k = kk*32 + 8*(l >> 4) + j, j = 0..7: the operand map
// of v_mfma_f32_16x16x32_bf16 for both its A and its B operand.
template <bool KC>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int rt, int kk, int lane) {
  if constexpr (KC) {
    const int row = rt * 16 + (lane & 15);
    const int chunk = kk * 4 + (lane >> 4);
    return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ (row & 7)) << 4));
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int kb = kk * 4 + g;
    const int sw = (kb & 1) << 2;
    const char* blk = lds + (kb * 8 + rt) * 256;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(blk + ((q ^ sw) * 32) + p * 8));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(blk + (((4 + q) ^ sw) * 32) + p * 8));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

template <int EPI>
__device__ __forceinline__ float apply_epi(float v, float bias, float aux) {
  if constexpr (EPI == EPI_BIAS) return v + bias;
  if constexpr (EPI == EPI_BIAS_RELU) return fmaxf(v + bias, 0.f);
  if constexpr (EPI == EPI_BIAS_SIGMOID) return 1.f / (1.f + __expf(-(v + bias)));
  if constexpr (EPI == EPI_DRELU) return aux > 0.f ? v : 0.f;
  if constexpr (EPI == EPI_DSIGMOID) return v * aux * (1.f - aux);
  return v;
}

template <bool A_KC, bool B_KC, int EPI, bool OUT_F32>
__global__ __launch_bounds__(kThreads, 2) void gemm_kernel(GemmParams p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * kTileBytes];  // [buf][A|B]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // ---- tile id: XCD remap, then grouped ordering for L2 reuse
  const int tiles_m = (p.M + BM - 1) / BM, tiles_n = (p.N + BN - 1) / BN;
  const int nwg = tiles_m * tiles_n;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int per_group = GROUP_M * tiles_n;
  const int group = id / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  const int tm = first_m + (id % per_group) % gsize;
  const int tn = (id % per_group) / gsize;
  const int m0 = tm * BM, n0 = tn * BN;

  floatx4 acc[4][4];  // [n-tile j][m-tile i]
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};

  const int nk = (p.K + BK - 1) / BK;
  u32x4 ra[4], rb[4];
  load_tile<A_KC>(ra, p.A, p.lda, p.M, p.K, m0, 0, tid);
  load_tile<B_KC>(rb, p.B, p.ldb, p.N, p.K, n0, 0, tid);
  store_tile<A_KC>(ra, smem, tid);
  store_tile<B_KC>(rb, smem + kTileBytes, tid);
  __syncthreads();

  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    const bool more = (kt + 1) < nk;
    if (more) {
      load_tile<A_KC>(ra, p.A, p.lda, p.M, p.K, m0, (kt + 1) * BK, tid);
      load_tile<B_KC>(rb, p.B, p.ldb, p.N, p.K, n0, (kt + 1) * BK, tid);
    }
    const char* la = smem + cur * 2 * kTileBytes;
    const char* lb = la + kTileBytes;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 fa[4], fb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) fa[i] = read_frag<A_KC>(la, wm * 4 + i, kk, lane);
#pragma unroll
      for (int j = 0; j < 4; ++j) fb[j] = read_frag<B_KC>(lb, wn * 4 + j, kk, lane);
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

  // ---- epilogue: lane owns C[m][n..n+3] for each (i, j)
  const bool do_dbias = p.dbias != nullptr;
  float colsum[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < 4; ++r) colsum[j][r] = 0.f;

#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
    const bool nok = n < p.N;  // N % 8 == 0 is enforced on the host
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_SIGMOID) {
      if (nok) {
        const floatx4 b4 = *reinterpret_cast<const floatx4*>(p.bias + n);
        bias[0] = b4[0]; bias[1] = b4[1]; bias[2] = b4[2]; bias[3] = b4[3];
      }
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int m = m0 + wm * 64 + i * 16 + (lane & 15);
      if (!(nok && m < p.M)) continue;
      float aux[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == EPI_DRELU || EPI == EPI_DSIGMOID) {
        const u16x4 a4 = *reinterpret_cast<const u16x4*>(p.aux + (size_t)m * p.ldaux + n);
        aux[0] = bf2f(a4[0]); aux[1] = bf2f(a4[1]); aux[2] = bf2f(a4[2]); aux[3] = bf2f(a4[3]);
      }
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = apply_epi<EPI>(acc[j][i][r], bias[r], aux[r]);
      if constexpr (OUT_F32) {
        float* c = reinterpret_cast<float*>(p.C) + (size_t)m * p.ldc + n;
        floatx4 o{v[0], v[1], v[2], v[3]};
        if (p.beta != 0.f) {
          const floatx4 old = *reinterpret_cast<const floatx4*>(c);
          o = o + p.beta * old;
        }
        *reinterpret_cast<floatx4*>(c) = o;
#pragma unroll
        for (int r = 0; r < 4; ++r) colsum[j][r] += o[r];
      } else {
        u16x4 o;
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = f2bf(v[r]);
        *reinterpret_cast<u16x4*>(reinterpret_cast<bf16_t*>(p.C) + (size_t)m * p.ldc + n) = o;
#pragma unroll
        for (int r = 0; r < 4; ++r) colsum[j][r] += bf2f(o[r]);
      }
    }
  }

  if (do_dbias) {
    // reduce over the 16 lanes that share (lane >> 4), i.e. over m
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float s = colsum[j][r];
        s += __shfl_xor(s, 1, 64);
        s += __shfl_xor(s, 2, 64);
        s += __shfl_xor(s, 4, 64);
        s += __shfl_xor(s, 8, 64);
        colsum[j][r] = s;
      }
    if ((lane & 15) == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = n0 + wn * 64 + j * 16 + 4 * (lane >> 4);
        if (n < p.N) {
#pragma unroll
          for (int r = 0; r < 4; ++r) atomicAdd(p.dbias + n + r, colsum[j][r]);
        }
      }
    }
  }
}

template <bool A_KC, bool B_KC, bool OUT_F32>
hipError_t dispatch_epi(const GemmParams& p, int epi, hipStream_t s) {
  const int tiles = ((p.M + BM - 1) / BM) * ((p.N + BN - 1) / BN);
  dim3 grid(tiles), block(kThreads);
  switch (epi) {
    case EPI_NONE: gemm_kernel<A_KC, B_KC, EPI_NONE, OUT_F32><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS: gemm_kernel<A_KC, B_KC, EPI_BIAS, OUT_F32><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS_RELU: gemm_kernel<A_KC, B_KC, EPI_BIAS_RELU, OUT_F32><<<grid, block, 0, s>>>(p); break;
    case EPI_BIAS_SIGMOID: gemm_kernel<A_KC, B_KC, EPI_BIAS_SIGMOID, OUT_F32><<<grid, block, 0, s>>>(p); break;
    case EPI_DRELU: gemm_kernel<A_KC, B_KC, EPI_DRELU, OUT_F32><<<grid, block, 0, s>>>(p); break;
    case EPI_DSIGMOID: gemm_kernel<A_KC, B_KC, EPI_DSIGMOID, OUT_F32><<<grid, block, 0, s>>>(p); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

hipError_t gemm_bf16(const GemmParams& p, bool a_kcontig, bool b_kcontig, int epi, bool out_f32,
                     hipStream_t s) {
  if (p.M <= 0 || p.N <= 0) return hipSuccess;
  if (a_kcontig) {
    if (b_kcontig) return out_f32 ? dispatch_epi<true, true, true>(p, epi, s) : dispatch_epi<true, true, false>(p, epi, s);
    return out_f32 ? dispatch_epi<true, false, true>(p, epi, s) : dispatch_epi<true, false, false>(p, epi, s);
  }
  if (b_kcontig) return out_f32 ? dispatch_epi<false, true, true>(p, epi, s) : dispatch_epi<false, true, false>(p, epi, s);
  return out_f32 ? dispatch_epi<false, false, true>(p, epi, s) : dispatch_epi<false, false, false>(p, epi, s);
}

}  // namespace ldnn
