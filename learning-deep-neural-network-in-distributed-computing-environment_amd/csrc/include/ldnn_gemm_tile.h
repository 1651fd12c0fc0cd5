// Shared device-side building blocks of the MFMA GEMM and implicit-GEMM conv
// kernels (gemm.hip, conv.hip): LDS image layouts, fragment reads, the fused
// epilogue, XCD-aware tile mapping.  Header-only, internal linkage per TU.
#pragma once
#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {
namespace {

constexpr int BK = 64;
constexpr int GROUP_M = 8;

typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;
typedef __attribute__((address_space(3))) void lds_void;

// ---- LDS image addressing --------------------------------------------------
// KC image, BK 64:  [ROWS][64 k], 128-B rows, chunk' = chunk ^ (row & 7)
// KC image, BK 32:  [ROWS][32 k],  64-B rows, chunk' = chunk ^ (row & 8 ? 3 : 0)
//   (ds_read_b128 lane groups {0-3,12-15,20-27}, ... each cover all 64 banks)
// strided image:    [BK/8 kb][ROWS/16 rb][8 k][16 r], 256-B blocks, odd kb: k ^= 4
__device__ __forceinline__ int kc32_sw(int row) { return (row & 8) ? 3 : 0; }

template <bool KC, int ROWS, int BKt = BK>
__device__ __forceinline__ int lds_offset(int row, int k) {
  if constexpr (KC) {
    if constexpr (BKt == 64) return row * 128 + ((((k >> 3) ^ (row & 7))) << 4) + (k & 7) * 2;
    else return row * 64 + ((((k >> 3) ^ kc32_sw(row))) << 4) + (k & 7) * 2;
  } else {
    const int kb = k >> 3, rb = row >> 4;
    const int rowp = (k & 7) ^ ((kb & 1) << 2);
    return (kb * (ROWS / 16) + rb) * 256 + rowp * 32 + (row & 15) * 2;
  }
}

// Inverse map: which (row, k) lands at 16-B LDS slot `o` (o multiple of 16).
template <bool KC, int ROWS, int BKt = BK>
__device__ __forceinline__ void lds_slot_to_rk(int o, int& row, int& k) {
  if constexpr (KC) {
    if constexpr (BKt == 64) {
      row = o >> 7;
      const int pch = (o >> 4) & 7;
      k = (pch ^ (row & 7)) * 8;
    } else {
      row = o >> 6;
      const int pch = (o >> 4) & 3;
      k = (pch ^ kc32_sw(row)) * 8;
    }
  } else {
    const int blk = o >> 8;
    const int kb = blk / (ROWS / 16), rb = blk % (ROWS / 16);
    const int rowp = (o >> 5) & 7, half = (o >> 4) & 1;
    k = kb * 8 + (rowp ^ ((kb & 1) << 2));
    row = rb * 16 + half * 8;
  }
}

// ---- fragment read: 16 rows (row tile rt) x 8 consecutive k (k-sub kk) ------
// Lane l gets row (l & 15), k = kk*32 + 8*(l >> 4) + j, j = 0..7: the operand map
// of v_mfma_f32_16x16x32_bf16 for both its A and its B operand.
template <bool KC, int ROWS, int BKt = BK>
__device__ __forceinline__ bf16x8 read_frag(const char* lds, int rt, int kk, int lane) {
  if constexpr (KC) {
    const int row = rt * 16 + (lane & 15);
    const int chunk = kk * 4 + (lane >> 4);
    if constexpr (BKt == 64)
      return *reinterpret_cast<const bf16x8*>(lds + row * 128 + ((chunk ^ (row & 7)) << 4));
    else
      return *reinterpret_cast<const bf16x8*>(lds + row * 64 + ((chunk ^ kc32_sw(row)) << 4));
  } else {
    const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
    const int kb = kk * 4 + g;
    const int sw = (kb & 1) << 2;
    const char* blk = lds + (kb * (ROWS / 16) + rt) * 256;
    const bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(blk + ((q ^ sw) * 32) + p * 8));
    const bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(blk + (((4 + q) ^ sw) * 32) + p * 8));
    return bf16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  }
}

template <int EPI>
__device__ __forceinline__ float apply_epi(float v, float bias, float aux) {
  if constexpr (EPI == EPI_BIAS) return v + bias;
  if constexpr (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_RELU_MASK) return fmaxf(v + bias, 0.f);
  if constexpr (EPI == EPI_BIAS_SIGMOID) return 1.f / (1.f + __expf(-(v + bias)));
  if constexpr (EPI == EPI_DRELU || EPI == EPI_DRELU_MASK) return aux > 0.f ? v : 0.f;
  if constexpr (EPI == EPI_DSIGMOID) return v * aux * (1.f - aux);
  return v;
}

// Tile id -> (tm, tn): XCD remap, then GROUP_M-row groups for L2 reuse.  (bid: the workgroup's
// x index -- blockIdx.x, or a virtual one when two GEMMs share a launch)
__device__ __forceinline__ void tile_coords_id(int M, int N, int BMt, int BNt, int bid, int& m0, int& n0) {
  const int tiles_m = (M + BMt - 1) / BMt, tiles_n = (N + BNt - 1) / BNt;
  const int nwg = tiles_m * tiles_n;
  const int id = xcd_remap(bid, nwg);
  const int per_group = GROUP_M * tiles_n;
  const int group = id / per_group;
  const int first_m = group * GROUP_M;
  const int gsize = min(tiles_m - first_m, GROUP_M);
  m0 = (first_m + (id % per_group) % gsize) * BMt;
  n0 = ((id % per_group) / gsize) * BNt;
}
__device__ __forceinline__ void tile_coords(int M, int N, int BMt, int BNt, int& m0, int& n0) {
  tile_coords_id(M, N, BMt, BNt, (int)blockIdx.x, m0, n0);
}

// ---- fused optimizer update of 4 consecutive weights (EPI_OPT_*) -------------
// Same arithmetic as optim.hip's sgd / adam kernels (torch semantics), applied
// in the wgrad epilogue so the gradient never round-trips through HBM.
struct OptConst {
  float lr, bc1, bc2s;
};

template <int EPI>
__device__ __forceinline__ OptConst opt_const(const OptEpi& o) {
  OptConst c;
  c.lr = o.hp[0];
  c.bc1 = 1.f;
  c.bc2s = 1.f;
  if constexpr (EPI == EPI_OPT_ADAM) {
    const float t = o.hp[1];
    c.bc1 = 1.f - powf(o.beta1, t);
    c.bc2s = sqrtf(1.f - powf(o.beta2, t));
  }
  return c;
}

// The update arithmetic on registers: p (weights), m (momentum / exp_avg), v (exp_avg_sq).
template <int EPI>
__device__ __forceinline__ void opt_math(const OptEpi& o, const OptConst& k, floatx4& p, floatx4& m, floatx4& v,
                                         floatx4 g) {
  g = g * o.grad_scale;
  if constexpr (EPI == EPI_OPT_SGD) {
    if (o.weight_decay != 0.f) g += o.weight_decay * p;
    if (o.m != nullptr) {
      m = o.momentum * m + (1.f - o.dampening) * g;
      g = o.nesterov ? g + o.momentum * m : m;
    }
    p -= k.lr * g;
  } else {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      float gr = g[r], pr = p[r];
      if (o.weight_decay != 0.f) {
        if (o.decoupled) pr *= (1.f - k.lr * o.weight_decay);
        else gr += o.weight_decay * pr;
      }
      m[r] = o.beta1 * m[r] + (1.f - o.beta1) * gr;
      v[r] = o.beta2 * v[r] + (1.f - o.beta2) * gr * gr;
      p[r] = pr - (k.lr / k.bc1) * m[r] / (sqrtf(v[r]) / k.bc2s + o.eps);
    }
  }
}

template <int EPI>
__device__ __forceinline__ void opt_load4(const OptEpi& o, size_t off, floatx4& p, floatx4& m, floatx4& v) {
  // (streaming accesses: every optimizer byte is touched once per step, as in optim.hip)
  p = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(o.master + off));
  m = floatx4{0.f, 0.f, 0.f, 0.f};
  v = m;
  if (o.m != nullptr) m = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(o.m + off));
  if constexpr (EPI == EPI_OPT_ADAM) v = __builtin_nontemporal_load(reinterpret_cast<const floatx4*>(o.v + off));
}

template <int EPI>
__device__ __forceinline__ void opt_store4(const OptEpi& o, size_t off, const floatx4& p, const floatx4& m,
                                           const floatx4& v) {
  if (o.m != nullptr) __builtin_nontemporal_store(m, reinterpret_cast<floatx4*>(o.m + off));
  if constexpr (EPI == EPI_OPT_ADAM) __builtin_nontemporal_store(v, reinterpret_cast<floatx4*>(o.v + off));
  __builtin_nontemporal_store(p, reinterpret_cast<floatx4*>(o.master + off));
  if (o.shadow) *reinterpret_cast<u16x4*>(o.shadow + off) = u16x4{f2bf(p[0]), f2bf(p[1]), f2bf(p[2]), f2bf(p[3])};
}

template <int EPI>
__device__ __forceinline__ void opt_update4(const OptEpi& o, const OptConst& k, size_t off, floatx4 g) {
  floatx4 p, m, v;
  opt_load4<EPI>(o, off, p, m, v);
  opt_math<EPI>(o, k, p, m, v, g);
  opt_store4<EPI>(o, off, p, m, v);
}

// U independent 8-weight runs (two floatx4 each, at off[u] and off[u] + 4): every
// state load of the batch is issued before its first store, so a lane keeps up to
// 6 U 16-B loads in flight instead of one load -> store round trip per run.
template <int EPI, int U>
__device__ __forceinline__ void opt_update8_batch(const OptEpi& o, const OptConst& k, const size_t (&off)[U],
                                                  const bool (&ok)[U], const floatx4 (&g)[U][2]) {
  floatx4 p[U][2], m[U][2], v[U][2];
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (ok[u]) opt_load4<EPI>(o, off[u] + 4 * h, p[u][h], m[u][h], v[u][h]);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int h = 0; h < 2; ++h)
      if (ok[u]) {
        opt_math<EPI>(o, k, p[u][h], m[u][h], v[u][h], g[u][h]);
        opt_store4<EPI>(o, off[u] + 4 * h, p[u][h], m[u][h], v[u][h]);
      }
}

// ---- shared epilogue: acc[j][i] is the 16x16 tile (n-tile j, m-tile i) -----
// Processed one n-tile at a time (sched_barrier keeps the compiler from hoisting
// every bias/aux load of the tile up front), with the optional bias-gradient
// column sum reduced and atomically added per n-tile, so only a handful of
// registers are live beside the accumulators.
template <int EPI, bool OUT_F32, int MT, int NT>
__device__ __forceinline__ void epilogue(const GemmParams& p, floatx4 (&acc)[NT][MT], int mbase, int nbase,
                                         int lane) {
  if constexpr (EPI == EPI_OPT_SGD || EPI == EPI_OPT_ADAM) {
    static_assert(OUT_F32, "optimizer epilogues take the fp32 gradient");
    const OptConst k = opt_const<EPI>(p.opt);
#pragma unroll
    for (int j = 0; j < NT; ++j) {
      const int n = nbase + j * 16 + 4 * (lane >> 4);
      if (n >= p.N) continue;
#pragma unroll
      for (int i = 0; i < MT; ++i) {
        const int m = mbase + i * 16 + (lane & 15);
        if (m < p.M) opt_update4<EPI>(p.opt, k, (size_t)m * p.ldc + n, acc[j][i]);
      }
    }
    return;
  }
  const bool do_dbias = p.dbias != nullptr;
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    __builtin_amdgcn_sched_barrier(0);
    const int n = nbase + j * 16 + 4 * (lane >> 4);
    const bool nok = n < p.N;  // N % 8 == 0 is enforced on the host
    floatx4 bias = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_SIGMOID) {
      if (nok) bias = *reinterpret_cast<const floatx4*>(p.bias + n);
    }
    floatx4 cs = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MT; ++i) {
      const int m = mbase + i * 16 + (lane & 15);
      if (nok && m < p.M) {
        floatx4 aux = {0.f, 0.f, 0.f, 0.f};
        if constexpr (EPI == EPI_DRELU || EPI == EPI_DSIGMOID) {
          const u16x4 a4 = *reinterpret_cast<const u16x4*>(p.aux + (size_t)m * p.ldaux + n);
          aux = floatx4{bf2f(a4[0]), bf2f(a4[1]), bf2f(a4[2]), bf2f(a4[3])};
        }
        floatx4 v;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = apply_epi<EPI>(acc[j][i][r], bias[r], aux[r]);
        if constexpr (OUT_F32) {
          float* c = reinterpret_cast<float*>(p.C) + (size_t)m * p.ldc + n;
          if (p.beta != 0.f) v = v + p.beta * *reinterpret_cast<const floatx4*>(c);
          *reinterpret_cast<floatx4*>(c) = v;
          cs += v;
        } else {
          const u16x4 o{f2bf(v[0]), f2bf(v[1]), f2bf(v[2]), f2bf(v[3])};
          *reinterpret_cast<u16x4*>(reinterpret_cast<bf16_t*>(p.C) + (size_t)m * p.ldc + n) = o;
          cs += floatx4{bf2f(o[0]), bf2f(o[1]), bf2f(o[2]), bf2f(o[3])};
        }
      }
    }
    if (do_dbias) {
      // reduce over the 16 lanes that share (lane >> 4), i.e. over m
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float t = cs[r];
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 4, 64);
        t += __shfl_xor(t, 8, 64);
        cs[r] = t;
      }
      if ((lane & 15) == 0 && nok) {
#pragma unroll
        for (int r = 0; r < 4; ++r) atomicAdd(p.dbias + n + r, cs[r]);
      }
    }
  }
}

// LDS-staged bf16 epilogue: each wave parks its fp32 128x64 tile in LDS (two
// 64-row halves of 16 KiB, 16-B chunk XOR-swizzled by row so the staging
// writes are conflict-free), then re-reads it ROW-wise: 8 lanes cover one
// 64-column row segment, so aux loads and output stores are full 128-B row
// runs instead of 16 rows x 32 B per instruction.  Bias-gradient column sums
// stay per lane (8 fixed columns) and are shuffle-reduced once at the end.
template <int EPI>
__device__ __forceinline__ void epilogue_lds_bf16(const GemmParams& p, floatx4 (&acc)[4][8], char* smem, int wid,
                                                  int mbase, int nbase, int lane) {
  float* wbuf = reinterpret_cast<float*>(smem + wid * 16384);  // [64 rows][64 cols] fp32, swizzled
  const int col8 = lane & 7;                                     // this lane's 8 columns
  const int n = nbase + col8 * 8;
  const bool nok = n < p.N;
  float bias[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RELU || EPI == EPI_BIAS_SIGMOID) {
    if (nok) {
      const floatx4 b0 = *reinterpret_cast<const floatx4*>(p.bias + n);
      const floatx4 b1 = *reinterpret_cast<const floatx4*>(p.bias + n + 4);
      bias[0] = b0[0]; bias[1] = b0[1]; bias[2] = b0[2]; bias[3] = b0[3];
      bias[4] = b1[0]; bias[5] = b1[1]; bias[6] = b1[2]; bias[7] = b1[3];
    }
  }
  float cs[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    // stage m-tiles 4h..4h+3: lane holds C[m = i*16 + (l&15)][n = j*16 + 4*(l>>4) + r]
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = i * 16 + (lane & 15);
        const int chunk = j * 4 + (lane >> 4);  // 16-B chunk (4 floats) within the 256-B row
        *reinterpret_cast<floatx4*>(reinterpret_cast<char*>(wbuf) + row * 256 + ((chunk ^ (row & 15)) << 4)) =
            acc[j][h * 4 + i];
      }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): own staging writes landed (wave-private region)
    __builtin_amdgcn_wave_barrier();
#pragma unroll 2
    for (int it = 0; it < 8; ++it) {
      const int row = it * 8 + (lane >> 3);
      const int m = mbase + h * 64 + row;
      const char* rb = reinterpret_cast<const char*>(wbuf) + row * 256;
      const floatx4 v0 = *reinterpret_cast<const floatx4*>(rb + (((2 * col8) ^ (row & 15)) << 4));
      const floatx4 v1 = *reinterpret_cast<const floatx4*>(rb + (((2 * col8 + 1) ^ (row & 15)) << 4));
      if (!(nok && m < p.M)) continue;
      float aux[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == EPI_DRELU || EPI == EPI_DSIGMOID) {
        const u16x8 a8 = *reinterpret_cast<const u16x8*>(p.aux + (size_t)m * p.ldaux + n);
#pragma unroll
        for (int q = 0; q < 8; ++q) aux[q] = bf2f(a8[q]);
      }
      u16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const float v = apply_epi<EPI>(q < 4 ? v0[q] : v1[q - 4], bias[q], aux[q]);
        o[q] = f2bf(v);
        cs[q] += bf2f(o[q]);
      }
      *reinterpret_cast<u16x8*>(reinterpret_cast<bf16_t*>(p.C) + (size_t)m * p.ldc + n) = o;
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (p.dbias != nullptr) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float t = cs[q];
      t += __shfl_xor(t, 8, 64);
      t += __shfl_xor(t, 16, 64);
      t += __shfl_xor(t, 32, 64);
      cs[q] = t;
    }
    if (lane < 8 && nok) {
#pragma unroll
      for (int q = 0; q < 8; ++q) atomicAdd(p.dbias + n + q, cs[q]);
    }
  }
}

// ---- in-launch split-K combine ----------------------------------------------
// (cdna_hip_programming.md §5 "Projection GEMM at M = 256" item 2, write-through
// form; §6 Guideline 16.)  Every K-slice workgroup stores its fp32 accumulators
// WRITE-THROUGH (sc1) into its own slab of the tile's workspace, in
// thread-linear order, so the reducer thread with the same tid reads back
// exactly the fragments it owns (16-B per lane per register, fully coalesced).
// Every wave drains its stores, and after a workgroup barrier one lane draws a
// ticket from the tile's counter (relaxed agent-scope atomic).  The workgroup
// that draws the last ticket resets the counter, acquires at agent scope, sums
// ALL slabs in slice order with sc1 loads -- deterministic, independent of the
// arrival order -- and returns true: the caller then runs its normal epilogue
// on the full sum.  The others return false.  `cnt` must be zero before the
// first launch (callers allocate it zeroed); the reducer leaves it zero again.
// `smem` is any 4 bytes of the kernel's (single) LDS array, free by now.
constexpr int kSc1 = 16;  // buffer cache-policy bit: sc1 (write-through / L1 bypass)

template <int NT, int MT, int NTHREADS>
__device__ __forceinline__ bool splitk_combine(floatx4 (&acc)[NT][MT], float* ws, int* cnt, int tile, int splits,
                                               int split, char* smem, uint64_t* tr = nullptr) {
  // tr (phase-trace builds, thread 0 only): [4] slab stores drained, [5] ticket drawn, [6] slabs summed
  constexpr uint32_t kSlab = (uint32_t)(NT * MT) * NTHREADS * 16u;
  const int tid = threadIdx.x;
  const uint32_t tile_bytes = kSlab * (uint32_t)splits;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char*>(ws) + (size_t)tile * tile_bytes, (short)0, (int)tile_bytes, 0x00020000);
  const uint32_t own = (uint32_t)split * kSlab + (uint32_t)tid * 16u;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[j][i]), rs,
                                             (int)(own + (uint32_t)((j * MT + i) * NTHREADS * 16)), 0, kSc1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its slab stores
  __syncthreads();
  if (tr != nullptr) tr[4] = __builtin_amdgcn_s_memrealtime();
  int* flag = reinterpret_cast<int*>(smem);
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == splits - 1 ? 1 : 0;
    if (last) {
      __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *flag = last;
  }
  __syncthreads();
  if (tr != nullptr) tr[5] = __builtin_amdgcn_s_memrealtime();
  if (*flag == 0) return false;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < MT; ++i) acc[j][i] = floatx4{0.f, 0.f, 0.f, 0.f};
  auto load = [&](int s, int j, int i) {
    const uint32_t o = (uint32_t)s * kSlab + (uint32_t)tid * 16u;
    return __builtin_bit_cast(
        floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(o + (uint32_t)((j * MT + i) * NTHREADS * 16)), 0,
                                                       kSc1));
  };
  int s = 0;
  if constexpr (NT * MT <= 16) {
    // two slabs per round trip (the summing workgroup's combine is latency-bound: one
    // split's 64 KiB per round trip left a 4-way split's last arrival ~20 us in its tail)
    for (; s + 1 < splits; s += 2) {
      floatx4 t0[NT][MT], t1[NT][MT];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          t0[j][i] = load(s, j, i);
          t1[j][i] = load(s + 1, j, i);
        }
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[j][i] += t0[j][i] + t1[j][i];
    }
  }
  for (; s < splits; ++s) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[j][i] += load(s, j, i);
  }
  if (tr != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr[6] = __builtin_amdgcn_s_memrealtime();
  }
  return true;
}

// The same hand-off with a FIXED summer: the tile's last K slice (split == splits - 1).  The
// other slices deposit their slabs (write-through, drained) and count themselves in; the summer
// never stores its own partial -- it waits until all the others are in, then adds their slabs to
// its registers in slice order (deterministic: own + s_0 + s_1 + ...).  That removes the
// summer's 64 KiB store drain, its ticket and the re-read of its own slab: EnhancedCNN's 16x16 /
// 8x8 convs measured the last arriver at 2.5 us store drain + 0.7 ticket + 1.3 waiting for the
// last + 2.5-3.4 summing + 1.4 epilogue (profiles/r5/conv_phase_trace_combine.jsonl).
// Progress: the summer waits only for workgroups of LOWER linear id (same tile, lower slice) --
// the dispatcher issues a kernel's workgroups to each XCD in id order, so every workgroup the
// summer waits for was dispatched before it and waits for nothing itself; a capped spin keeps
// even a broken assumption from hanging the GPU.  Callers must not remap (tile, slice) to
// workgroup ids (xcd_split).
template <int NT, int MT, int NTHREADS>
__device__ __forceinline__ bool splitk_combine_last(floatx4 (&acc)[NT][MT], float* ws, int* cnt, int tile, int splits,
                                                    int split, char* smem, uint64_t* tr = nullptr) {
  constexpr uint32_t kSlab = (uint32_t)(NT * MT) * NTHREADS * 16u;
  const int tid = threadIdx.x;
  const uint32_t tile_bytes = kSlab * (uint32_t)(splits - 1);
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char*>(ws) + (size_t)tile * kSlab * (uint32_t)splits, (short)0, (int)tile_bytes, 0x00020000);
  if (split != splits - 1) {
    const uint32_t own = (uint32_t)split * kSlab + (uint32_t)tid * 16u;
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[j][i]), rs,
                                               (int)(own + (uint32_t)((j * MT + i) * NTHREADS * 16)), 0, kSc1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // EVERY storing wave drains its slab stores
    __syncthreads();
    if (tr != nullptr) tr[4] = __builtin_amdgcn_s_memrealtime();
    if (tid == 0) __hip_atomic_fetch_add(cnt + tile, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return false;
  }
  if (tid == 0) {
    if (tr != nullptr) tr[4] = __builtin_amdgcn_s_memrealtime();
    for (int spin = 0; spin < (1 << 22); ++spin) {
      if (__hip_atomic_load(cnt + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= splits - 1) break;
      __builtin_amdgcn_s_sleep(2);
    }
    __hip_atomic_store(cnt + tile, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  if (tr != nullptr) tr[5] = __builtin_amdgcn_s_memrealtime();
  auto load = [&](int s, int j, int i) {
    const uint32_t o = (uint32_t)s * kSlab + (uint32_t)tid * 16u;
    return __builtin_bit_cast(
        floatx4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(o + (uint32_t)((j * MT + i) * NTHREADS * 16)), 0,
                                                       kSc1));
  };
  const int nother = splits - 1;
  int s = 0;
  if constexpr (NT * MT <= 16) {
    for (; s + 1 < nother; s += 2) {
      floatx4 t0[NT][MT], t1[NT][MT];
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) {
          t0[j][i] = load(s, j, i);
          t1[j][i] = load(s + 1, j, i);
        }
#pragma unroll
      for (int j = 0; j < NT; ++j)
#pragma unroll
        for (int i = 0; i < MT; ++i) acc[j][i] += t0[j][i] + t1[j][i];
    }
  }
  for (; s < nother; ++s) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
#pragma unroll
      for (int i = 0; i < MT; ++i) acc[j][i] += load(s, j, i);
  }
  if (tr != nullptr) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tr[6] = __builtin_amdgcn_s_memrealtime();
  }
  return true;
}

}  // namespace
}  // namespace ldnn
