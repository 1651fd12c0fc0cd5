// BatchNorm statistics finalize, shared by the BN reduce kernel (bn_pool.hip) and
// the conv forward epilogue that accumulates the following BN's statistics
// (conv_lds.hip): the last of `nblk` contributing workgroups turns the fp32
// totals into mean / invstd, running-stat EMA and the apply coefficients.
#pragma once

#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {

constexpr int kBnCopies = 8;  // accumulator copies of the BN statistics (conv epilogue and BN reduce)
constexpr int kGrpMax = 128;  // row groups of the grouped statistics passes (BnFin::part rows), at most

// Totals of every block are complete in `acc` when the last block draws its
// ticket: the fp32 atomics execute at the memory side and every block waits
// for its own (vmcnt) before adding to the ticket; the finalizer reads AND
// clears the totals with atomic exchanges (memory-side too, so no cache can
// hand it a stale line).  (Measured: making the contributions returning atomics
// costs ~0.2 ms per ResNet-18 b64 step and changes no result beyond arrival-order
// noise, profiles/cnn_bn_reduce_r2.jsonl.)
// NCOP: the totals are spread over NCOP [2C] accumulator copies (contributors
// pick copy `block % NCOP`, NCOP x less same-address serialisation at the
// memory-side atomic units); ncop = 1 at run time when few blocks contribute (the
// finalizer's exchanges are its latency: 8 copies of a 1024-channel BN cost a
// single finalizing block ~10 us).  The finalizer sums the copies into the caller's LDS
// scratch (`cap` floats, free once the caller's own reduction has been read)
// with all NCOP exchanges of an element in flight together, then finalizes per
// channel; with 2C > cap it sums the copies in the per-channel loop.  (The
// scratch is the caller's: a static LDS array here would cost the conv kernels
// that inline this occupancy.)
__device__ __forceinline__ void bn_acc_add(float* p, float v) { atomicAdd(p, v); }

// Channel c's totals (forward: sum x, sum x^2; backward: sum g, sum g * xhat) -> saved
// statistics, running-stat EMA and apply coefficients (forward), or the backward
// coefficients and dgamma / dbeta.
template <bool BWD>
__device__ __forceinline__ void bn_finalize_channel(const BnFin& f, int M, int C, int c, float S0, float S1,
                                                    float invM) {
  const float gm = f.gamma ? f.gamma[c] : 1.f;
  if constexpr (!BWD) {
    const float m = S0 * invM;
    const float var = fmaxf(S1 * invM - m * m, 0.f);
    const float is = rsqrtf(var + f.eps);
    f.save_mean[c] = m;
    f.save_invstd[c] = is;
    const float b = f.beta ? f.beta[c] : 0.f;
    f.coef[c] = gm * is;
    f.coef[C + c] = b - m * gm * is;
    if (f.running_mean) {
      f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * m;
      const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
      f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * unb;
    }
  } else {
    const float is = f.save_invstd[c];
    const float A = gm * is, B = -gm * is * is * S1 * invM;
    f.coef[c] = A;
    f.coef[C + c] = B;
    f.coef[2 * C + c] = -gm * is * S0 * invM - B * f.save_mean[c];
    if (f.dgamma) f.dgamma[c] = f.grad_assign ? S1 : f.dgamma[c] + S1;
    if (f.dbeta) f.dbeta[c] = f.grad_assign ? S0 : f.dbeta[c] + S0;
  }
}

template <bool BWD, int NCOP>
__device__ __forceinline__ void bn_finalize_last(const BnFin& f, int M, int C, int nblk, float* tot, int cap,
                                                 int ncop = NCOP) {
  // the "last block" flag lives in the caller's scratch (its last float): a second
  // __shared__ object would add 4 bytes to the kernels that inline this (the trap of
  // cdna_hip_programming.md, and an 80-KiB kernel would lose its second workgroup)
  int& last = *reinterpret_cast<int*>(tot + cap - 1);
  cap -= 1;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(f.ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = t == nblk - 1;
    if (last) __hip_atomic_store(f.ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (!last) return;
  const bool lds = 2 * C <= cap;
  if (lds) {
    const int n2 = 2 * C, nt = blockDim.x;
    if (ncop == 1) {  // one copy: 8 elements per thread in flight together (large C, few blocks)
      for (int i0 = threadIdx.x; i0 < n2; i0 += 8 * nt) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = i0 + u * nt < n2 ? atomicExch(f.acc + i0 + u * nt, 0.f) : 0.f;
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (i0 + u * nt < n2) tot[i0 + u * nt] = v[u];
      }
    } else {  // NCOP copies: two elements x NCOP exchanges in flight
      for (int i0 = threadIdx.x; i0 < n2; i0 += 2 * nt) {
        float v[2][NCOP];
#pragma unroll
        for (int u = 0; u < 2; ++u)
#pragma unroll
          for (int k = 0; k < NCOP; ++k)
            v[u][k] = i0 + u * nt < n2 ? atomicExch(f.acc + (size_t)k * n2 + i0 + u * nt, 0.f) : 0.f;
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          float t = 0.f;
#pragma unroll
          for (int k = 0; k < NCOP; ++k) t += v[u][k];
          if (i0 + u * nt < n2) tot[i0 + u * nt] = t;
        }
      }
    }
    __syncthreads();
  }
  const float invM = 1.f / (float)M;
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float S0 = 0.f, S1 = 0.f;
    if (lds) {
      S0 = tot[c];
      S1 = tot[C + c];
    } else {
#pragma unroll
      for (int k = 0; k < NCOP; ++k) {
        if (k >= ncop) break;
        S0 += atomicExch(f.acc + (size_t)k * 2 * C + c, 0.f);
        S1 += atomicExch(f.acc + (size_t)k * 2 * C + C + c, 0.f);
      }
    }
    bn_finalize_channel<BWD>(f, M, C, c, S0, S1, invM);
  }
  if (!BWD && threadIdx.x == 0 && f.num_batches) f.num_batches[0] += 1;
}

// ---- grouped statistics (bn_reduce_small_kernel in bn_pool.hip, the conv slab epilogue in
// conv_lds.hip): a grid of (64-channel columns) x (row groups); every workgroup publishes its
// columns' partial sums to BnFin::part ([row group][2][C]) and the LAST workgroup of a column
// (per-column ticket) sums them and finalizes those 64 channels -- a short chain per column,
// all columns in parallel.
__device__ __forceinline__ void grp_store(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float grp_load(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// After wave 0 stored this workgroup's partials: true in every thread of the workgroup that
// draws the column's last ticket (it resets the ticket).  As in bn_finalize_last, no fences: the
// partials are agent-scope atomic stores (coherent at the memory side), wave 0 waits for their
// completion before its ticket, and the finalizer reads them with agent-scope atomic loads.
__device__ __forceinline__ bool grp_ticket(int* ticket, int n, int& flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(ticket, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = t == n - 1;
    if (flag) __hip_atomic_store(ticket, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return flag;
}
// the finalizer's column totals: thread (q = tid / 64, channel tid % 64) sums every 4th row
// group's partial k into tot[k][q][64]; the caller reads tot after a barrier
__device__ __forceinline__ void grp_sum(const float* part, int C, int c, int k, int ny, float* tot) {
  const int q = threadIdx.x >> 6;
  float v = 0.f;
  if (c < C)
    for (int y0 = q; y0 < ny; y0 += 32) {   // 8 loads in flight (atomic loads are not batched for us)
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = y0 + 4 * u < ny ? grp_load(part + ((size_t)(y0 + 4 * u) * 2 + k) * C + c) : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) v += t[u];
    }
  tot[(k * 4 + q) * 64 + (threadIdx.x & 63)] = v;
}

}  // namespace ldnn
