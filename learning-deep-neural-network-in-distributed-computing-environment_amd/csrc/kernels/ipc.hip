// One-shot intra-node all-reduce over IPC-mapped peer buffers (SURVEY §5
// "distributed comm backend": the small-message path that reads from all peers).
//
// An MI355X node is a full xGMI mesh: every GPU has a direct link to each of the
// other 7.  A ring collective moves a small message through N-1 dependent hops,
// one link at a time; for messages of a few MB or less that latency, not the
// link bandwidth, is the cost.  Here every rank maps the other ranks' staging
// buffers (hipIpcGetMemHandle / hipIpcOpenMemHandle) and ONE kernel per rank
// reads all N copies at once -- each peer's bytes over its own link, concurrently
// -- and sums them in fp32.  One barrier per call:
//
//  * each rank owns a staging region (2 x max_bytes: calls alternate halves by
//    epoch parity) and a signal region of uncached device memory,
//    sig[block][rank] = epoch of the last call that block reached;
//  * block b of rank r stores `epoch` into sig[b][r] of every peer (release,
//    system scope), then spins until its own sig[b][j] >= epoch for every j
//    (acquire, system scope), then reads slice b of every rank's staging half;
//  * reuse safety: a rank writes staging half p again two calls later, after its
//    next call's barrier -- which every peer only reaches once its previous
//    kernel (the last reader of half p) has finished.
// Every spin has a wall-clock limit: a rank that never arrives sets the error
// word and the kernel exits instead of hanging the GPU.
#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {
namespace {

constexpr int kIpcThreads = 512;
constexpr uint64_t kSpinLimit = 500000000ull;  // 5 s of the 100 MHz wall clock

__device__ __forceinline__ void to_f32(float (&v)[8], const uint4& raw, bool bf16_in, int half) {
  if (bf16_in) {
    const uint32_t w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = __uint_as_float(w[i] << 16);
      v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  } else {
    v[half * 4 + 0] = __uint_as_float(raw.x);
    v[half * 4 + 1] = __uint_as_float(raw.y);
    v[half * 4 + 2] = __uint_as_float(raw.z);
    v[half * 4 + 3] = __uint_as_float(raw.w);
  }
}

// n8: number of 8-element groups; each thread sums whole groups (fp32: two 16-B
// loads per rank, bf16: one).  out may alias this rank's input tensor (not the
// staging buffers).
template <bool BF16>
__global__ __launch_bounds__(kIpcThreads) void oneshot_ar_kernel(IpcPeers p, int rank, int world, uint32_t epoch,
                                                                 int half, int64_t n8, void* out) {
  const int b = blockIdx.x;
  // ---- barrier: announce this block to every rank, wait for theirs
  if (threadIdx.x < (unsigned)world) {
    const int j = threadIdx.x;
    __hip_atomic_store(p.sig[j] + b * kIpcMaxRanks + rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* mine = p.sig[rank] + b * kIpcMaxRanks + j;
    const uint64_t t0 = wall_clock64();
    while (__hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < epoch) {
      if (wall_clock64() - t0 > kSpinLimit) {
        __hip_atomic_store(p.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  // ---- sum every rank's copy of this block's slice
  const size_t esz = BF16 ? 2 : 4;
  const size_t base = (size_t)half * p.half_bytes;
  for (int64_t g = (int64_t)b * blockDim.x + threadIdx.x; g < n8; g += (int64_t)gridDim.x * blockDim.x) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < world; ++j) {
      const char* src = p.data[j] + base + (size_t)g * 8 * esz;
      float v[8];
      if constexpr (BF16) {
        to_f32(v, *reinterpret_cast<const uint4*>(src), true, 0);
      } else {
        to_f32(v, *reinterpret_cast<const uint4*>(src), false, 0);
        to_f32(v, *reinterpret_cast<const uint4*>(src + 16), false, 1);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) s[q] += v[q];
    }
    if constexpr (BF16) {
      u16x8 o;
#pragma unroll
      for (int q = 0; q < 8; ++q) o[q] = f2bf(s[q]);
      reinterpret_cast<u16x8*>(out)[g] = o;
    } else {
      floatx4* o = reinterpret_cast<floatx4*>(out) + 2 * g;
      o[0] = floatx4{s[0], s[1], s[2], s[3]};
      o[1] = floatx4{s[4], s[5], s[6], s[7]};
    }
  }
}

}  // namespace

hipError_t oneshot_all_reduce(const IpcPeers& p, int rank, int world, uint32_t epoch, int half, int64_t n, bool bf16,
                              void* out, int blocks, hipStream_t s) {
  if (world < 1 || world > kIpcMaxRanks || rank < 0 || rank >= world || n % 8 != 0) return hipErrorInvalidValue;
  if (blocks < 1 || blocks > kIpcMaxBlocks) return hipErrorInvalidValue;
  if ((size_t)n * (bf16 ? 2 : 4) > p.half_bytes) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  if (bf16) oneshot_ar_kernel<true><<<blocks, kIpcThreads, 0, s>>>(p, rank, world, epoch, half, n8, out);
  else oneshot_ar_kernel<false><<<blocks, kIpcThreads, 0, s>>>(p, rank, world, epoch, half, n8, out);
  return hipGetLastError();
}

}  // namespace ldnn
