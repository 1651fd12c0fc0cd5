// One-shot intra-node all-reduce over IPC-mapped peer buffers (SURVEY §5
// "distributed comm backend": the small-message path that reads from all peers).
//
// An MI355X node is a full xGMI mesh: every GPU has a direct link to each of the
// other 7.  A ring collective moves a small message through N-1 dependent hops,
// one link at a time; for messages of a few MB or less that latency, not the
// link bandwidth, is the cost.  Here every rank maps the other ranks' staging
// buffers (hipIpcGetMemHandle / hipIpcOpenMemHandle) and ONE kernel per rank
// stages its own copy, meets the peers at one barrier and reads all N copies at
// once -- each peer's bytes over its own link, concurrently -- summing in fp32.
//
//  * each rank owns a staging region (2 x max_bytes: calls alternate halves by
//    epoch parity), a signal region of uncached device memory,
//    sig[block][rank] = epoch of the last call that block reached, and one epoch
//    counter per block in its own memory;
//  * block b reads its counter (epoch = ctr[b] + 1: the kernel takes no host-side
//    call number, so a launch captured into a hipGraph and replayed N times runs
//    N distinct, correctly ordered calls), copies ITS slice of the tensor into
//    staging half (epoch & 1), releases it at system scope (L2 write-back, peers
//    read it over xGMI), stores `epoch` into sig[b][rank] of every peer, spins
//    until its own sig[b][j] >= epoch for every j, then sums slice b of every
//    rank's staging half into the tensor and stores ctr[b] = epoch;
//  * reuse safety: a rank writes staging half p again two calls later, after its
//    next call's barrier -- which every peer only reaches once its previous
//    kernel (the last reader of half p) has finished.
// Every spin has a wall-clock limit: a rank that never arrives sets the sticky
// error word and the kernel returns leaving the tensor UNSUMMED; every later call
// sees the word and does the same.  The host reads it (OneShotAllReduce.check,
// called from Comm.check_schedule every global epoch / every few hundred DP steps)
// and raises, so training never goes on silently with unsynchronised gradients.
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

// n8: number of 8-element groups; each thread handles whole groups (fp32: two 16-B
// loads per rank, bf16: one).  `buf` is the tensor, read (staged) and overwritten.
template <bool BF16>
__global__ __launch_bounds__(kIpcThreads) void oneshot_ar_kernel(IpcPeers p, int rank, int world, int64_t n8,
                                                                 void* buf) {
  const int b = blockIdx.x;
  __shared__ uint32_t s_epoch;
  __shared__ int s_err;
  if (threadIdx.x == 0) {
    s_epoch = p.ctr[b] + 1u;
    s_err = __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  __syncthreads();
  const uint32_t epoch = s_epoch;
  if (s_err != 0) return;
  constexpr size_t esz = BF16 ? 2 : 4;
  const size_t base = (size_t)(epoch & 1u) * p.half_bytes;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  // ---- stage this block's slice of the local tensor
  for (int64_t g = (int64_t)b * blockDim.x + threadIdx.x; g < n8; g += stride) {
    const uint4* src = reinterpret_cast<const uint4*>(static_cast<const char*>(buf) + (size_t)g * 8 * esz);
    uint4* dst = reinterpret_cast<uint4*>(p.mine + base + (size_t)g * 8 * esz);
    dst[0] = src[0];
    if constexpr (!BF16) dst[1] = src[1];
  }
  __threadfence_system();   // the staged slice is visible to the peers (system-scope release)
  __syncthreads();
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
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  if (__hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0) return;
  // ---- sum every rank's copy of this block's slice
  for (int64_t g = (int64_t)b * blockDim.x + threadIdx.x; g < n8; g += stride) {
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
      reinterpret_cast<u16x8*>(buf)[g] = o;
    } else {
      floatx4* o = reinterpret_cast<floatx4*>(buf) + 2 * g;
      o[0] = floatx4{s[0], s[1], s[2], s[3]};
      o[1] = floatx4{s[4], s[5], s[6], s[7]};
    }
  }
  if (threadIdx.x == 0) p.ctr[b] = epoch;   // (a vector store: thread 0 only)
}

}  // namespace

hipError_t oneshot_all_reduce(const IpcPeers& p, int rank, int world, int64_t n, bool bf16, void* buf, int blocks,
                              hipStream_t s) {
  if (world < 1 || world > kIpcMaxRanks || rank < 0 || rank >= world || n % 8 != 0) return hipErrorInvalidValue;
  if (blocks < 1 || blocks > kIpcMaxBlocks) return hipErrorInvalidValue;
  if ((size_t)n * (bf16 ? 2 : 4) > p.half_bytes) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  if (bf16) oneshot_ar_kernel<true><<<blocks, kIpcThreads, 0, s>>>(p, rank, world, n8, buf);
  else oneshot_ar_kernel<false><<<blocks, kIpcThreads, 0, s>>>(p, rank, world, n8, buf);
  return hipGetLastError();
}

}  // namespace ldnn
