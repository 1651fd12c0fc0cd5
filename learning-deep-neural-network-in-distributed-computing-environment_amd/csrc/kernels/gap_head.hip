// Pooled classifier head of the CNNs: global average pool + Linear (<= 16 classes), forward
// and backward in one launch each (EnhancedCNN: AdaptiveAvgPool2d(1) -> Linear(1024, 10),
// BAR/model.py:99-100,108-110; SURVEY §2 K12 + K13).
//
// At batch 64 the head is 64 x 4 x 1024 activations and a 10 x 1024 weight: pure latency.  The
// separate path runs gap_fwd + the skinny GEMM forward and colsum + two small GEMMs + gap_bwd
// backward -- six dependent launches of ~5 us.  Here:
//  * forward: one workgroup per sample pools its H*W x C activations into LDS (the bf16-rounded
//    means are also stored: the weight gradient's operand) and takes the <= 16 dot products
//    from LDS -- no cross-workgroup dependency at all;
//  * backward: one workgroup per 64-channel column computes that column's dW (sum over the
//    batch of dlogits x pooled), its share of the input gradient (dlogits . W / HW broadcast to
//    the H*W positions, 16-B stores) and, in column 0, the bias gradient.
#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

constexpr int kHeadMaxC = 4096;   // pooled features held in LDS (fp32) per forward workgroup
constexpr int kHeadMaxN = 65536;  // batch rows (the backward stages 256 at a time)

// x [N][HW][C] bf16, W [ncls_pad][ldw] bf16 (rows >= ncls zero), b [ncls_pad] fp32
// -> pooled [N][C] bf16, logits [N][ldl] bf16 (columns < ncls_pad written)
__global__ __launch_bounds__(256) void gap_linear_fwd_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ W,
                                                             const float* __restrict__ b, bf16_t* __restrict__ pooled,
                                                             bf16_t* __restrict__ logits, int HW, int C, int ldw,
                                                             int ncls, int ldl) {
  __shared__ float pl[kHeadMaxC];
  const int n = blockIdx.x, tid = threadIdx.x;
  const float inv = 1.f / (float)HW;
  const bf16_t* xs = x + (size_t)n * HW * C;
  for (int c8 = tid; c8 < C / 8; c8 += 256) {
    float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int p = 0; p < HW; ++p) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(xs + (size_t)p * C + c8 * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) s[j] += bf2f(v[j]);
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = f2bf(s[j] * inv);
      pl[c8 * 8 + j] = bf2f(o[j]);   // the Linear reads the stored bf16 value, as the unfused path
    }
    *reinterpret_cast<u16x8*>(pooled + (size_t)n * C + c8 * 8) = o;
  }
  __syncthreads();
  // class k = tid / 16 (16 classes), 16 lanes per class walk 8-channel chunks
  const int k = tid >> 4, q = tid & 15;
  float acc = 0.f;
  if (k < ncls) {
    const bf16_t* wr = W + (size_t)k * ldw;
    for (int c0 = q * 8; c0 < C; c0 += 128) {
      const u16x8 w = *reinterpret_cast<const u16x8*>(wr + c0);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += bf2f(w[j]) * pl[c0 + j];
    }
  }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) acc += __shfl_xor(acc, o, 64);
  if (q == 0 && k < ldl) logits[(size_t)n * ldl + k] = k < ncls ? f2bf(acc + (b ? b[k] : 0.f)) : (bf16_t)0;
}

// g [N][ldg] bf16 (dlogits, columns >= ncls zero), pooled [N][C] bf16, W [ncls][ldw] bf16
// -> dW [ncls][lddw] fp32 (= beta_w * dW + sum), db [ncls] fp32 (beta_b), dx [N][HW][C] bf16
// Every operand is staged into LDS first with all of a thread's loads in flight together (one
// round trip each), then the products run out of LDS: the batch is kHeadRows rows at a time.
constexpr int kHeadRows = 256;
__global__ __launch_bounds__(256) void gap_linear_bwd_kernel(const bf16_t* __restrict__ g, const bf16_t* __restrict__ pooled,
                                                             const bf16_t* __restrict__ W, float* __restrict__ dW,
                                                             float* __restrict__ db, bf16_t* __restrict__ dx, int N,
                                                             int HW, int C, int ldg, int ldw, int lddw, int ncls,
                                                             float beta_w, float beta_b) {
  __shared__ float gl[kHeadRows * 17];        // dlogits rows (pitch 17: conflict-free column reads)
  __shared__ float wl[16][64];                // this column's weights
  __shared__ __attribute__((aligned(16))) bf16_t pl[kHeadRows * 64];   // this column's pooled rows
  const int tid = threadIdx.x, c0 = blockIdx.x * 64;
  {
    float wv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = tid + u * 256, k = i >> 6, c = c0 + (i & 63);
      wv[u] = (k < ncls && c < C) ? bf2f(W[(size_t)k * ldw + c]) : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) wl[(tid + u * 256) >> 6][(tid + u * 256) & 63] = wv[u];
  }
  const int cw = c0 + (tid & 63), k0 = 4 * (tid >> 6);   // dW: channel cw, classes k0 .. k0 + 3
  float a[4] = {0.f, 0.f, 0.f, 0.f}, dbs = 0.f;
  const int lane = tid & 7, cc = c0 + lane * 8;          // dx: channels cc .. cc + 7, rows tid / 8 + 32 i
  const float inv = 1.f / (float)HW;
  for (int r0 = 0; r0 < N; r0 += kHeadRows) {
    const int nr = min(kHeadRows, N - r0);
    __syncthreads();   // the previous chunk's LDS reads are done
    {
      float gv[16];
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = tid + u * 256, n = i >> 4, k = i & 15;
        gv[u] = (n < nr && k < ncls) ? bf2f(g[(size_t)(r0 + n) * ldg + k]) : 0.f;
      }
      u16x8 pv[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int n = (tid >> 3) + 32 * u;
        pv[u] = u16x8{0, 0, 0, 0, 0, 0, 0, 0};
        if (n < nr && cc < C) pv[u] = *reinterpret_cast<const u16x8*>(pooled + (size_t)(r0 + n) * C + cc);
      }
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = tid + u * 256;
        gl[(i >> 4) * 17 + (i & 15)] = gv[u];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) *reinterpret_cast<u16x8*>(pl + ((tid >> 3) + 32 * u) * 64 + lane * 8) = pv[u];
    }
    __syncthreads();
    if (cw < C && k0 < ncls)
      for (int n = 0; n < nr; ++n) {
        const float p = bf2f(pl[n * 64 + (tid & 63)]);
#pragma unroll
        for (int u = 0; u < 4; ++u) a[u] += gl[n * 17 + k0 + u] * p;
      }
    if (blockIdx.x == 0 && tid < ncls)
      for (int n = 0; n < nr; ++n) dbs += gl[n * 17 + tid];
    if (cc < C)
      for (int n = tid >> 3; n < nr; n += 32) {
        float d[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < ncls; ++k) {
          const float gk = gl[n * 17 + k];
#pragma unroll
          for (int j = 0; j < 8; ++j) d[j] += gk * wl[k][lane * 8 + j];
        }
        u16x8 o;
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = f2bf(d[j] * inv);
        bf16_t* dst = dx + (size_t)(r0 + n) * HW * C + cc;
        for (int p = 0; p < HW; ++p) *reinterpret_cast<u16x8*>(dst + (size_t)p * C) = o;
      }
  }
  if (cw < C && k0 < ncls) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k0 + u >= ncls) break;
      float* d = dW + (size_t)(k0 + u) * lddw + cw;
      *d = beta_w != 0.f ? beta_w * *d + a[u] : a[u];
    }
  }
  if (blockIdx.x == 0 && tid < ncls && db != nullptr) db[tid] = beta_b != 0.f ? beta_b * db[tid] + dbs : dbs;
}

}  // namespace

bool gap_linear_ok(int N, int HW, int C, int ncls) {
  return N > 0 && HW > 0 && C % 8 == 0 && C <= kHeadMaxC && ncls >= 1 && ncls <= 16 && N <= kHeadMaxN;
}

hipError_t gap_linear_fwd(const uint16_t* x, const uint16_t* W, const float* b, uint16_t* pooled, uint16_t* logits,
                          int N, int HW, int C, int ldw, int ncls, int ldl, hipStream_t s) {
  if (!gap_linear_ok(N, HW, C, ncls) || ldw % 8 != 0 || ldl < ncls) return hipErrorInvalidValue;
  gap_linear_fwd_kernel<<<N, 256, 0, s>>>(x, W, b, pooled, logits, HW, C, ldw, ncls, ldl);
  return hipGetLastError();
}

hipError_t gap_linear_bwd(const uint16_t* g, const uint16_t* pooled, const uint16_t* W, float* dW, float* db,
                          uint16_t* dx, int N, int HW, int C, int ldg, int ldw, int lddw, int ncls, float beta_w,
                          float beta_b, hipStream_t s) {
  if (!gap_linear_ok(N, HW, C, ncls) || ldg < ncls) return hipErrorInvalidValue;
  gap_linear_bwd_kernel<<<(C + 63) / 64, 256, 0, s>>>(g, pooled, W, dW, db, dx, N, HW, C, ldg, ldw, lddw, ncls,
                                                      beta_w, beta_b);
  return hipGetLastError();
}

}  // namespace ldnn
