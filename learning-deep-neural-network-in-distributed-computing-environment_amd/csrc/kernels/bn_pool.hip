// BatchNorm (train / eval), fused BN + residual-add + ReLU, and pooling on NHWC
// bf16 activations (BAR/model.py BatchNorm2d, the
// `out += shortcut(x)` / F.relu of ResBlock.forward, AdaptiveAvgPool2d, and the
// BASELINE LeNet / ResNet-18 pools).
//
// With channels innermost, every per-channel reduction is a column sum over an
// [M = N*H*W][C] matrix: blocks own 256 channels (32 lanes x 8 channels via
// 16-B loads) x 8 row lanes, split rows over gridDim.y, reduce in LDS and add
// one fp32 atomic per channel per block.  Statistics are fp32 throughout; the
// normalise / affine / residual / ReLU pass is one vectorised elementwise sweep.
#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n) {
  int64_t g = (n + kBlock - 1) / kBlock;
  return (int)(g < 1 ? 1 : (g > 2048 ? 2048 : g));
}

// ---- per-channel partial sums: acc[0][c] += sum x, acc[1][c] += sum x^2 -----
// (backward variant: acc[0] += sum g, acc[1] += sum g * xhat, with g = dy * relu'(y))
template <bool BWD, bool RELU>
__global__ void chan_reduce_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                   const bf16_t* __restrict__ y, const float* __restrict__ mean,
                                   const float* __restrict__ invstd, float* __restrict__ acc, int M, int C,
                                   int rows_per_block) {
  __shared__ float part[2][8][32 * 8];
  const int cg = threadIdx.x & 31, ty = threadIdx.x >> 5;
  const int c0 = (blockIdx.x * 32 + cg) * 8;
  const int r_begin = blockIdx.y * rows_per_block;
  const int r_end = min(M, r_begin + rows_per_block);
  float s0[8], s1[8], mu[8], is[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    s0[j] = 0.f;
    s1[j] = 0.f;
    mu[j] = 0.f;
    is[j] = 0.f;
  }
  if (c0 < C) {
    if constexpr (BWD) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        mu[j] = mean[c0 + j];
        is[j] = invstd[c0 + j];
      }
    }
    for (int r = r_begin + ty; r < r_end; r += 8) {
      const size_t o = (size_t)r * C + c0;
      const u16x8 xv = *reinterpret_cast<const u16x8*>(x + o);
      if constexpr (BWD) {
        const u16x8 gv = *reinterpret_cast<const u16x8*>(dy + o);
        u16x8 yv;
        if constexpr (RELU) yv = *reinterpret_cast<const u16x8*>(y + o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float g = bf2f(gv[j]);
          if constexpr (RELU) g = bf2f(yv[j]) > 0.f ? g : 0.f;
          s0[j] += g;
          s1[j] += g * (bf2f(xv[j]) - mu[j]) * is[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float v = bf2f(xv[j]);
          s0[j] += v;
          s1[j] += v * v;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    part[0][ty][cg * 8 + j] = s0[j];
    part[1][ty][cg * 8 + j] = s1[j];
  }
  __syncthreads();
  if (ty < 2 && c0 < C) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float t = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) t += part[ty][q][cg * 8 + j];
      atomicAdd(acc + ty * C + c0 + j, t);
    }
  }
}

// mean / invstd / scale / shift (+ running-stat EMA, PyTorch semantics: unbiased var)
__global__ void bn_finalize_kernel(const float* __restrict__ acc, const float* __restrict__ gamma,
                                   const float* __restrict__ beta, float* __restrict__ running_mean,
                                   float* __restrict__ running_var, float* __restrict__ save_mean,
                                   float* __restrict__ save_invstd, float* __restrict__ scale,
                                   float* __restrict__ shift, int M, int C, float eps, float momentum) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float m = acc[c] / (float)M;
  const float var = fmaxf(acc[C + c] / (float)M - m * m, 0.f);
  const float is = rsqrtf(var + eps);
  save_mean[c] = m;
  save_invstd[c] = is;
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - m * g * is;
  if (running_mean) {
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * m;
    const float unb = M > 1 ? var * (float)M / (float)(M - 1) : var;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unb;
  }
}

__global__ void bn_eval_coeff_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                     const float* __restrict__ rm, const float* __restrict__ rv,
                                     float* __restrict__ scale, float* __restrict__ shift, int C, float eps) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float is = rsqrtf(rv[c] + eps);
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  scale[c] = g * is;
  shift[c] = b - rm[c] * g * is;
}

// y = relu?( x * scale[c] + shift[c] (+ res) )
template <bool RES, bool RELU>
__global__ void bn_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ res,
                                const float* __restrict__ scale, const float* __restrict__ shift,
                                bf16_t* __restrict__ y, int64_t nvec, int C) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int c0 = (int)((i * 8) % C);
    const u16x8 xv = reinterpret_cast<const u16x8*>(x)[i];
    u16x8 rv;
    if constexpr (RES) rv = reinterpret_cast<const u16x8*>(res)[i];
    const floatx4 sa = *reinterpret_cast<const floatx4*>(scale + c0);
    const floatx4 sb = *reinterpret_cast<const floatx4*>(scale + c0 + 4);
    const floatx4 ha = *reinterpret_cast<const floatx4*>(shift + c0);
    const floatx4 hb = *reinterpret_cast<const floatx4*>(shift + c0 + 4);
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float v = bf2f(xv[j]) * (j < 4 ? sa[j] : sb[j - 4]) + (j < 4 ? ha[j] : hb[j - 4]);
      if constexpr (RES) v += bf2f(rv[j]);
      if constexpr (RELU) v = fmaxf(v, 0.f);
      o[j] = f2bf(v);
    }
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
}

// dx = gamma*invstd * (g - (sum g)/M - xhat * (sum g xhat)/M);  g = dy * relu'(y)
template <bool RELU>
__global__ void bn_bwd_apply_kernel(const bf16_t* __restrict__ x, const bf16_t* __restrict__ dy,
                                    const bf16_t* __restrict__ y, const float* __restrict__ mean,
                                    const float* __restrict__ invstd, const float* __restrict__ gamma,
                                    const float* __restrict__ acc, bf16_t* __restrict__ dx, bf16_t* __restrict__ dres,
                                    int64_t nvec, int C, float invM) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < nvec; i += stride) {
    const int c0 = (int)((i * 8) % C);
    const u16x8 xv = reinterpret_cast<const u16x8*>(x)[i];
    const u16x8 gv = reinterpret_cast<const u16x8*>(dy)[i];
    u16x8 yv;
    if constexpr (RELU) yv = reinterpret_cast<const u16x8*>(y)[i];
    u16x8 o, og;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = c0 + j;
      float g = bf2f(gv[j]);
      if constexpr (RELU) g = bf2f(yv[j]) > 0.f ? g : 0.f;
      const float is = invstd[c];
      const float xh = (bf2f(xv[j]) - mean[c]) * is;
      const float gm = gamma ? gamma[c] : 1.f;
      const float v = gm * is * (g - acc[c] * invM - xh * acc[C + c] * invM);
      o[j] = f2bf(v);
      og[j] = f2bf(g);
    }
    reinterpret_cast<u16x8*>(dx)[i] = o;
    if (dres) reinterpret_cast<u16x8*>(dres)[i] = og;
  }
}

// ---- pooling (NHWC): one thread per 8 channels of one output pixel ----------
template <bool MAX>
__global__ void pool_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, uint8_t* __restrict__ arg,
                                int N, int H, int W, int C, int P, int Q, int R, int S, int st, int pad) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * P * Q * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % cv);
    int64_t t = i / cv;
    const int q = (int)(t % Q);
    t /= Q;
    const int p = (int)(t % P);
    const int n = (int)(t / P);
    float best[8];
    int bidx[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      best[j] = MAX ? -INFINITY : 0.f;
      bidx[j] = 0;
    }
    int cnt = 0;
    for (int r = 0; r < R; ++r) {
      const int h = p * st - pad + r;
      if (h < 0 || h >= H) continue;
      for (int s = 0; s < S; ++s) {
        const int w = q * st - pad + s;
        if (w < 0 || w >= W) continue;
        const u16x8 v = *reinterpret_cast<const u16x8*>(x + (((size_t)n * H + h) * W + w) * C + c8 * 8);
        ++cnt;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float f = bf2f(v[j]);
          if (MAX) {
            if (f > best[j]) { best[j] = f; bidx[j] = r * S + s; }
          } else {
            best[j] += f;
          }
        }
      }
    }
    u16x8 o;
    const float inv = MAX ? 1.f : 1.f / (float)(R * S);  // count_include_pad=True (torch default)
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(best[j] * inv);
    (void)cnt;
    reinterpret_cast<u16x8*>(y)[i] = o;
    if (MAX) {
#pragma unroll
      for (int j = 0; j < 8; ++j) arg[i * 8 + j] = (uint8_t)bidx[j];
    }
  }
}

// gather form (no atomics): each input pixel sums the outputs whose window holds it
template <bool MAX>
__global__ void pool_bwd_kernel(const bf16_t* __restrict__ dy, const uint8_t* __restrict__ arg,
                                bf16_t* __restrict__ dx, int N, int H, int W, int C, int P, int Q, int R, int S,
                                int st, int pad) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * H * W * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % cv);
    int64_t t = i / cv;
    const int w = (int)(t % W);
    t /= W;
    const int h = (int)(t % H);
    const int n = (int)(t / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // outputs p with p*st - pad <= h <= p*st - pad + R - 1
    const int p_lo = max(0, (h + pad - R + st) / st), p_hi = min(P - 1, (h + pad) / st);
    const int q_lo = max(0, (w + pad - S + st) / st), q_hi = min(Q - 1, (w + pad) / st);
    for (int p = p_lo; p <= p_hi; ++p) {
      const int r = h - (p * st - pad);
      if (r < 0 || r >= R) continue;
      for (int q = q_lo; q <= q_hi; ++q) {
        const int s = w - (q * st - pad);
        if (s < 0 || s >= S) continue;
        const size_t o = (((size_t)n * P + p) * Q + q) * cv + c8;
        const u16x8 g = reinterpret_cast<const u16x8*>(dy)[o];
        if (MAX) {
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (arg[o * 8 + j] == (uint8_t)(r * S + s)) acc[j] += bf2f(g[j]);
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += bf2f(g[j]);
        }
      }
    }
    u16x8 out;
    const float inv = MAX ? 1.f : 1.f / (float)(R * S);
#pragma unroll
    for (int j = 0; j < 8; ++j) out[j] = f2bf(acc[j] * inv);
    reinterpret_cast<u16x8*>(dx)[i] = out;
  }
}

// global average pool [N][HW][C] -> [N][C] (fp32 accumulate), and its backward
__global__ void gap_fwd_kernel(const bf16_t* __restrict__ x, bf16_t* __restrict__ y, int N, int HW, int C) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % cv), n = (int)(i / cv);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int k = 0; k < HW; ++k) {
      const u16x8 v = *reinterpret_cast<const u16x8*>(x + ((size_t)n * HW + k) * C + c8 * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[j]);
    }
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(acc[j] / (float)HW);
    reinterpret_cast<u16x8*>(y)[i] = o;
  }
}

__global__ void gap_bwd_kernel(const bf16_t* __restrict__ dy, bf16_t* __restrict__ dx, int N, int HW, int C) {
  const int cv = C / 8;
  const int64_t total = (int64_t)N * HW * cv;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += stride) {
    const int c8 = (int)(i % cv);
    const int n = (int)(i / cv / HW);
    const u16x8 g = reinterpret_cast<const u16x8*>(dy)[(size_t)n * cv + c8];
    u16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = f2bf(bf2f(g[j]) / (float)HW);
    reinterpret_cast<u16x8*>(dx)[i] = o;
  }
}

void reduce_grid(int M, int C, dim3& grid, int& rpb) {
  const int gx = (C + 255) / 256;
  int gy = (M + 511) / 512;
  const int cap = max(1, 2048 / gx);
  if (gy > cap) gy = cap;
  rpb = (M + gy - 1) / gy;
  grid = dim3(gx, gy);
}

}  // namespace

hipError_t bn_forward(const BnArgs& a, hipStream_t s) {
  const int M = a.M, C = a.C;
  if (C % 8) return hipErrorInvalidValue;
  const int64_t nvec = (int64_t)M * C / 8;
  if (a.training) {
    hipError_t e = zero2d_f32(a.ws, 1, 2 * C, 2 * C, s);
    if (e != hipSuccess) return e;
    dim3 grid;
    int rpb;
    reduce_grid(M, C, grid, rpb);
    chan_reduce_kernel<false, false><<<grid, kBlock, 0, s>>>(a.x, nullptr, nullptr, nullptr, nullptr, a.ws, M, C, rpb);
    bn_finalize_kernel<<<(C + 255) / 256, 256, 0, s>>>(a.ws, a.gamma, a.beta, a.running_mean, a.running_var,
                                                       a.save_mean, a.save_invstd, a.scale, a.shift, M, C, a.eps,
                                                       a.momentum);
  } else {
    bn_eval_coeff_kernel<<<(C + 255) / 256, 256, 0, s>>>(a.gamma, a.beta, a.running_mean, a.running_var, a.scale,
                                                         a.shift, C, a.eps);
  }
  const int g = grid_for(nvec);
  if (a.residual) {
    if (a.relu) bn_apply_kernel<true, true><<<g, kBlock, 0, s>>>(a.x, a.residual, a.scale, a.shift, a.y, nvec, C);
    else bn_apply_kernel<true, false><<<g, kBlock, 0, s>>>(a.x, a.residual, a.scale, a.shift, a.y, nvec, C);
  } else {
    if (a.relu) bn_apply_kernel<false, true><<<g, kBlock, 0, s>>>(a.x, nullptr, a.scale, a.shift, a.y, nvec, C);
    else bn_apply_kernel<false, false><<<g, kBlock, 0, s>>>(a.x, nullptr, a.scale, a.shift, a.y, nvec, C);
  }
  return hipGetLastError();
}

hipError_t bn_backward(const BnArgs& a, const uint16_t* dy, uint16_t* dx, uint16_t* dres, float* dgamma,
                       float* dbeta, hipStream_t s) {
  const int M = a.M, C = a.C;
  if (C % 8) return hipErrorInvalidValue;
  hipError_t e = zero2d_f32(a.ws, 1, 2 * C, 2 * C, s);
  if (e != hipSuccess) return e;
  dim3 grid;
  int rpb;
  reduce_grid(M, C, grid, rpb);
  if (a.relu)
    chan_reduce_kernel<true, true><<<grid, kBlock, 0, s>>>(a.x, dy, a.y, a.save_mean, a.save_invstd, a.ws, M, C, rpb);
  else
    chan_reduce_kernel<true, false><<<grid, kBlock, 0, s>>>(a.x, dy, nullptr, a.save_mean, a.save_invstd, a.ws, M, C,
                                                           rpb);
  const int64_t nvec = (int64_t)M * C / 8;
  const int g = grid_for(nvec);
  if (a.relu)
    bn_bwd_apply_kernel<true><<<g, kBlock, 0, s>>>(a.x, dy, a.y, a.save_mean, a.save_invstd, a.gamma, a.ws, dx, dres,
                                                   nvec, C, 1.f / (float)M);
  else
    bn_bwd_apply_kernel<false><<<g, kBlock, 0, s>>>(a.x, dy, nullptr, a.save_mean, a.save_invstd, a.gamma, a.ws, dx,
                                                    dres, nvec, C, 1.f / (float)M);
  // dgamma += sum g*xhat ; dbeta += sum g  (accumulate into the flat gradient buffer)
  if (dgamma || dbeta) {
    if (dgamma) e = mix3_f32(dgamma, dgamma, a.ws + C, nullptr, 1.f, 1.f, 0.f, C, nullptr, s);
    if (e != hipSuccess) return e;
    if (dbeta) e = mix3_f32(dbeta, dbeta, a.ws, nullptr, 1.f, 1.f, 0.f, C, nullptr, s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

hipError_t pool2d_fwd(const uint16_t* x, uint16_t* y, uint8_t* argmax, int N, int H, int W, int C, int P, int Q,
                      int R, int S, int stride, int pad, bool is_max, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const int g = grid_for((int64_t)N * P * Q * C / 8);
  if (is_max) pool_fwd_kernel<true><<<g, kBlock, 0, s>>>(x, y, argmax, N, H, W, C, P, Q, R, S, stride, pad);
  else pool_fwd_kernel<false><<<g, kBlock, 0, s>>>(x, y, argmax, N, H, W, C, P, Q, R, S, stride, pad);
  return hipGetLastError();
}

hipError_t pool2d_bwd(const uint16_t* dy, const uint8_t* argmax, uint16_t* dx, int N, int H, int W, int C, int P,
                      int Q, int R, int S, int stride, int pad, bool is_max, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  const int g = grid_for((int64_t)N * H * W * C / 8);
  if (is_max) pool_bwd_kernel<true><<<g, kBlock, 0, s>>>(dy, argmax, dx, N, H, W, C, P, Q, R, S, stride, pad);
  else pool_bwd_kernel<false><<<g, kBlock, 0, s>>>(dy, argmax, dx, N, H, W, C, P, Q, R, S, stride, pad);
  return hipGetLastError();
}

hipError_t global_avgpool_fwd(const uint16_t* x, uint16_t* y, int N, int HW, int C, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  gap_fwd_kernel<<<grid_for((int64_t)N * C / 8), kBlock, 0, s>>>(x, y, N, HW, C);
  return hipGetLastError();
}

hipError_t global_avgpool_bwd(const uint16_t* dy, uint16_t* dx, int N, int HW, int C, hipStream_t s) {
  if (C % 8) return hipErrorInvalidValue;
  gap_bwd_kernel<<<grid_for((int64_t)N * HW * C / 8), kBlock, 0, s>>>(dy, dx, N, HW, C);
  return hipGetLastError();
}

}  // namespace ldnn
