// Input pipeline kernel: gather + AutoAugment(CIFAR10) / flip + crop +
// normalise + cast, one workgroup per image, the image resident in LDS.
//
// The reference runs torchvision's AutoAugment per image in PIL on the host,
// inside a num_workers=0 DataLoader (BAR/dataloader.py:14-21): the GPU waits on
// the CPU every step.  Here the uint8 dataset already sits in HBM;
// a batch is one launch of B workgroups.  Each workgroup
//   1. copies its image row (C*H*W bytes, 3 KiB for CIFAR) into LDS,
//   2. draws its sub-policy / probabilities / signs / flip / crop offsets from a
//      counter hash of (batch seed, sample) -- reproducible and independent of
//      the launch geometry,
//   3. applies the sub-policy's two ops LDS -> LDS (ping-pong buffers); the
//      whole-image reductions (Contrast mean, AutoContrast min/max, Equalize
//      histograms + LUT scan) are LDS atomics + one wave per channel,
//   4. flips / crops, normalises x * a[c] + b[c] and writes bf16 or fp32.
// Arithmetic mirrors data/autoaugment.py (float32, no contraction) bit for bit;
// that module documents the torchvision semantics each op follows.
#include "ldnn_common.h"
#include "ldnn_kernels.h"

namespace ldnn {
namespace {

constexpr int kT = 256;
enum {
  kShearX, kShearY, kTranslateX, kTranslateY, kRotate, kBrightness, kColor, kContrast, kSharpness, kPosterize,
  kSolarize, kAutoContrast, kEqualize, kInvert, kIdentity
};

__device__ __forceinline__ uint64_t smix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ uint8_t trunc_u8(float v) {
#pragma clang fp contract(off)
  return (uint8_t)(int)fminf(fmaxf(v, 0.f), 255.f);
}

// torchvision _blend: (r * x + (1 - r) * o).clamp(0, 255).to(uint8), r = 1 + magnitude in double
struct Blend {
  float c1, c2;
  __device__ explicit Blend(float mag) {
    const double r = 1.0 + (double)mag;
    c1 = (float)r;
    c2 = (float)(1.0 - r);
  }
  __device__ __forceinline__ uint8_t operator()(float x, float o) const {
#pragma clang fp contract(off)
    return trunc_u8(c1 * x + c2 * o);
  }
};

__device__ __forceinline__ uint8_t gray_u8(const uint8_t* in, int q, int C, int HW) {
#pragma clang fp contract(off)
  if (C == 1) return in[q];
  const float v = 0.2989f * (float)in[q] + 0.587f * (float)in[HW + q] + 0.114f * (float)in[2 * HW + q];
  return (uint8_t)(int)v;
}

// scratch ints: [0, 3*256) histograms / LUTs, then 16 reduction slots
constexpr int kRed = 3 * 256;

// One op, `in` -> `out` (both LDS), ends with a barrier.  `op` and `mag` are uniform.
__device__ void apply_op(const AugParams& p, int op, int bin, float mag, const uint8_t* in, uint8_t* out, int* scr) {
#pragma clang fp contract(off)
  const int tid = threadIdx.x;
  const int C = p.C, H = p.H, W = p.W, HW = H * W, CHW = C * HW;
  switch (op) {
    case kShearX: case kShearY: case kTranslateX: case kTranslateY: case kRotate: {
      // inverse affine map in centred pixel coordinates (torchvision _get_inverse_affine_matrix,
      // grid_sample nearest / zeros / align_corners=False)
      float m0 = 1.f, m1 = 0.f, m2 = 0.f, m3 = 0.f, m4 = 1.f, m5 = 0.f;
      if (op == kShearX) { m1 = mag; m2 = mag * (float)(H * 0.5); }
      else if (op == kShearY) { m3 = mag; m5 = mag * (float)(W * 0.5); }
      else if (op == kTranslateX) { m2 = -(float)(int)mag; }
      else if (op == kTranslateY) { m5 = -(float)(int)mag; }
      else {
        const float c = p.rot_cos[bin], s = mag < 0.f ? -p.rot_sin[bin] : p.rot_sin[bin];
        m0 = c; m1 = s; m3 = -s; m4 = c;
      }
      const float hw = (float)W * 0.5f, hh = (float)H * 0.5f;
      const float ox = (float)(W * 0.5 - 0.5), oy = (float)(H * 0.5 - 0.5);
      for (int q = tid; q < HW; q += kT) {
        const int j = q / W, i = q - j * W;
        const float X = ((float)i - hw) + 0.5f, Y = ((float)j - hh) + 0.5f;
        const float xs = (m0 * X + m1 * Y) + m2, ys = (m3 * X + m4 * Y) + m5;
        const int sx = (int)rintf(xs + ox), sy = (int)rintf(ys + oy);
        const bool ok = sx >= 0 && sx < W && sy >= 0 && sy < H;
        for (int c = 0; c < C; ++c) out[c * HW + q] = ok ? in[c * HW + sy * W + sx] : (uint8_t)0;
      }
      break;
    }
    case kBrightness: {
      const Blend bl(mag);
      for (int q = tid; q < CHW; q += kT) out[q] = bl((float)in[q], 0.f);
      break;
    }
    case kColor: {
      if (C == 1) {
        for (int q = tid; q < CHW; q += kT) out[q] = in[q];
        break;
      }
      const Blend bl(mag);
      for (int q = tid; q < HW; q += kT) {
        const float g = (float)gray_u8(in, q, C, HW);
        for (int c = 0; c < C; ++c) out[c * HW + q] = bl((float)in[c * HW + q], g);
      }
      break;
    }
    case kContrast: {
      if (tid == 0) scr[kRed] = 0;
      __syncthreads();
      int s = 0;
      for (int q = tid; q < HW; q += kT) s += gray_u8(in, q, C, HW);
      atomicAdd(&scr[kRed], s);
      __syncthreads();
      const float mean = (float)scr[kRed] / (float)HW;
      const Blend bl(mag);
      for (int q = tid; q < CHW; q += kT) out[q] = bl((float)in[q], mean);
      break;
    }
    case kSharpness: {
      const Blend bl(mag);
      for (int q = tid; q < CHW; q += kT) {
        const int c = q / HW, r = q - c * HW, j = r / W, i = r - j * W;
        const float x = (float)in[q];
        float deg = x;
        if (j > 0 && j < H - 1 && i > 0 && i < W - 1) {
          const uint8_t* b = in + q;
          const int s = b[-W - 1] + b[-W] + b[-W + 1] + b[-1] + 5 * b[0] + b[1] + b[W - 1] + b[W] + b[W + 1];
          deg = rintf((float)s / 13.0f);
        }
        out[q] = bl(x, deg);
      }
      break;
    }
    case kPosterize: {
      const int bits = (int)mag;
      const uint8_t mask = (uint8_t)((0xFF << (8 - bits)) & 0xFF);
      for (int q = tid; q < CHW; q += kT) out[q] = in[q] & mask;
      break;
    }
    case kSolarize: {
      for (int q = tid; q < CHW; q += kT) out[q] = (float)in[q] >= mag ? (uint8_t)(255 - in[q]) : in[q];
      break;
    }
    case kAutoContrast: {
      if (tid < C) {
        scr[kRed + tid] = 255;      // min
        scr[kRed + 4 + tid] = 0;    // max
      }
      __syncthreads();
      for (int c = 0; c < C; ++c) {
        int lo = 255, hi = 0;
        for (int q = tid; q < HW; q += kT) {
          const int v = in[c * HW + q];
          lo = min(lo, v);
          hi = max(hi, v);
        }
        atomicMin(&scr[kRed + c], lo);
        atomicMax(&scr[kRed + 4 + c], hi);
      }
      __syncthreads();
      for (int q = tid; q < CHW; q += kT) {
        const int c = q / HW;
        float lo = (float)scr[kRed + c];
        const float hi = (float)scr[kRed + 4 + c];
        float scale;
        if (hi == lo) {
          lo = 0.f;
          scale = 1.f;
        } else {
          scale = 255.f / (hi - lo);
        }
        out[q] = trunc_u8(((float)in[q] - lo) * scale);
      }
      break;
    }
    case kEqualize: {
      for (int q = tid; q < C * 256; q += kT) scr[q] = 0;
      __syncthreads();
      for (int q = tid; q < CHW; q += kT) atomicAdd(&scr[(q / HW) * 256 + in[q]], 1);
      __syncthreads();
      // one wave per channel: step = (sum of all bins but the highest non-empty one) / 255,
      // lut[v] = v == 0 ? 0 : min(255, (cdf[v-1] + step/2) / step)  (torchvision _scale_channel)
      const int wave = tid >> 6, lane = tid & 63;
      if (wave < C) {
        int* h = scr + wave * 256;
        int v4[4], s = 0, top = -1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v4[k] = h[lane * 4 + k];
          s += v4[k];
          if (v4[k] > 0) top = lane * 4 + k;
        }
        int incl = s;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
          const int t = __shfl_up(incl, o, 64);
          if (lane >= o) incl += t;
        }
        int tmax = top;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) tmax = max(tmax, __shfl_xor(tmax, o, 64));
        const int total = __shfl(incl, 63, 64);
        const int top_count = __shfl(v4[tmax & 3], tmax >> 2, 64);
        const int step = (total - top_count) / 255;
        int cdf = incl - s;  // exclusive prefix before this lane's first bin
        int lut[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int v = lane * 4 + k;
          lut[k] = v == 0 ? 0 : min(255, step > 0 ? (cdf + step / 2) / step : v);
          cdf += v4[k];
        }
        // identity when step == 0 (lut[v] = v); all lanes read their bins before any write
#pragma unroll
        for (int k = 0; k < 4; ++k) h[lane * 4 + k] = step > 0 ? lut[k] : lane * 4 + k;
      }
      __syncthreads();
      for (int q = tid; q < CHW; q += kT) out[q] = (uint8_t)scr[(q / HW) * 256 + in[q]];
      break;
    }
    case kInvert: {
      for (int q = tid; q < CHW; q += kT) out[q] = (uint8_t)(255 - in[q]);
      break;
    }
    default: {
      for (int q = tid; q < CHW; q += kT) out[q] = in[q];
      break;
    }
  }
  __syncthreads();
}

__device__ __forceinline__ float signed_mag(const AugParams& p, int op, int bin, int sign) {
  if (bin < 0 || op < 0 || op >= kAugOps) return 0.f;
  const float m = p.mags[op][bin];
  return (p.signed_op[op] && sign == 0) ? -m : m;
}

template <bool OUT_F32>
__global__ __launch_bounds__(kT) void augment_kernel(AugParams p) {
#pragma clang fp contract(off)
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  const int C = p.C, H = p.H, W = p.W, HW = H * W, CHW = C * HW;
  const int img_bytes = (CHW + 15) & ~15;
  uint8_t* buf0 = smem;
  uint8_t* buf1 = smem + img_bytes;
  int* scr = reinterpret_cast<int*>(smem + 2 * img_bytes);
  const int tid = threadIdx.x, b = blockIdx.x;
  int64_t row = p.index[b];
  if (row < 0 || row >= p.n_images) row = 0;  // (the host validates the index range)
  const uint8_t* src = p.images + row * (int64_t)CHW;
  if ((CHW & 3) == 0) {
    for (int q = tid; q < CHW / 4; q += kT) reinterpret_cast<uint32_t*>(buf0)[q] = reinterpret_cast<const uint32_t*>(src)[q];
  } else {
    for (int q = tid; q < CHW; q += kT) buf0[q] = src[q];
  }
  __syncthreads();

  const uint64_t h0 = smix64(p.seed ^ ((uint64_t)b * 0xD1B54A32D192ED03ull));
  const uint64_t h1 = smix64(h0);
  uint8_t* cur = buf0;
  uint8_t* nxt = buf1;
  if (p.fixed_op >= 0) {
    apply_op(p, p.fixed_op, p.fixed_bin, signed_mag(p, p.fixed_op, p.fixed_bin, p.fixed_sign), cur, nxt, scr);
    uint8_t* t = cur; cur = nxt; nxt = t;
  } else if ((p.mode & 1) && p.n_policies > 0) {
    const int pol = (int)((h0 >> 32) % (uint64_t)p.n_policies);
    const float u[2] = {(float)(h0 & 0xFFFFFF) * (1.0f / 16777216.0f), (float)(h1 >> 40) * (1.0f / 16777216.0f)};
    const int sg[2] = {(int)((h1 >> 1) & 1), (int)((h1 >> 2) & 1)};
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int slot = 2 * pol + k;
      if (u[k] <= p.pol_prob[slot]) {
        const int op = p.pol_op[slot], bin = p.pol_bin[slot];
        apply_op(p, op, bin, signed_mag(p, op, bin, sg[k]), cur, nxt, scr);
        uint8_t* t = cur; cur = nxt; nxt = t;
      }
    }
  }
  const bool fc = (p.mode & 2) != 0;
  const int flip = fc ? (int)((h1 >> 3) & 1) : 0;
  const int span = 2 * p.pad + 1;
  const int dy = fc ? (int)(((h1 >> 8) & 0xFF) % (uint64_t)span) - p.pad : 0;
  const int dx = fc ? (int)(((h1 >> 16) & 0xFF) % (uint64_t)span) - p.pad : 0;
  const int64_t obase = (int64_t)b * CHW;
  for (int q = tid; q < CHW; q += kT) {
    const int c = q / HW, r = q - c * HW, j = r / W, i = r - j * W;
    const int sy = j + dy, sxf = i + dx;  // position in the (flipped) image
    float v = 0.f;
    if (sy >= 0 && sy < H && sxf >= 0 && sxf < W) v = (float)cur[c * HW + sy * W + (flip ? W - 1 - sxf : sxf)];
    const float y = v * p.a[c] + p.b[c];
    if constexpr (OUT_F32) reinterpret_cast<float*>(p.out)[obase + q] = y;
    else reinterpret_cast<bf16_t*>(p.out)[obase + q] = f2bf(y);
  }
}

}  // namespace

hipError_t augment_batch(const AugParams& p, bool out_f32, hipStream_t s) {
  if (p.B <= 0) return hipSuccess;
  const int CHW = p.C * p.H * p.W;
  if (p.C < 1 || p.C > 3 || CHW > kAugMaxPixels || p.n_policies * 2 > kAugPolicySlots || p.pad < 0 || p.pad > 64)
    return hipErrorInvalidValue;
  const size_t lds = 2 * (size_t)((CHW + 15) & ~15) + (size_t)(3 * 256 + 16) * 4;
  if (out_f32) augment_kernel<true><<<p.B, kT, lds, s>>>(p);
  else augment_kernel<false><<<p.B, kT, lds, s>>>(p);
  return hipGetLastError();
}

}  // namespace ldnn
