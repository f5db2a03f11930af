// GPU input pipeline for CrowdDataset samples (gfx950).
//
// Reference semantics (model/CrowdDataset.py:38-67): image/255 -> optional
// horizontal flip -> cv2.resize(INTER_LINEAR) to (W//8*8, H//8*8) ->
// ImageNet normalisation; density -> same flip -> cv2.resize to (W//8, H//8)
// -> x64.  cv2's INTER_LINEAR = half-pixel-centre bilinear, source
// coordinate clamped at 0 (left/top) and taps clamped at the last pixel,
// no anti-aliasing.  Here both run on the GPU straight from the decoded uint8
// image and write the first conv layer's NHWC4 bf16 layout (channel 3 = 0),
// so the host only decodes JPEGs.
#include "common.h"

namespace can {

__device__ __forceinline__ void lin_tap(int o, float scale, int in, int& i0, int& i1, float& f) {
  float src = ((float)o + 0.5f) * scale - 0.5f;
  if (src < 0.f) src = 0.f;
  int x0 = (int)src;
  f = src - (float)x0;
  if (x0 >= in - 1) { x0 = in - 1; f = 0.f; }
  i0 = x0;
  i1 = min(x0 + 1, in - 1);
}

// img: uint8 [H0][W0][C] (C = 1, 3 or 4) -> out NHWC4 bf16 [Ho][Wo][4] (sample n of a batch)
template <int DT>
__global__ void __launch_bounds__(256) preprocess_image_kernel(const unsigned char* __restrict__ img, int H0, int W0,
                                                               int C, int flip, uint2* __restrict__ out, int Ho,
                                                               int Wo, float m0, float m1, float m2, float is0,
                                                               float is1, float is2) {
  const float sy = (float)H0 / (float)Ho, sx = (float)W0 / (float)Wo;
  const int total = Ho * Wo;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int oy = i / Wo, ox = i % Wo;
    int y0, y1, x0, x1;
    float fy, fx;
    lin_tap(oy, sy, H0, y0, y1, fy);
    lin_tap(ox, sx, W0, x0, x1, fx);
    if (flip) {   // flip happens BEFORE the resize in the reference: mirror the source columns
      x0 = W0 - 1 - x0;
      x1 = W0 - 1 - x1;
    }
    float v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int cc = (C == 1) ? 0 : c;
      const float a = img[((size_t)y0 * W0 + x0) * C + cc], b = img[((size_t)y0 * W0 + x1) * C + cc];
      const float d = img[((size_t)y1 * W0 + x0) * C + cc], e = img[((size_t)y1 * W0 + x1) * C + cc];
      const float top = a + (b - a) * fx, bot = d + (e - d) * fx;
      v[c] = (top + (bot - top) * fy) * (1.f / 255.f);
    }
    out[i] = make_uint2(pack2<DT>((v[0] - m0) * is0, (v[1] - m1) * is1), pack2<DT>((v[2] - m2) * is2, 0.f));
  }
}

// density fp32 [H0][W0] -> [Ho][Wo] x mult (after optional flip)
__global__ void __launch_bounds__(256) preprocess_density_kernel(const float* __restrict__ d, int H0, int W0, int flip,
                                                                 float* __restrict__ out, int Ho, int Wo, float mult) {
  const float sy = (float)H0 / (float)Ho, sx = (float)W0 / (float)Wo;
  const int total = Ho * Wo;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < total; i += gridDim.x * 256) {
    const int oy = i / Wo, ox = i % Wo;
    int y0, y1, x0, x1;
    float fy, fx;
    lin_tap(oy, sy, H0, y0, y1, fy);
    lin_tap(ox, sx, W0, x0, x1, fx);
    if (flip) { x0 = W0 - 1 - x0; x1 = W0 - 1 - x1; }
    const float a = d[(size_t)y0 * W0 + x0], b = d[(size_t)y0 * W0 + x1];
    const float c = d[(size_t)y1 * W0 + x0], e = d[(size_t)y1 * W0 + x1];
    const float top = a + (b - a) * fx, bot = c + (e - c) * fx;
    out[i] = (top + (bot - top) * fy) * mult;
  }
}

// Whole batch in ONE launch: variable-size samples packed back to back in one uint8 image buffer and one
// fp32 density buffer (one H2D copy each); desc[n] = {image byte offset, H0, W0, C, flip, density float
// offset, 0, 0}.  blockIdx.y = sample, blockIdx.z = 0: image -> NHWC4 [Ho][Wo][4], 1: density -> [Ho/d][Wo/d].
template <int DT>
__global__ void __launch_bounds__(256) preprocess_batch_kernel(const unsigned char* __restrict__ imgs,
                                                               const float* __restrict__ dens,
                                                               const long long* __restrict__ desc,
                                                               uint2* __restrict__ x4, float* __restrict__ gt, int Ho,
                                                               int Wo, int ds, float mult) {
  const long long* d = desc + (size_t)blockIdx.y * 8;
  const int H0 = (int)d[1], W0 = (int)d[2], C = (int)d[3], flip = (int)d[4];
  if (blockIdx.z == 0) {
    const unsigned char* img = imgs + d[0];
    uint2* out = x4 + (size_t)blockIdx.y * Ho * Wo;
    const float sy = (float)H0 / (float)Ho, sx = (float)W0 / (float)Wo;
    const float m[3] = {0.485f, 0.456f, 0.406f}, is[3] = {1.f / 0.229f, 1.f / 0.224f, 1.f / 0.225f};
    for (int i = blockIdx.x * 256 + threadIdx.x; i < Ho * Wo; i += gridDim.x * 256) {
      const int oy = i / Wo, ox = i % Wo;
      int y0, y1, x0, x1;
      float fy, fx;
      lin_tap(oy, sy, H0, y0, y1, fy);
      lin_tap(ox, sx, W0, x0, x1, fx);
      if (flip) { x0 = W0 - 1 - x0; x1 = W0 - 1 - x1; }
      float v[3];
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const int cc = (C == 1) ? 0 : c;
        const float a = img[((size_t)y0 * W0 + x0) * C + cc], b = img[((size_t)y0 * W0 + x1) * C + cc];
        const float e0 = img[((size_t)y1 * W0 + x0) * C + cc], e1 = img[((size_t)y1 * W0 + x1) * C + cc];
        const float top = a + (b - a) * fx, bot = e0 + (e1 - e0) * fx;
        v[c] = ((top + (bot - top) * fy) * (1.f / 255.f) - m[c]) * is[c];
      }
      out[i] = make_uint2(pack2<DT>(v[0], v[1]), pack2<DT>(v[2], 0.f));
    }
  } else {
    const float* dm = dens + d[5];
    const int Hd = Ho / ds, Wd = Wo / ds;
    float* out = gt + (size_t)blockIdx.y * Hd * Wd;
    const float sy = (float)H0 / (float)Hd, sx = (float)W0 / (float)Wd;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < Hd * Wd; i += gridDim.x * 256) {
      const int oy = i / Wd, ox = i % Wd;
      int y0, y1, x0, x1;
      float fy, fx;
      lin_tap(oy, sy, H0, y0, y1, fy);
      lin_tap(ox, sx, W0, x0, x1, fx);
      if (flip) { x0 = W0 - 1 - x0; x1 = W0 - 1 - x1; }
      const float a = dm[(size_t)y0 * W0 + x0], b = dm[(size_t)y0 * W0 + x1];
      const float c = dm[(size_t)y1 * W0 + x0], e = dm[(size_t)y1 * W0 + x1];
      const float top = a + (b - a) * fx, bot = c + (e - c) * fx;
      out[i] = (top + (bot - top) * fy) * mult;
    }
  }
}

// ---------------------------------------------------------------------------
// Synthetic crowd batch on the GPU (train.py --synthetic / bench data; data/synthetic.py is the CPU
// reference of the same recipe): per image, head points (host RNG, tiny) -> fixed-sigma Gaussian
// density (density_splat, density.hip) -> 8x8 sum-pool to the 1/8 ground truth (count preserving);
// image = bilinear upsample of a coarse noise grid + 0.3 * density / max(density), ImageNet-normalised,
// written as NHWC4 16-bit.
// dens: [N][H][W] fp32 full-res density, noise: [N][3][H/16][W/16] fp32, dmax: [N] per-image max.
__global__ void __launch_bounds__(256) synth_gt_kernel(const float* __restrict__ dens, float* __restrict__ gt,
                                                       float* __restrict__ dmax, int H, int W) {
  // blockIdx.y = image: 8x8 sum pool + per-image max (block-level max -> atomicMax on the float bits,
  // valid for the non-negative densities)
  const float* d = dens + (size_t)blockIdx.y * H * W;
  const int Hd = H / 8, Wd = W / 8;
  float mx = 0.f;
  for (int i = blockIdx.x * 256 + threadIdx.x; i < Hd * Wd; i += gridDim.x * 256) {
    const int oy = i / Wd, ox = i % Wd;
    float s = 0.f;
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const float v = d[(size_t)(oy * 8 + r) * W + ox * 8 + c];
        s += v;
        mx = fmaxf(mx, v);
      }
    gt[(size_t)blockIdx.y * Hd * Wd + i] = s;
  }
  mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 16, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 8, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 4, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 2, 64));
  mx = fmaxf(mx, __shfl_xor(mx, 1, 64));
  if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<int*>(dmax + blockIdx.y), __float_as_int(mx));
}

template <int DT>
__global__ void __launch_bounds__(256) synth_image_kernel(const float* __restrict__ dens,
                                                          const float* __restrict__ noise,
                                                          const float* __restrict__ dmax, uint2* __restrict__ x4,
                                                          int H, int W) {
  const int n = blockIdx.y, Hn = H / 16, Wn = W / 16;
  const float* d = dens + (size_t)n * H * W;
  const float* nz = noise + (size_t)n * 3 * Hn * Wn;
  const float inv = 1.f / (dmax[n] + 1e-6f);
  const float m[3] = {0.485f, 0.456f, 0.406f}, is[3] = {1.f / 0.229f, 1.f / 0.224f, 1.f / 0.225f};
  for (int i = blockIdx.x * 256 + threadIdx.x; i < H * W; i += gridDim.x * 256) {
    const int oy = i / W, ox = i % W;
    int y0, y1, x0, x1;
    float fy, fx;
    lin_tap(oy, (float)Hn / (float)H, Hn, y0, y1, fy);
    lin_tap(ox, (float)Wn / (float)W, Wn, x0, x1, fx);
    const float blob = 0.3f * d[i] * inv;
    float v[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float* p = nz + (size_t)c * Hn * Wn;
      const float top = p[y0 * Wn + x0] + (p[y0 * Wn + x1] - p[y0 * Wn + x0]) * fx;
      const float bot = p[y1 * Wn + x0] + (p[y1 * Wn + x1] - p[y1 * Wn + x0]) * fx;
      const float px = fminf(fmaxf(0.7f * (top + (bot - top) * fy) + blob, 0.f), 1.f);
      v[c] = (px - m[c]) * is[c];
    }
    x4[(size_t)n * H * W + i] = make_uint2(pack2<DT>(v[0], v[1]), pack2<DT>(v[2], 0.f));
  }
}

}  // namespace can

extern "C" int can_preprocess_batch(const void* imgs, const float* dens, const long long* desc, int n, void* x4,
                                    float* gt, int Ho, int Wo, int ds, int dt, void* stream) {
  using namespace can;
  if (n <= 0 || Ho % ds || Wo % ds) return -2;
  int bx = (Ho * Wo + 255) / 256;
  if (bx > 512) bx = 512;
  // dens == nullptr: the ground truth arrived already at 1/ds resolution (images only)
  CAN_LAUNCH_DT(dt, preprocess_batch_kernel, dim3(bx, n, (dens != nullptr && gt != nullptr) ? 2 : 1), dim3(256), 0,
                (hipStream_t)stream,
                (const unsigned char*)imgs, dens, desc, (uint2*)x4, gt, Ho, Wo, ds, (float)(ds * ds));
  return (int)hipGetLastError();
}

extern "C" int can_synth_render(const float* dens, const float* noise, float* dmax, void* x4, float* gt, int n, int H,
                                int W, int dt, void* stream) {
  using namespace can;
  if (n <= 0 || H % 16 || W % 16) return -2;
  hipStream_t s = (hipStream_t)stream;
  CAN_HIP_CHECK(hipMemsetAsync(dmax, 0, sizeof(float) * n, s));
  int bx = (H / 8 * (W / 8) + 255) / 256;
  if (bx > 256) bx = 256;
  hipLaunchKernelGGL(synth_gt_kernel, dim3(bx, n), dim3(256), 0, s, dens, gt, dmax, H, W);
  int bi = (H * W + 255) / 256;
  if (bi > 1024) bi = 1024;
  CAN_LAUNCH_DT(dt, synth_image_kernel, dim3(bi, n), dim3(256), 0, s, dens, noise, dmax, (uint2*)x4, H, W);
  return (int)hipGetLastError();
}

extern "C" int can_preprocess_image(const void* img, int H0, int W0, int C, int flip, void* out, int Ho, int Wo, int dt,
                                    void* stream) {
  using namespace can;
  if (C != 1 && C != 3 && C != 4) return -2;
  const int total = Ho * Wo;
  const int grid = (total + 255) / 256 > 4096 ? 4096 : (total + 255) / 256;
  CAN_LAUNCH_DT(dt, preprocess_image_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const unsigned char*)img,
                H0, W0, C, flip, (uint2*)out, Ho, Wo, 0.485f, 0.456f, 0.406f, 1.f / 0.229f, 1.f / 0.224f,
                1.f / 0.225f);
  return (int)hipGetLastError();
}

extern "C" int can_preprocess_density(const float* d, int H0, int W0, int flip, float* out, int Ho, int Wo,
                                      float mult, void* stream) {
  using namespace can;
  const int total = Ho * Wo;
  const int grid = (total + 255) / 256 > 4096 ? 4096 : (total + 255) / 256;
  hipLaunchKernelGGL(preprocess_density_kernel, dim3(grid), dim3(256), 0, (hipStream_t)stream, d, H0, W0, flip, out,
                     Ho, Wo, mult);
  return (int)hipGetLastError();
}
