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

}  // namespace can

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
