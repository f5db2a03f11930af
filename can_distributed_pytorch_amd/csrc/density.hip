// Geometry-adaptive Gaussian density-map generator on the GPU (gfx950).
//
// Reference: data_preparation/k_nearest_gaussian_kernel.py:14-54 — KD-tree
// 4-NN query, sigma = 0.1 * (d1 + d2 + d3) (avg(shape)/4 for a single
// head), a unit delta at (int(y), int(x)) filtered by scipy gaussian_filter
// (mode='constant', truncate=4.0), summed over heads: O(N*H*W) on the CPU,
// "one minute or more per thousand heads".
//
// Here: (1) knn: one thread per head, brute-force over all heads staged
// through LDS in 256-point tiles, keeping the 4 smallest squared distances
// (self included, like the tree query); (2) splat: one workgroup per head
// writes the clipped outer product of two normalised 1-D Gaussians of radius
// R = int(4*sigma + 0.5) — exactly what gaussian_filter does to a delta
// (SURVEY §2.7), for any radius (the sigma = (H+W)/8 single-head case at
// 768x1024 has R = 896) — with fp32 atomics (the sum order across heads is not fixed:
// bitwise run-to-run reproducibility is NOT guaranteed, equality to ~1e-7 is).
#include "common.h"

namespace can {

__global__ void __launch_bounds__(256) density_knn_kernel(const float2* __restrict__ pts, int n,
                                                          float* __restrict__ sigma, float single_sigma) {
  __shared__ float2 tile[256];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const float2 me = (i < n) ? pts[i] : make_float2(0.f, 0.f);
  float d[4] = {3.4e38f, 3.4e38f, 3.4e38f, 3.4e38f};
  for (int base = 0; base < n; base += 256) {
    const int j = base + threadIdx.x;
    tile[threadIdx.x] = (j < n) ? pts[j] : make_float2(3.0e18f, 3.0e18f);
    __syncthreads();
    const int cnt = min(256, n - base);
    for (int t = 0; t < cnt; ++t) {
      const float dx = tile[t].x - me.x, dy = tile[t].y - me.y;
      float v = dx * dx + dy * dy;
      // insertion into the sorted 4-list
      if (v < d[3]) {
        if (v < d[2]) {
          d[3] = d[2];
          if (v < d[1]) {
            d[2] = d[1];
            if (v < d[0]) { d[1] = d[0]; d[0] = v; }
            else d[1] = v;
          } else d[2] = v;
        } else d[3] = v;
      }
    }
    __syncthreads();
  }
  if (i < n) {
    if (n == 1) sigma[i] = single_sigma;
    else {
      // k=4 with fewer than 4 points: scipy returns inf distances -> sigma inf;
      // the reference then filters with an infinite sigma (degenerate).  Use the
      // available neighbours only.
      float s = 0.f;
      for (int k = 1; k < 4 && k < n; ++k) s += sqrtf(d[k]);
      sigma[i] = 0.1f * s;
    }
  }
}

// one block per head; threads cover the clipped (2R+1)^2 footprint.  Any radius: the normaliser
// sum_{t=-R..R} exp(-t^2 / 2 s^2) is a block reduction over the WHOLE kernel (mass outside the image is
// dropped after normalising, like gaussian_filter on a delta), the 1-D weights are tabulated in dynamic
// LDS only over the clipped window (<= H rows + W columns).  max_r > 0 optionally caps R.
__global__ void __launch_bounds__(256) density_splat_kernel(const float2* __restrict__ pts,
                                                            const float* __restrict__ sigma, int n, int H, int W,
                                                            float* __restrict__ out, int max_r) {
  extern __shared__ float tab[];                 // [H] row weights, then [W] column weights
  __shared__ float red[4];
  const int i = blockIdx.x;
  if (i >= n) return;
  const float2 p = pts[i];
  const int px = (int)p.x, py = (int)p.y;      // python int() truncation
  if (p.x < 0.f || p.y < 0.f || px >= W || py >= H) return;   // reference skips out-of-image heads
  const float s = sigma[i];
  if (s <= 0.f) {   // degenerate: delta
    if (threadIdx.x == 0) atomicAdd(out + (size_t)py * W + px, 1.f);
    return;
  }
  const float rf = 4.0f * s + 0.5f;
  int R = (rf >= 2.0e9f) ? 2000000000 : (int)rf;
  if (max_r > 0 && R > max_r) R = max_r;
  const float k = -0.5f / (s * s);
  // normaliser over the full 2R+1 taps (fixed per-thread stride order + fixed tree: deterministic)
  float part = 0.f;
  for (long long t = (long long)threadIdx.x - R; t <= R; t += 256) {
    const float x = (float)t;
    part += __expf(k * x * x);
  }
  part = wave_sum(part);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = part;
  __syncthreads();
  const float inv_sum = 1.f / ((red[0] + red[1]) + (red[2] + red[3]));
  const int y0 = max(0, py - R), y1 = min(H - 1, py + R);
  const int x0 = max(0, px - R), x1 = min(W - 1, px + R);
  const int w = x1 - x0 + 1, h = y1 - y0 + 1;
  float* ky = tab;
  float* kx = tab + h;
  for (int t = threadIdx.x; t < h; t += 256) {
    const float d = (float)(y0 + t - py);
    ky[t] = __expf(k * d * d) * inv_sum;
  }
  for (int t = threadIdx.x; t < w; t += 256) {
    const float d = (float)(x0 + t - px);
    kx[t] = __expf(k * d * d) * inv_sum;
  }
  __syncthreads();
  for (int t = threadIdx.x; t < w * h; t += 256) {
    const int yy = t / w, xx = t - yy * w;
    atomicAdd(out + (size_t)(y0 + yy) * W + x0 + xx, ky[yy] * kx[xx]);
  }
}

__global__ void density_fill_kernel(float* __restrict__ sigma, int n, float v) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) sigma[i] = v;
}

}  // namespace can

// fixed_sigma > 0: every head gets that sigma (no kNN; the synthetic-data generator's fixed-width heads)
extern "C" int can_density_map(const float* pts, int n, int H, int W, float* sigma_ws, float* out, int max_r,
                               void* stream, float fixed_sigma) {
  using namespace can;
  hipStream_t s = (hipStream_t)stream;
  if (n <= 0) return 0;
  const size_t lds = (size_t)(H + W) * sizeof(float);
  if (lds > 150 * 1024) return -2;                      // weight tables of one clipped footprint in LDS
  if (fixed_sigma > 0.f) {
    hipLaunchKernelGGL(density_fill_kernel, dim3((n + 255) / 256), dim3(256), 0, s, sigma_ws, n, fixed_sigma);
  } else {
    const float single = 0.25f * 0.5f * (float)(H + W);   // avg(shape)/2/2 (reference intent, Q9)
    hipLaunchKernelGGL(density_knn_kernel, dim3((n + 255) / 256), dim3(256), 0, s, (const float2*)pts, n, sigma_ws,
                       single);
  }
  if (lds > 64 * 1024)
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)density_splat_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                      (int)lds));
  hipLaunchKernelGGL(density_splat_kernel, dim3(n), dim3(256), lds, s, (const float2*)pts, sigma_ws, n, H, W, out,
                     max_r);
  return (int)hipGetLastError();
}
