// Memory-bound kernels of the CANNet step (gfx950): all NHWC bf16, 16-B
// vectorised per lane (8 channels), grid-stride, no atomics on hot paths.
//
//   maxpool2x2_fwd      nn.MaxPool2d(2,2)                  model/CANNet.py:112
//                       (+ optional max-pool codes: first-max one-hots, see conv_igemm.hip)
//   maxpool2x2_bwd_codes max-pool backward + ReLU mask from the codes alone
//   maxpool2x2_bwd_relu max_pool2d_with_indices_backward + threshold_backward
//                       (gather form: first-max-in-window wins, as ATen; the
//                       ReLU mask of the pooled layer is folded in)
//   head_fwd            output_layer 1x1 64->1 + bias       model/CANNet.py:17,90
//   head_train          head fwd + MSELoss(sum) + its backward + ReLU mask of
//                       the last backend layer, one pass      utils/train_eval_utils.py:20,37-38
//   sgd_momentum        torch.optim.SGD(momentum=0.95) step over the flat fp32
//                       arena, gradient averaging folded in, skipped on a
//                       device-side non-finite flag             train.py:126
//   pack_conv           fp32 [Co][Ci][kh][kw] -> bf16 forward / dgrad packs
//   img_to_nhwc4        [N,3,H,W] fp32 -> [N,H,W,4] bf16 (first-layer input)
#include "common.h"

namespace can {

// ---------------------------------------------------------------- maxpool
// codes (optional): per pooled pixel and 8-channel chunk, one uint32 of 4-bit one-hot first-max positions
// (ATen order, 0 when the max is not > 0) — the layout of the conv pool epilogues (conv_igemm.hip)
template <int DT>
__global__ void __launch_bounds__(256) maxpool_fwd_kernel(const uint4* __restrict__ x, uint4* __restrict__ y,
                                                          uint32_t* __restrict__ codes, int N, int H, int W, int C8) {
  const int Ho = H >> 1, Wo = W >> 1;
  const size_t total = (size_t)N * Ho * Wo * C8;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int c = i % C8;
    size_t p = i / C8;
    const int ox = p % Wo; p /= Wo;
    const int oy = p % Ho; const int n = p / Ho;
    const size_t base = (((size_t)n * H + 2 * oy) * W + 2 * ox) * C8 + c;
    float t[4][8], m[8];
    unpack8h<DT>(x[base], t[0]);
    unpack8h<DT>(x[base + C8], t[1]);
    unpack8h<DT>(x[base + (size_t)W * C8], t[2]);
    unpack8h<DT>(x[base + (size_t)W * C8 + C8], t[3]);
#pragma unroll
    for (int k = 0; k < 8; ++k) m[k] = fmaxf(fmaxf(t[0][k], t[1][k]), fmaxf(t[2][k], t[3][k]));
    y[i] = pack8h<DT>(m);  // exact: max of bf16 values is a bf16 value
    if (codes != nullptr) {
      uint32_t cw = 0u;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const uint32_t first = (t[0][k] == m[k]) ? 1u : (t[1][k] == m[k]) ? 2u : (t[2][k] == m[k]) ? 4u : 8u;
        cw |= ((m[k] > 0.f) ? first : 0u) << (4 * k);
      }
      codes[i] = cw;
    }
  }
}

// dx[full] = dy[pooled] at the window position the code marks, 0 elsewhere (max-pool backward + the ReLU
// mask of the pool input, from the codes alone: the pool input is not read)
template <int DT>
__global__ void __launch_bounds__(256) maxpool_bwd_codes_kernel(const uint32_t* __restrict__ codes,
                                                                const uint4* __restrict__ dy, uint4* __restrict__ dx,
                                                                int N, int H, int W, int C8) {
  const int Ho = H >> 1, Wo = W >> 1;
  const size_t total = (size_t)N * Ho * Wo * C8;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int c = i % C8;
    size_t p = i / C8;
    const int ox = p % Wo; p /= Wo;
    const int oy = p % Ho; const int n = p / Ho;
    const size_t b0 = (((size_t)n * H + 2 * oy) * W + 2 * ox) * C8 + c;
    const size_t off[4] = {b0, b0 + C8, b0 + (size_t)W * C8, b0 + (size_t)W * C8 + C8};
    float g[8], o[4][8];
    unpack8h<DT>(dy[i], g);
    const uint32_t cw = codes[i];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t nib = (cw >> (4 * k)) & 0xFu;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q][k] = ((nib >> q) & 1u) ? g[k] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) dx[off[q]] = pack8h<DT>(o[q]);
  }
}

// dx[full] = (x is the first max of its window) * (x > 0) * dy[pooled]
template <int DT>
__global__ void __launch_bounds__(256) maxpool_bwd_relu_kernel(const uint4* __restrict__ x, const uint4* __restrict__ dy,
                                                               uint4* __restrict__ dx, int N, int H, int W, int C8) {
  const int Ho = H >> 1, Wo = W >> 1;
  const size_t total = (size_t)N * Ho * Wo * C8;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int c = i % C8;
    size_t p = i / C8;
    const int ox = p % Wo; p /= Wo;
    const int oy = p % Ho; const int n = p / Ho;
    const size_t b0 = (((size_t)n * H + 2 * oy) * W + 2 * ox) * C8 + c;
    const size_t off[4] = {b0, b0 + C8, b0 + (size_t)W * C8, b0 + (size_t)W * C8 + C8};
    float v[4][8], g[8];
#pragma unroll
    for (int q = 0; q < 4; ++q) unpack8h<DT>(x[off[q]], v[q]);
    unpack8h<DT>(dy[i], g);
    float o[4][8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      // ATen scan order: (0,0),(0,1),(1,0),(1,1); strict '>' keeps the first max
      int arg = 0;
      float mv = v[0][k];
#pragma unroll
      for (int q = 1; q < 4; ++q)
        if (v[q][k] > mv) { mv = v[q][k]; arg = q; }
      const float gg = (mv > 0.f) ? g[k] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) o[q][k] = (q == arg) ? gg : 0.f;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) dx[off[q]] = pack8h<DT>(o[q]);
  }
}

// ---------------------------------------------------------------- head
// et[p] = sum_c y[p][c] * w[c] + b      (y: [P][64] bf16 post-ReLU)
template <int DT>
__global__ void __launch_bounds__(256) head_fwd_kernel(const uint4* __restrict__ y, const float* __restrict__ w,
                                                       const float* __restrict__ b, float* __restrict__ et, int P) {
  // 8 lanes per pixel (8 channels each)
  const int lane8 = threadIdx.x & 7;
  float wl[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) wl[k] = w[lane8 * 8 + k];
  const float bias = b[0];
  for (size_t p = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 3; p < (size_t)P; p += ((size_t)gridDim.x * 256) >> 3) {
    float v[8];
    unpack8h<DT>(y[p * 8 + lane8], v);
    float s = 0.f;   // explicit fma chain: head_fwd and head_train produce bitwise-identical et
#pragma unroll
    for (int k = 0; k < 8; ++k) s = fmaf(v[k], wl[k], s);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    if (lane8 == 0) et[p] = s + bias;
  }
}

// Training head: et = y.w + b; loss = sum (et-gt)^2; det = 2(et-gt)*gscale;
// dy[p][c] = det * S * w[c] * (y > 0) (S = device loss scale, 1 if null); partial dw[c] = sum_p det*y[p][c], db = sum det.
// Per-block partials -> part[block][66] (64 dw, db, loss); reduced by head_reduce.
template <int DT>
__global__ void __launch_bounds__(256) head_train_kernel(const uint4* __restrict__ y, const float* __restrict__ w,
                                                         const float* __restrict__ b, const float* __restrict__ gt,
                                                         float* __restrict__ et, uint4* __restrict__ dy,
                                                         float* __restrict__ part, int P, float gscale,
                                                         const float* __restrict__ lscale) {
  __shared__ float red[256 / 8][66];
  const float dys = (lscale != nullptr) ? lscale[0] : 1.f;   // loss scale: applied to dy only
  const int lane8 = threadIdx.x & 7;
  const int pg = threadIdx.x >> 3;
  float wl[8], dwl[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) { wl[k] = w[lane8 * 8 + k]; dwl[k] = 0.f; }
  const float bias = b[0];
  float dbl = 0.f, lossl = 0.f;
  for (size_t p = ((size_t)blockIdx.x * 256 + threadIdx.x) >> 3; p < (size_t)P; p += ((size_t)gridDim.x * 256) >> 3) {
    float v[8];
    unpack8h<DT>(y[p * 8 + lane8], v);
    float s = 0.f;   // explicit fma chain: head_fwd and head_train produce bitwise-identical et
#pragma unroll
    for (int k = 0; k < 8; ++k) s = fmaf(v[k], wl[k], s);
    s += __shfl_xor(s, 1, 64);
    s += __shfl_xor(s, 2, 64);
    s += __shfl_xor(s, 4, 64);
    const float e = s + bias;
    const float d = e - gt[p];
    const float g = 2.f * d * gscale;
    if (lane8 == 0) { et[p] = e; lossl += d * d; dbl += g; }
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o[k] = (v[k] > 0.f) ? g * dys * wl[k] : 0.f;
      dwl[k] += g * v[k];
    }
    dy[p * 8 + lane8] = pack8h<DT>(o);
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) red[pg][lane8 * 8 + k] = dwl[k];
  if (lane8 == 0) { red[pg][64] = dbl; red[pg][65] = lossl; }
  __syncthreads();
  if (threadIdx.x < 66) {
    float s = 0.f;
    for (int r = 0; r < 256 / 8; ++r) s += red[r][threadIdx.x];
    part[(size_t)blockIdx.x * 66 + threadIdx.x] = s;
  }
}

// out[0..63] = dw, out[64] = db, loss_out[0] = loss  (fixed-order, deterministic):
// 15 groups x 66 outputs, group g sums blocks g, g+15, ... then the 15 group
// sums are added in order (a single thread per output serialised ~1k loads).
// nonfinite (optional): 1.0 if the loss is inf/NaN, else 0.0 -- the
// reference's `if not isfinite(loss)` guard (utils/train_eval_utils.py:48)
// computed where the loss is produced, no extra launch.
__global__ void __launch_bounds__(1024) head_reduce_kernel(const float* __restrict__ part, int nblk,
                                                           float* __restrict__ dw, float* __restrict__ db,
                                                           float* __restrict__ loss, float beta,
                                                           float* __restrict__ nonfinite) {
  constexpr int G = 15;
  __shared__ float red[G][66];
  const int t = threadIdx.x;
  const int o = t % 66, g = t / 66;
  if (g < G) {
    float s0 = 0.f, s1 = 0.f;
    int i = g;
    for (; i + G < nblk; i += 2 * G) {
      s0 += part[(size_t)i * 66 + o];
      s1 += part[(size_t)(i + G) * 66 + o];
    }
    if (i < nblk) s0 += part[(size_t)i * 66 + o];
    red[g][o] = s0 + s1;
  }
  __syncthreads();
  if (t < 66) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < G; ++q) s += red[q][t];
    if (t < 64) dw[t] = (beta != 0.f) ? dw[t] * beta + s : s;
    else if (t == 64) db[0] = (beta != 0.f) ? db[0] * beta + s : s;
    else {
      loss[0] = s;
      if (nonfinite != nullptr) nonfinite[0] = isfinite(s) ? 0.f : 1.f;
    }
  }
}

// ---------------------------------------------------------------- SGD
// torch.optim.SGD semantics (dampening 0, nesterov False, wd 0):
//   buf = g (first step) | momentum*buf + g ;  p -= lr*buf,  g = grad*gscale.
// flags = {non-finite loss (all-reduced: any rank), loss, non-finite gradient
// (fp16 step), sticky "a non-finite loss happened since the last reset"}.
// flags[0] != 0 or flags[2] != 0 -> the whole update is skipped (graph-safe,
// no host sync); flags[0] != 0 also latches flags[3], which the host polls at
// its logging cadence (a NaN on a step it does not read is never lost).
// lr_dev (optional): the learning rate read from device memory, so a captured
// step follows an lr schedule (the host updates the scalar between replays).
// Vectorised float4 over a 16-B aligned arena.
__global__ void __launch_bounds__(256) sgd_momentum_kernel(float4* __restrict__ p, float4* __restrict__ buf,
                                                           const float4* __restrict__ g, size_t n4, float lr,
                                                           float momentum, float gscale, int first,
                                                           float* __restrict__ flags, const float* __restrict__ lr_dev) {
  if (flags != nullptr) {
    const bool bad_loss = flags[0] != 0.f;
    if (bad_loss && blockIdx.x == 0 && threadIdx.x == 0) flags[3] = 1.f;
    if (bad_loss || flags[2] != 0.f) return;
  }
  if (lr_dev != nullptr) lr = lr_dev[0];
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    float4 gv = g[i];
    gv.x *= gscale; gv.y *= gscale; gv.z *= gscale; gv.w *= gscale;
    float4 b;
    if (first) b = gv;
    else {
      b = buf[i];
      b.x = momentum * b.x + gv.x; b.y = momentum * b.y + gv.y;
      b.z = momentum * b.z + gv.z; b.w = momentum * b.w + gv.w;
    }
    buf[i] = b;
    float4 pv = p[i];
    pv.x -= lr * b.x; pv.y -= lr * b.y; pv.z -= lr * b.z; pv.w -= lr * b.w;
    p[i] = pv;
  }
}

// ---------------------------------------------------------------- loss scaling
// Dynamic loss scaling for the fp16 step, entirely device-side (graph-safe):
// grad_nonfinite ORs "some gradient is inf/NaN" into *flag (the step's
// flags[2], which the fused SGD skips on); scale_update then backs the scale
// off on overflow or grows it after `interval` clean steps.
// scaler = {S, 1/S, clean steps, 0}.
__global__ void __launch_bounds__(256) grad_nonfinite_kernel(const float4* __restrict__ g, size_t n4,
                                                             float* __restrict__ flag) {
  bool bad = false;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) {
    const float4 v = g[i];
    bad |= !(isfinite(v.x) && isfinite(v.y) && isfinite(v.z) && isfinite(v.w));
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<int*>(flag), 0x3f800000);   // 1.0f
}

// ---------------------------------------------------------------- split-bf16 (fp32 path)
// x = hi + lo with hi = bf16(x), lo = bf16(x - hi): the fp32 path (ops/fp32.py) computes every conv GEMM as
// hi*hi + hi*lo + lo*hi on the bf16 MFMA kernels with fp32 accumulation.  src fp32 [M][C]; three blocks,
// block b = lo if bit b of `pattern` is set, else hi:
//   mode 0 (K-concatenated operand): dst [M][stride], block b at channels [b*C, (b+1)*C), zero from 3*C on;
//   mode 1 (M-stacked operand):      dst [3][M][stride], block b = rows [b*M, (b+1)*M), zero from C on.
// General form (small or padded C, e.g. the 3-channel image into 64-channel rows): one thread per output row
// chunk of 8 values (one 16-byte store; stride % 8 == 0).
__global__ void __launch_bounds__(256) split_x3_kernel(const float* __restrict__ src, uint4* __restrict__ dst,
                                                       int M, int C, int stride, int mode, int pattern) {
  const int rows = (mode == 0 ? 1 : 3) * M, s8 = stride >> 3;
  const long long total = (long long)rows * s8;
  for (long long t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (long long)gridDim.x * 256) {
    const int row = (int)(t / s8), col0 = (int)(t - (long long)row * s8) * 8;
    const int b0 = (mode == 0) ? 0 : row / M;
    const int m = (mode == 0) ? row : row - b0 * M;
    unsigned short v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int col = col0 + k;
      const int b = (mode == 0) ? col / C : b0;
      const int c = (mode == 0) ? col - b * C : col;
      unsigned short o = 0;
      if (b < 3 && c < C) {
        const float x = src[(size_t)m * C + c];
        const unsigned short hi = f2bf(x);
        o = ((pattern >> b) & 1) ? f2bf(x - bf2f(hi)) : hi;
      }
      v[k] = o;
    }
    dst[t] = make_uint4(v[0] | ((unsigned)v[1] << 16), v[2] | ((unsigned)v[3] << 16), v[4] | ((unsigned)v[5] << 16),
                        v[6] | ((unsigned)v[7] << 16));
  }
}

// Fast path (C % 4 == 0, no padding columns): one thread per 4 source values; one float4 read, three 8-byte
// stores, 32-bit index math (the generic kernel's 64-bit divisions made it 30 % of the fp32 step).
__global__ void __launch_bounds__(256) split_x3_vec_kernel(const float4* __restrict__ src, uint2* __restrict__ dst,
                                                           int M, int C4, int mode, int pattern) {
  const int total = M * C4;
  for (int t = blockIdx.x * 256 + threadIdx.x; t < total; t += gridDim.x * 256) {
    const float4 x = src[t];
    const float xv[4] = {x.x, x.y, x.z, x.w};
    unsigned short hi[4], lo[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      hi[k] = f2bf(xv[k]);
      lo[k] = f2bf(xv[k] - bf2f(hi[k]));
    }
    const uint2 h = make_uint2(hi[0] | ((unsigned)hi[1] << 16), hi[2] | ((unsigned)hi[3] << 16));
    const uint2 l = make_uint2(lo[0] | ((unsigned)lo[1] << 16), lo[2] | ((unsigned)lo[3] << 16));
    const int m = t / C4, c4 = t - m * C4;
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const uint2 v = ((pattern >> b) & 1) ? l : h;
      if (mode == 0) dst[(size_t)m * 3 * C4 + b * C4 + c4] = v;      // [M][3C]
      else dst[(size_t)b * total + t] = v;                           // [3][M][C]
    }
  }
}

__global__ void scale_update_kernel(const float* __restrict__ flag, float* __restrict__ scaler, int interval,
                                    float growth, float backoff, float max_scale) {
  if (threadIdx.x != 0) return;
  float S = scaler[0], n = scaler[2];
  if (flag[0] != 0.f) {
    S = fmaxf(S * backoff, 1.f);
    n = 0.f;
  } else if (n + 1.f >= (float)interval) {
    S = fminf(S * growth, max_scale);
    n = 0.f;
  } else {
    n += 1.f;
  }
  scaler[0] = S;
  scaler[1] = 1.f / S;
  scaler[2] = n;
}

// ---------------------------------------------------------------- packing
// w fp32 [Co][Ci][k][k] -> fwd bf16 [Co][tap][Ci] and dgrad bf16 [Ci][8-tap][Co]
// (first layer: fwd [Co][64] with k = tap*4 + c, no dgrad).
template <int DT>
__global__ void __launch_bounds__(256) pack_conv_kernel(const float* __restrict__ w, bf16_t* __restrict__ fwd,
                                                        bf16_t* __restrict__ dgr, int Co, int Ci, int taps,
                                                        int first) {
  const size_t total = (size_t)Co * Ci * taps;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const int tap = i % taps;
    const size_t r = i / taps;
    const int ci = r % Ci;
    const int co = r / Ci;
    const unsigned short v = f2h<DT>(w[i]);
    if (first) {
      fwd[(size_t)co * 64 + tap * 4 + ci] = v;
    } else {
      fwd[((size_t)co * taps + tap) * Ci + ci] = v;
      if (dgr) dgr[((size_t)ci * taps + (taps - 1 - tap)) * Co + co] = v;
    }
  }
}

// All layers' packs in one launch: blockIdx.y = layer, descriptor rows
// {w, fwd, dgr, Co, Ci, taps, first, mode} (int64; mode 1 + si: the scale-si rows of the interleaved context
// packs, see below).  blockIdx.x = a 32(co) x
// 32(ci) x taps tile transposed through LDS, so the fp32 reads (ci, tap
// contiguous per co), the fwd-pack writes (ci contiguous per co, tap) and the
// dgrad-pack writes (co contiguous per ci, tap) are all coalesced.
template <int DT>
__global__ void __launch_bounds__(256) pack_multi_kernel(const long long* __restrict__ desc) {
  __shared__ unsigned short t[32][32 * 9 + 2];       // [co][ci*taps + tap] bf16 bits
  const long long* d = desc + (size_t)blockIdx.y * 8;
  const float* w = reinterpret_cast<const float*>(d[0]);
  bf16_t* fwd = reinterpret_cast<bf16_t*>(d[1]);
  bf16_t* dgr = reinterpret_cast<bf16_t*>(d[2]);
  const int Co = (int)d[3], Ci = (int)d[4], taps = (int)d[5], first = (int)d[6];
  const int nci = (Ci + 31) / 32, nco = (Co + 31) / 32;
  if ((int)blockIdx.x >= nci * nco) return;
  const int co0 = (blockIdx.x / nci) * 32, ci0 = (blockIdx.x % nci) * 32;
  const int cis = min(32, Ci - ci0), cos_ = min(32, Co - co0);
  const int row = cis * taps;                          // contiguous floats per co in the tile
  // whole 32 x 32 tiles of 8-aligned channel counts (every non-first layer): 16-B loads and stores, 8 channels
  // per thread (the 2-byte-store form took 81 us per step for the 41 M weights); ragged tiles: element-wise
  const bool v4 = !first && cis == 32 && cos_ == 32 && Ci % 8 == 0 && Co % 8 == 0 && (row & 3) == 0 &&
                  ((((size_t)co0 * Ci + ci0) * taps) & 3) == 0 && (((size_t)Ci * taps) & 3) == 0 &&
                  ((uintptr_t)w & 15) == 0;
  if (v4) {
    const int r4 = row >> 2;
    for (int i = threadIdx.x; i < 32 * r4; i += 256) {
      const int c = i / r4, r = (i - c * r4) * 4;
      const float4 v = *reinterpret_cast<const float4*>(w + ((size_t)(co0 + c) * Ci + ci0) * taps + r);
      t[c][r] = f2h<DT>(v.x); t[c][r + 1] = f2h<DT>(v.y); t[c][r + 2] = f2h<DT>(v.z); t[c][r + 3] = f2h<DT>(v.w);
    }
  } else {
    for (int i = threadIdx.x; i < cos_ * row; i += 256) {
      const int c = i / row, r = i - c * row;
      t[c][r] = f2h<DT>(w[((size_t)(co0 + c) * Ci + ci0) * taps + r]);
    }
  }
  __syncthreads();
  if (first) {
    for (int i = threadIdx.x; i < cos_ * row; i += 256) {
      const int c = i / row, r = i - c * row, ci = r / taps, tap = r - ci * taps;
      fwd[(size_t)(co0 + c) * 64 + tap * 4 + ci0 + ci] = t[c][r];
    }
    return;
  }
  if (d[7] > 0) {
    // linearised context module (conv_igemm.hip): W2cat[4co + si][ci] = W2_S[co][ci] (fwd, rows interleaved over
    // the four scales) and its transpose W2cat^T[ci][4co + si] (dgr); 1x1 only, si = d[7] - 1
    const int si = (int)d[7] - 1;
    for (int i = threadIdx.x; i < cos_ * cis; i += 256) {
      const int ci = i % cis, c = i / cis;
      fwd[((size_t)4 * (co0 + c) + si) * Ci + ci0 + ci] = t[c][ci];
    }
    for (int i = threadIdx.x; i < cis * cos_; i += 256) {
      const int c = i % cos_, ci = i / cos_;
      dgr[(size_t)(ci0 + ci) * 4 * Co + 4 * (co0 + c) + si] = t[c][ci];
    }
    return;
  }
  if (cis == 32 && cos_ == 32 && Ci % 8 == 0 && Co % 8 == 0 && ((uintptr_t)fwd & 15) == 0 &&
      ((uintptr_t)dgr & 15) == 0) {
    // fwd[co][tap][ci]: 8 consecutive ci per 16-B store
    for (int i = threadIdx.x; i < 32 * taps * 4; i += 256) {
      const int g = i & 3, rest = i >> 2, tap = rest % taps, c = rest / taps;
      unsigned short e[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) e[j] = t[c][(g * 8 + j) * taps + tap];
      *reinterpret_cast<uint4*>(fwd + ((size_t)(co0 + c) * taps + tap) * Ci + ci0 + g * 8) =
          make_uint4(e[0] | ((unsigned)e[1] << 16), e[2] | ((unsigned)e[3] << 16), e[4] | ((unsigned)e[5] << 16),
                     e[6] | ((unsigned)e[7] << 16));
    }
    if (dgr) {
      // dgr[ci][taps-1-tap][co]: 8 consecutive co per 16-B store
      for (int i = threadIdx.x; i < 32 * taps * 4; i += 256) {
        const int g = i & 3, rest = i >> 2, tap = rest % taps, ci = rest / taps;
        unsigned short e[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) e[j] = t[g * 8 + j][ci * taps + tap];
        *reinterpret_cast<uint4*>(dgr + ((size_t)(ci0 + ci) * taps + (taps - 1 - tap)) * Co + co0 + g * 8) =
            make_uint4(e[0] | ((unsigned)e[1] << 16), e[2] | ((unsigned)e[3] << 16), e[4] | ((unsigned)e[5] << 16),
                       e[6] | ((unsigned)e[7] << 16));
      }
    }
    return;
  }
  // fwd[co][tap][ci]: ci fastest
  for (int i = threadIdx.x; i < cos_ * taps * cis; i += 256) {
    const int ci = i % cis, rest = i / cis, tap = rest % taps, c = rest / taps;
    fwd[((size_t)(co0 + c) * taps + tap) * Ci + ci0 + ci] = t[c][ci * taps + tap];
  }
  if (dgr) {
    // dgr[ci][taps-1-tap][co]: co fastest
    for (int i = threadIdx.x; i < cis * taps * cos_; i += 256) {
      const int c = i % cos_, rest = i / cos_, tap = rest % taps, ci = rest / taps;
      dgr[((size_t)(ci0 + ci) * taps + (taps - 1 - tap)) * Co + co0 + c] = t[c][ci * taps + tap];
    }
  }
}

// [N,3,H,W] fp32 -> [N,H,W,4] bf16 (4th channel zero)
template <int DT>
__global__ void __launch_bounds__(256) img_to_nhwc4_kernel(const float* __restrict__ img, uint2* __restrict__ out,
                                                           int N, int H, int W) {
  const size_t HW = (size_t)H * W;
  const size_t total = (size_t)N * HW;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < total; i += (size_t)gridDim.x * 256) {
    const size_t n = i / HW, p = i % HW;
    const float* b = img + n * 3 * HW + p;
    out[i] = make_uint2(pack2<DT>(b[0], b[HW]), pack2<DT>(b[2 * HW], 0.f));
  }
}

static inline int grid_for(size_t n, int per = 256, int cap = 4096) {
  size_t g = (n + per - 1) / per;
  if (g > (size_t)cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace can

using namespace can;

extern "C" int can_maxpool_fwd(const void* x, void* y, void* codes, int N, int H, int W, int C, int dt,
                               void* stream) {
  if ((C & 7) || (H & 1) || (W & 1)) return -2;
  const size_t tot = (size_t)N * (H / 2) * (W / 2) * (C / 8);
  CAN_LAUNCH_DT(dt, maxpool_fwd_kernel, dim3(grid_for(tot, 256, 8192)), dim3(256), 0,
                (hipStream_t)stream, (const uint4*)x, (uint4*)y, (uint32_t*)codes, N, H, W, C / 8);
  return (int)hipGetLastError();
}

extern "C" int can_maxpool_bwd_codes(const void* codes, const void* dy, void* dx, int N, int H, int W, int C, int dt,
                                     void* stream) {
  if ((C & 7) || (H & 1) || (W & 1)) return -2;
  const size_t tot = (size_t)N * (H / 2) * (W / 2) * (C / 8);
  CAN_LAUNCH_DT(dt, maxpool_bwd_codes_kernel, dim3(grid_for(tot, 256, 8192)), dim3(256), 0,
                (hipStream_t)stream, (const uint32_t*)codes, (const uint4*)dy, (uint4*)dx, N, H, W, C / 8);
  return (int)hipGetLastError();
}

extern "C" int can_maxpool_bwd_relu(const void* x, const void* dy, void* dx, int N, int H, int W, int C, int dt,
                                    void* stream) {
  if ((C & 7) || (H & 1) || (W & 1)) return -2;
  const size_t tot = (size_t)N * (H / 2) * (W / 2) * (C / 8);
  CAN_LAUNCH_DT(dt, maxpool_bwd_relu_kernel, dim3(grid_for(tot, 256, 8192)), dim3(256), 0,
                (hipStream_t)stream, (const uint4*)x, (const uint4*)dy, (uint4*)dx, N, H, W,
                C / 8);
  return (int)hipGetLastError();
}

extern "C" int can_head_fwd(const void* y, const float* w, const float* b, float* et, int P, int dt, void* stream) {
  CAN_LAUNCH_DT(dt, head_fwd_kernel, dim3(grid_for((size_t)P * 8, 256, 2048)), dim3(256),
                0, (hipStream_t)stream, (const uint4*)y, w, b, et, P);
  return (int)hipGetLastError();
}

extern "C" int can_head_train(const void* y, const float* w, const float* b, const float* gt, float* et, void* dy,
                              float* part, int nblk, float* dw, float* db, float* loss, int P, float gscale,
                              float beta, const float* lscale, float* nonfinite, int dt, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dt == DT_F16)
    hipLaunchKernelGGL(head_train_kernel<DT_F16>, dim3(nblk), dim3(256), 0, s, (const uint4*)y, w, b, gt, et,
                       (uint4*)dy, part, P, gscale, lscale);
  else if (dt == DT_BF16)
    hipLaunchKernelGGL(head_train_kernel<DT_BF16>, dim3(nblk), dim3(256), 0, s, (const uint4*)y, w, b, gt, et,
                       (uint4*)dy, part, P, gscale, lscale);
  else
    return -20;
  hipLaunchKernelGGL(head_reduce_kernel, dim3(1), dim3(1024), 0, s, part, nblk, dw, db, loss, beta, nonfinite);
  return (int)hipGetLastError();
}

extern "C" int can_sgd_momentum(float* p, float* buf, const float* g, size_t n, float lr, float momentum,
                                float gscale, int first, float* flags, const float* lr_dev, void* stream) {
  if (n & 3) return -2;
  hipLaunchKernelGGL(sgd_momentum_kernel, dim3(grid_for(n / 4, 256, 4096)), dim3(256), 0, (hipStream_t)stream,
                     (float4*)p, (float4*)buf, (const float4*)g, n / 4, lr, momentum, gscale, first, flags, lr_dev);
  return (int)hipGetLastError();
}

extern "C" int can_grad_nonfinite(const float* g, size_t n, float* flag, void* stream) {
  if (n & 3) return -2;
  hipLaunchKernelGGL(grad_nonfinite_kernel, dim3(grid_for(n / 4, 256, 2048)), dim3(256), 0, (hipStream_t)stream,
                     (const float4*)g, n / 4, flag);
  return (int)hipGetLastError();
}

extern "C" int can_split_x3(const float* src, void* dst, long long M, int C, int stride, int mode, int pattern,
                            void* stream) {
  if (M < 1 || C < 1 || (mode == 0 && stride < 3 * C) || (mode == 1 && stride < C) || mode < 0 || mode > 1) return -2;
  const size_t total = (size_t)(mode == 0 ? 1 : 3) * (size_t)M * (size_t)stride;
  const bool dense = (mode == 0) ? stride == 3 * C : stride == C;
  if (dense && C % 4 == 0 && (size_t)M * C < (1u << 31) && ((uintptr_t)src & 15) == 0 && ((uintptr_t)dst & 7) == 0) {
    const size_t n4 = (size_t)M * (C / 4);
    hipLaunchKernelGGL(split_x3_vec_kernel, dim3(grid_for(n4, 256, 16384)), dim3(256), 0, (hipStream_t)stream,
                       (const float4*)src, (uint2*)dst, (int)M, C / 4, mode, pattern);
    return (int)hipGetLastError();
  }
  if (stride % 8 || (size_t)M * 3 >= (1u << 31) || ((uintptr_t)dst & 15)) return -3;
  hipLaunchKernelGGL(split_x3_kernel, dim3(grid_for(total / 8, 256, 16384)), dim3(256), 0, (hipStream_t)stream, src,
                     (uint4*)dst, (int)M, C, stride, mode, pattern);
  return (int)hipGetLastError();
}

extern "C" int can_scale_update(const float* flag, float* scaler, int interval, float growth, float backoff,
                                float max_scale, void* stream) {
  hipLaunchKernelGGL(scale_update_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, flag, scaler, interval, growth,
                     backoff, max_scale);
  return (int)hipGetLastError();
}

extern "C" int can_pack_conv(const float* w, void* fwd, void* dgr, int Co, int Ci, int taps, int first, int dt,
                             void* stream) {
  CAN_LAUNCH_DT(dt, pack_conv_kernel, dim3(grid_for((size_t)Co * Ci * taps, 256, 4096)),
                dim3(256), 0, (hipStream_t)stream, w, (bf16_t*)fwd, (bf16_t*)dgr, Co, Ci,
                taps, first);
  return (int)hipGetLastError();
}

extern "C" int can_img_to_nhwc4(const float* img, void* out, int N, int H, int W, int dt, void* stream) {
  CAN_LAUNCH_DT(dt, img_to_nhwc4_kernel, dim3(grid_for((size_t)N * H * W, 256, 8192)),
                dim3(256), 0, (hipStream_t)stream, img, (uint2*)out, N, H, W);
  return (int)hipGetLastError();
}

extern "C" int can_pack_multi(const long long* desc, int layers, int max_tiles, int dt, void* stream) {
  if (layers <= 0) return 0;
  // grid.x covers the largest layer's 32x32 tiles (B1: 512 -> 1024 channels = 512 tiles)
  CAN_LAUNCH_DT(dt, pack_multi_kernel, dim3(max_tiles, layers), dim3(256), 0,
                (hipStream_t)stream, desc);
  return (int)hipGetLastError();
}
