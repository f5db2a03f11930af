// Multi-scale context module of CANNet (model/CANNet.py:42-87), gfx950.
//
// Forward, per scale S in {1,2,3,6}:
//   ave_S = adaptive_avg_pool(fv, S)       -> ctx_rows(POOL) + ctx_cells(POOL)
//   A_S   = conv{S}_1(ave_S)               -> tiny [N*S*S,512]x[512,512] GEMM (host side)
//   s_S   = bilinear_up(A_S, align_corners)  (never materialised: recomputed
//                                            from the 50-cell table on the fly)
//   c_S   = s_S - fv                       -> ctx_expand (all 4 scales, one read of fv)
//   w_S   = sigmoid(conv{S}_2(c_S))        -> MFMA GEMM with sigmoid epilogue (conv_igemm)
//   fi    = sum w_S s_S / (sum w_S + 1e-12); out = cat(fv, fi)   -> ctx_fuse
// Backward:
//   ctx_bwd_e1  : dz_S = dfi (s_S - fi)/D * w_S(1-w_S),  sdir_S = dfi w_S / D
//   (host)      : dc_S = dz_S W_S2 (MFMA), dW_S2 = dz_S^T c_S (MFMA wgrad)
//   ctx_rows(BILINEAR) + ctx_cells(BILINEAR): dA_S = upsample^T (sdir_S + dc_S)
//   (host)      : dW_S1 = dA_S^T ave_S, dave_S = dA_S W_S1
//   ctx_bwd_final: dfv = (dcat_fv - sum dc_S + sum pool^T dave_S) * (fv > 0)
//
// The 50 cells of the four scales share one table layout [N][50][C]
// (cell offsets 0, 1, 5, 14); the 12 column bins of the separable row pass
// share [N][h][12][C] (bin offsets 0, 1, 3, 6).  All reductions are
// fixed-order (deterministic, no atomics).  Adaptive-pool bins follow ATen:
// start = floor(i*L/S), end = ceil((i+1)*L/S) (overlapping when L % S != 0).
#include "common.h"
#include <stdlib.h>

namespace can {

__constant__ int kScale[4] = {1, 2, 3, 6};
__constant__ int kCellOff[4] = {0, 1, 5, 14};
__constant__ int kBinOff[4] = {0, 1, 3, 6};

// adaptive-avg-pool bin [start,end) of index i at scale S over length L
__device__ __forceinline__ void pool_bin(int i, int S, int L, int& st, int& en) {
  st = (i * L) / S;
  en = ((i + 1) * L + S - 1) / S;
}
// weight of bin/cell j (scale S) for position x over length L
template <bool POOL>
__device__ __forceinline__ float axis_w(int j, int S, int x, int L) {
  if (POOL) {
    int st, en;
    pool_bin(j, S, L, st, en);
    return (x >= st && x < en) ? 1.f / (float)(en - st) : 0.f;
  } else {
    const float scale = (L > 1) ? (float)(S - 1) / (float)(L - 1) : 0.f;
    const float src = scale * (float)x;
    const int x0 = (int)src;
    const int x1 = x0 + ((x0 < S - 1) ? 1 : 0);
    const float lam = src - (float)x0;
    float wv = 0.f;
    if (j == x0) wv += 1.f - lam;
    if (j == x1) wv += lam;
    return wv;
  }
}
// bilinear taps of position x (align_corners=True)
__device__ __forceinline__ void bil(int S, int x, int L, int& x0, int& x1, float& lam) {
  const float scale = (L > 1) ? (float)(S - 1) / (float)(L - 1) : 0.f;
  const float src = scale * (float)x;
  x0 = (int)src;
  x1 = x0 + ((x0 < S - 1) ? 1 : 0);
  lam = src - (float)x0;
}

// ------------------------------------------------------------- row pass
// rowacc[n][y][bin][c] = sum_x wx(bin, x) * in_S(bin)[n][y][x][c]
// POOL: one input (fv) for all scales.  BILINEAR: per scale the sum of two
// inputs (sdir_S + dc_S), in[2*S_idx] and in[2*S_idx+1], each [P][C].
// Block = one image row (n, y) x 64 channel groups of 8; the row is split in 4
// column segments over adjacent lanes (thread = cg*4 + seg), the 4 partial
// sums are combined with lane shuffles (fixed order), and each lane stores 3
// of the 12 bins.  The 12 x w bin weights are tabulated once per block in LDS.
template <int DT, bool POOL>
__global__ void __launch_bounds__(256) ctx_rows_kernel(const uint4* __restrict__ in0, const uint4* __restrict__ sdir,
                                                       const uint4* __restrict__ dc, float* __restrict__ rowacc,
                                                       int N, int h, int w, int C) {
  extern __shared__ float wtab[];                  // [12][w]
  const int C8 = C >> 3;
  const size_t P = (size_t)N * h * w;
  const int ncgb = (C8 + 63) / 64;
  const size_t ny = blockIdx.x / ncgb;             // n*h + y
  const int cg = (blockIdx.x % ncgb) * 64 + (threadIdx.x >> 2);
  const int seg = threadIdx.x & 3;
  for (int i = threadIdx.x; i < 12 * w; i += 256) {
    const int b = i / w, x = i - b * w;
    const int si = (b >= 6) ? 3 : (b >= 3) ? 2 : (b >= 1) ? 1 : 0;
    const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
    const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
    wtab[i] = axis_w<POOL>(b - bo, S, x, w);
  }
  __syncthreads();
  float acc[12][8];
#pragma unroll
  for (int b = 0; b < 12; ++b)
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[b][k] = 0.f;
  const int xs = (w + 3) / 4;
  const int x0 = seg * xs, x1 = min(w, x0 + xs);
  if (cg < C8) {
    for (int x = x0; x < x1; ++x) {
      const size_t pix = ny * w + x;
      if (POOL) {
        float v[8];
        unpack8h<DT>(in0[pix * C8 + cg], v);
#pragma unroll
        for (int b = 0; b < 12; ++b) {
          const float wt = wtab[b * w + x];
#pragma unroll
          for (int k = 0; k < 8; ++k) acc[b][k] += wt * v[k];
        }
      } else {
#pragma unroll
        for (int si = 0; si < 4; ++si) {
          const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
          const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
          float v[8], u[8];
          unpack8h<DT>(sdir[(size_t)si * P * C8 + pix * C8 + cg], v);
          unpack8h<DT>(dc[(size_t)si * P * C8 + pix * C8 + cg], u);
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += u[k];
#pragma unroll
          for (int j = 0; j < 6; ++j) {
            if (j < S) {
              const float wt = wtab[(bo + j) * w + x];
#pragma unroll
              for (int k = 0; k < 8; ++k) acc[bo + j][k] += wt * v[k];
            }
          }
        }
      }
    }
  }
  // combine the 4 segments (lanes seg 0..3 of one channel group), fixed order
#pragma unroll
  for (int b = 0; b < 12; ++b)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float t = acc[b][k];
      t += __shfl_xor(t, 1);
      t += __shfl_xor(t, 2);
      acc[b][k] = t;
    }
  if (cg < C8) {
    float* o = rowacc + (ny * 12) * C + cg * 8;
#pragma unroll
    for (int b = 0; b < 12; ++b) {
      if (b % 4 == seg) {
        *reinterpret_cast<float4*>(o + (size_t)b * C) = make_float4(acc[b][0], acc[b][1], acc[b][2], acc[b][3]);
        *reinterpret_cast<float4*>(o + (size_t)b * C + 4) = make_float4(acc[b][4], acc[b][5], acc[b][6], acc[b][7]);
      }
    }
  }
}

// ------------------------------------------------------------- cell pass
// cells[n][cell(S,i,j)][c] = sum_y wy(i, y) * rowacc[n][y][bin(S,j)][c]
template <bool POOL>
__global__ void __launch_bounds__(256) ctx_cells_kernel(const float* __restrict__ rowacc, float* __restrict__ cells,
                                                        int N, int h, int C) {
  const size_t total = (size_t)N * 50 * C;
  for (size_t t = blockIdx.x * 256 + threadIdx.x; t < total; t += (size_t)gridDim.x * 256) {
    const int c = t % C;
    const int cell = (t / C) % 50;
    const int n = t / ((size_t)C * 50);
    int si = (cell >= 14) ? 3 : (cell >= 5) ? 2 : (cell >= 1) ? 1 : 0;
    const int S = kScale[si];
    const int local = cell - kCellOff[si];
    const int i = local / S, j = local % S;
    const int bin = kBinOff[si] + j;
    // rows y where the cell-row weight can be non-zero (a superset: axis_w is exact), then 4 independent
    // partial sums so the loads of 4 rows are in flight together (fixed order: deterministic)
    int y_lo = 0, y_hi = h;
    if (POOL) {
      pool_bin(i, S, h, y_lo, y_hi);
    } else if (S > 1) {
      y_lo = max(0, ((i - 1) * (h - 1)) / (S - 1) - 1);
      y_hi = min(h, ((i + 1) * (h - 1)) / (S - 1) + 2);
    }
    const float* col = rowacc + ((size_t)n * h * 12 + bin) * C + c;
    const size_t ystride = (size_t)12 * C;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    int y = y_lo;
    for (; y + 3 < y_hi; y += 4) {
      const float v0 = col[(size_t)y * ystride], v1 = col[(size_t)(y + 1) * ystride];
      const float v2 = col[(size_t)(y + 2) * ystride], v3 = col[(size_t)(y + 3) * ystride];
      s0 += axis_w<POOL>(i, S, y, h) * v0;
      s1 += axis_w<POOL>(i, S, y + 1, h) * v1;
      s2 += axis_w<POOL>(i, S, y + 2, h) * v2;
      s3 += axis_w<POOL>(i, S, y + 3, h) * v3;
    }
    for (; y < y_hi; ++y) s0 += axis_w<POOL>(i, S, y, h) * col[(size_t)y * ystride];
    cells[t] = (s0 + s1) + (s2 + s3);
  }
}

// value of the bilinear upsample of table T (cells of scale si) at (y, x), 8 channels
__device__ __forceinline__ void up8(const float* __restrict__ T, int n, int si, int y, int x, int h, int w, int C,
                                    int cg, float* out) {
  const int S = kScale[si];
  int y0, y1, x0, x1;
  float ly, lx;
  bil(S, y, h, y0, y1, ly);
  bil(S, x, w, x0, x1, lx);
  const float* base = T + ((size_t)n * 50 + kCellOff[si]) * C + cg * 8;
  const float w00 = (1.f - ly) * (1.f - lx), w01 = (1.f - ly) * lx, w10 = ly * (1.f - lx), w11 = ly * lx;
  const float* p00 = base + (size_t)(y0 * S + x0) * C;
  const float* p01 = base + (size_t)(y0 * S + x1) * C;
  const float* p10 = base + (size_t)(y1 * S + x0) * C;
  const float* p11 = base + (size_t)(y1 * S + x1) * C;
#pragma unroll
  for (int k = 0; k < 8; k += 4) {
    const float4 a = *reinterpret_cast<const float4*>(p00 + k), b = *reinterpret_cast<const float4*>(p01 + k);
    const float4 c = *reinterpret_cast<const float4*>(p10 + k), d = *reinterpret_cast<const float4*>(p11 + k);
    out[k + 0] = w00 * a.x + w01 * b.x + w10 * c.x + w11 * d.x;
    out[k + 1] = w00 * a.y + w01 * b.y + w10 * c.y + w11 * d.y;
    out[k + 2] = w00 * a.z + w01 * b.z + w10 * c.z + w11 * d.z;
    out[k + 3] = w00 * a.w + w01 * b.w + w10 * c.w + w11 * d.w;
  }
}

// ---------------------------------------------------------------------------
// Pixel-wise kernels.  Thread = (image row n*h+y, 8-channel group, one of 4
// column segments); a wave covers 64 channel groups of the same pixels
// (coalesced 1-KiB rows).  The row's y-interpolated cell values of all 12 bins
// (RowTab) are built once per thread in registers and reused along the run of
// pixels, so the bilinear upsample costs FMAs, not table reads.
// ---------------------------------------------------------------------------
struct RowTab {
  float v[12][8];
};

// R[bin] = y-bilinear mix of the table T at row y (bins of scale S = cells (i, j), j < S)
__device__ __forceinline__ void rowtab_bilinear(const float* __restrict__ T, int n, int y, int h, int C, int cg,
                                                RowTab& R) {
#pragma unroll
  for (int si = 0; si < 4; ++si) {
    const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
    const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
    const int co = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 5 : 14;
    int y0, y1;
    float ly;
    bil(S, y, h, y0, y1, ly);
    const float* base = T + ((size_t)n * 50 + co) * C + cg * 8;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      if (j < S) {
        const float* p0 = base + (size_t)(y0 * S + j) * C;
        const float* p1 = base + (size_t)(y1 * S + j) * C;
#pragma unroll
        for (int k = 0; k < 8; k += 4) {
          const float4 a = *reinterpret_cast<const float4*>(p0 + k), b = *reinterpret_cast<const float4*>(p1 + k);
          R.v[bo + j][k + 0] = (1.f - ly) * a.x + ly * b.x;
          R.v[bo + j][k + 1] = (1.f - ly) * a.y + ly * b.y;
          R.v[bo + j][k + 2] = (1.f - ly) * a.z + ly * b.z;
          R.v[bo + j][k + 3] = (1.f - ly) * a.w + ly * b.w;
        }
      }
    }
  }
}

// u = x-bilinear of the row table, scale si, column x
template <int SI>
__device__ __forceinline__ void up_row(const RowTab& R, int x, int w, float* u) {
  constexpr int S = (SI == 0) ? 1 : (SI == 1) ? 2 : (SI == 2) ? 3 : 6;
  constexpr int BO = (SI == 0) ? 0 : (SI == 1) ? 1 : (SI == 2) ? 3 : 6;
  int x0, x1;
  float lx;
  bil(S, x, w, x0, x1, lx);
#pragma unroll
  for (int k = 0; k < 8; ++k) u[k] = 0.f;
#pragma unroll
  for (int j = 0; j < S; ++j) {
    const float wj = ((j == x0) ? 1.f - lx : 0.f) + ((j == x1) ? lx : 0.f);
#pragma unroll
    for (int k = 0; k < 8; ++k) u[k] += wj * R.v[BO + j][k];
  }
}

template <typename F>
__device__ __forceinline__ void up_all(const RowTab& R, int x, int w, F&& f) {
  float u[8];
  up_row<0>(R, x, w, u); f(0, u);
  up_row<1>(R, x, w, u); f(1, u);
  up_row<2>(R, x, w, u); f(2, u);
  up_row<3>(R, x, w, u); f(3, u);
}

struct RowRun {
  size_t ny;   // n*h + y
  int n, y, cg, x0, x1;
  bool ok;
};
__device__ __forceinline__ RowRun row_run(int h, int w, int C8) {
  RowRun r;
  const int ncgb = (C8 + 63) / 64;
  const int seg = blockIdx.x & 1;
  const size_t rest = blockIdx.x >> 1;
  r.ny = rest / ncgb;
  r.cg = (int)(rest % ncgb) * 64 + (threadIdx.x & 63);
  // 256 threads = 4 waves: wave = sub-segment of the block's column segment
  const int xs = (w + 7) / 8;                      // 8 runs per row (2 blocks x 4 waves)
  const int run = seg * 4 + (threadIdx.x >> 6);
  r.x0 = run * xs;
  r.x1 = min(w, r.x0 + xs);
  r.n = (int)(r.ny / h);
  r.y = (int)(r.ny - (size_t)r.n * h);
  r.ok = r.cg < C8;
  return r;
}

// c_S = up_S - fv for the 4 scales: cs[si][P][C] bf16
template <int DT>
__global__ void __launch_bounds__(256) ctx_expand_kernel(const uint4* __restrict__ fv, const float* __restrict__ T,
                                                         uint4* __restrict__ cs, int N, int h, int w, int C) {
  const int C8 = C >> 3;
  const size_t total = (size_t)N * h * w * C8;
  const RowRun r = row_run(h, w, C8);
  if (!r.ok) return;
  RowTab R;
  rowtab_bilinear(T, r.n, r.y, h, C, r.cg, R);
  for (int x = r.x0; x < r.x1; ++x) {
    const size_t t = (r.ny * w + x) * C8 + r.cg;
    float f[8];
    unpack8h<DT>(fv[t], f);
    up_all(R, x, w, [&](int si, float* u) {
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] -= f[k];
      cs[(size_t)si * total + t] = pack8h<DT>(u);
    });
  }
}

// cat[p] = [fv | fi],  fi = sum w_S s_S / (sum w_S + 1e-12)
template <int DT>
__global__ void __launch_bounds__(256) ctx_fuse_kernel(const uint4* __restrict__ fv, const uint4* __restrict__ ws,
                                                       const float* __restrict__ T, uint4* __restrict__ cat, int N,
                                                       int h, int w, int C) {
  const int C8 = C >> 3;
  const size_t total = (size_t)N * h * w * C8;
  const RowRun r = row_run(h, w, C8);
  if (!r.ok) return;
  RowTab R;
  rowtab_bilinear(T, r.n, r.y, h, C, r.cg, R);
  for (int x = r.x0; x < r.x1; ++x) {
    const size_t p = r.ny * w + x;
    const size_t t = p * C8 + r.cg;
    float num[8], den[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { num[k] = 0.f; den[k] = 0.f; }
    up_all(R, x, w, [&](int si, float* u) {
      float wv[8];
      unpack8h<DT>(ws[(size_t)si * total + t], wv);
#pragma unroll
      for (int k = 0; k < 8; ++k) { num[k] += wv[k] * u[k]; den[k] += wv[k]; }
    });
#pragma unroll
    for (int k = 0; k < 8; ++k) num[k] = num[k] / (den[k] + 1e-12f);
    cat[p * 2 * C8 + r.cg] = fv[t];
    cat[p * 2 * C8 + C8 + r.cg] = pack8h<DT>(num);
  }
}

// backward elementwise: dz_S and sdir_S for the 4 scales
template <int DT>
__global__ void __launch_bounds__(256) ctx_bwd_e1_kernel(const uint4* __restrict__ dcat, const uint4* __restrict__ ws,
                                                         const float* __restrict__ T, uint4* __restrict__ dz,
                                                         uint4* __restrict__ sdir, int N, int h, int w, int C) {
  const int C8 = C >> 3;
  const size_t total = (size_t)N * h * w * C8;
  const RowRun r = row_run(h, w, C8);
  if (!r.ok) return;
  RowTab R;
  rowtab_bilinear(T, r.n, r.y, h, C, r.cg, R);
  for (int x = r.x0; x < r.x1; ++x) {
    const size_t p = r.ny * w + x;
    const size_t t = p * C8 + r.cg;
    float s[4][8], wv[4][8], num[8], den[8], dfi[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) { num[k] = 0.f; den[k] = 0.f; }
    up_all(R, x, w, [&](int si, float* u) {
      unpack8h<DT>(ws[(size_t)si * total + t], wv[si]);
#pragma unroll
      for (int k = 0; k < 8; ++k) { s[si][k] = u[k]; num[k] += wv[si][k] * u[k]; den[k] += wv[si][k]; }
    });
    unpack8h<DT>(dcat[p * 2 * C8 + C8 + r.cg], dfi);
#pragma unroll
    for (int k = 0; k < 8; ++k) { den[k] += 1e-12f; num[k] = num[k] / den[k]; }   // num := fi
#pragma unroll
    for (int si = 0; si < 4; ++si) {
      float a[8], b[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float g = dfi[k] / den[k];
        const float dws = g * (s[si][k] - num[k]);
        a[k] = dws * wv[si][k] * (1.f - wv[si][k]);
        b[k] = g * wv[si][k];
      }
      dz[(size_t)si * total + t] = pack8h<DT>(a);
      sdir[(size_t)si * total + t] = pack8h<DT>(b);
    }
  }
}

// dfv = (dcat_fv - sum_S dc_S + sum_S pool^T(dave_S)) * (fv > 0)
// pool^T: the row's pooled-cell gradients (bins containing y, divided by the
// bin height) are summed once per thread into a RowTab; per column the bins
// containing x contribute / bin width.
template <int DT>
__global__ void __launch_bounds__(256) ctx_bwd_final_kernel(const uint4* __restrict__ dcat,
                                                            const uint4* __restrict__ dc, const float* __restrict__ dave,
                                                            const uint4* __restrict__ fv, uint4* __restrict__ dfv,
                                                            int N, int h, int w, int C) {
  const int C8 = C >> 3;
  const size_t total = (size_t)N * h * w * C8;
  const RowRun r = row_run(h, w, C8);
  if (!r.ok) return;
  RowTab R;
  int xs_[12], xe_[12];
#pragma unroll
  for (int si = 0; si < 4; ++si) {
    const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
    const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
    const int co = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 5 : 14;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      if (j < S) {
        int xs, xe;
        pool_bin(j, S, w, xs, xe);
        xs_[bo + j] = xs;
        xe_[bo + j] = xe;
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        for (int i = 0; i < S; ++i) {
          int ys, ye;
          pool_bin(i, S, h, ys, ye);
          if (r.y < ys || r.y >= ye) continue;
          const float inv = 1.f / (float)((ye - ys) * (xe - xs));
          const float* d = dave + ((size_t)r.n * 50 + co + i * S + j) * C + r.cg * 8;
          const float4 a = *reinterpret_cast<const float4*>(d), b = *reinterpret_cast<const float4*>(d + 4);
          acc[0] += a.x * inv; acc[1] += a.y * inv; acc[2] += a.z * inv; acc[3] += a.w * inv;
          acc[4] += b.x * inv; acc[5] += b.y * inv; acc[6] += b.z * inv; acc[7] += b.w * inv;
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) R.v[bo + j][k] = acc[k];
      }
    }
  }
  for (int x = r.x0; x < r.x1; ++x) {
    const size_t p = r.ny * w + x;
    const size_t t = p * C8 + r.cg;
    float g[8], u[8];
    unpack8h<DT>(dcat[p * 2 * C8 + r.cg], g);
#pragma unroll
    for (int si = 0; si < 4; ++si) {
      unpack8h<DT>(dc[(size_t)si * total + t], u);
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] -= u[k];
    }
#pragma unroll
    for (int b = 0; b < 12; ++b) {
      const float m = (x >= xs_[b] && x < xe_[b]) ? 1.f : 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] += m * R.v[b][k];
    }
    float f[8];
    unpack8h<DT>(fv[t], f);
#pragma unroll
    for (int k = 0; k < 8; ++k) g[k] = (f[k] > 0.f) ? g[k] : 0.f;
    dfv[t] = pack8h<DT>(g);
  }
}


// ---------------------------------------------------------------------------
// Backward of the linearised context module (conv_igemm.hip, EPI_CTXF: z_S = up(t_S) - G_S,
// w_S = sigmoid(z_S), fi = sum_S w_S s_S / D, D = sum_S w_S + 1e-12, s_S = up(u_S)).  Per pixel and channel
// from dfi = dcat[:, C:] and the saved w (fi and s_S are recomputed in fp32 from w and the u table):
//   g = dfi / D,  dz_S = g (s_S - fi) w_S (1 - w_S),  ds_S = g w_S
//   dG = -dz  -> dg [P][4C] (interleaved like w; the operand of the data / weight gradient GEMMs)
//   up^T(dz_S) and up^T(ds_S) along x -> row partials rowacc[2][N*h][12][C] (y pass: ctx_cells_kernel)
// Block = one image row x 128 channels; thread = (x segment, channel pair): a wave reads 64 consecutive
// channel pairs of one pixel (256-B dfi, 1-KiB w / dg rows); the 4 segments of a row are summed through LDS
// in a fixed order (deterministic).
template <int DT>
__global__ void __launch_bounds__(256) ctx_bwd_lin_kernel(const uint32_t* __restrict__ dcat,
                                                          const uint4* __restrict__ wts, const float* __restrict__ U,
                                                          uint4* __restrict__ dg, float* __restrict__ rowacc, int N,
                                                          int h, int w, int C) {
  __shared__ float red[4][64][49];                 // [segment][pair][12 bins x 2 tensors x 2 channels] (+1 pad)
  const int ncb = C / 128;
  const size_t ny = blockIdx.x / ncb;              // n*h + y
  const int cbase = (blockIdx.x % ncb) * 128;
  const int seg = threadIdx.x >> 6, cp = threadIdx.x & 63;
  const int c = cbase + 2 * cp;
  const int n = (int)(ny / h), y = (int)(ny - (size_t)n * h);
  // y-interpolated u rows of the 12 column bins, this thread's two channels
  float R[12][2];
#pragma unroll
  for (int si = 0; si < 4; ++si) {
    const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
    const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
    const int co = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 5 : 14;
    int y0, y1;
    float ly;
    bil(S, y, h, y0, y1, ly);
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      if (j < S) {
        const float2 a = *reinterpret_cast<const float2*>(U + ((size_t)n * 50 + co + y0 * S + j) * C + c);
        const float2 b = *reinterpret_cast<const float2*>(U + ((size_t)n * 50 + co + y1 * S + j) * C + c);
        R[bo + j][0] = (1.f - ly) * a.x + ly * b.x;
        R[bo + j][1] = (1.f - ly) * a.y + ly * b.y;
      }
    }
  }
  float aT[12][2], aU[12][2];
#pragma unroll
  for (int b = 0; b < 12; ++b) { aT[b][0] = aT[b][1] = aU[b][0] = aU[b][1] = 0.f; }
  const int xs = (w + 3) / 4;
  const int x0 = seg * xs, x1 = min(w, x0 + xs);
  const int C2 = C >> 1;                            // dcat words (2 channels) per C
  for (int x = x0; x < x1; ++x) {
    const size_t p = ny * w + x;
    const uint32_t dw = dcat[p * C + C2 + (c >> 1)];          // dcat row = 2C elements = C words; fi half
    const uint4 wq = wts[(p * 4 * C + 4 * c) >> 3];
    float wv[8];
    unpack8h<DT>(wq, wv);                                     // [ch0: S0..S3, ch1: S0..S3]
    const float dfi[2] = {h2f<DT>((unsigned short)(dw & 0xffffu)), h2f<DT>((unsigned short)(dw >> 16))};
    // x weights of the 12 bins
    float wx[12];
#pragma unroll
    for (int si = 0; si < 4; ++si) {
      const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
      const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
      int xa, xb;
      float lx;
      bil(S, x, w, xa, xb, lx);
#pragma unroll
      for (int j = 0; j < 6; ++j)
        if (j < S) wx[bo + j] = ((j == xa) ? 1.f - lx : 0.f) + ((j == xb) ? lx : 0.f);
    }
    float o[8];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      float sS[4];
      float num = 0.f, den = 0.f;
#pragma unroll
      for (int si = 0; si < 4; ++si) {
        const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
        const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
        float v = 0.f;
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (j < S) v += wx[bo + j] * R[bo + j][k];
        sS[si] = v;
        const float ws = wv[4 * k + si];
        num += ws * v;
        den += ws;
      }
      const float rden = __builtin_amdgcn_rcpf(den + 1e-12f);     // v_rcp_f32 (1 ulp)
      const float fi = num * rden;
      const float g = dfi[k] * rden;
#pragma unroll
      for (int si = 0; si < 4; ++si) {
        const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
        const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
        const float ws = wv[4 * k + si];
        const float dz = g * (sS[si] - fi) * ws * (1.f - ws);
        const float ds = g * ws;
        o[4 * k + si] = -dz;
#pragma unroll
        for (int j = 0; j < 6; ++j)
          if (j < S) {
            aT[bo + j][k] += wx[bo + j] * dz;
            aU[bo + j][k] += wx[bo + j] * ds;
          }
      }
    }
    dg[(p * 4 * C + 4 * c) >> 3] = pack8h<DT>(o);
  }
  float* rr = &red[seg][cp][0];
#pragma unroll
  for (int b = 0; b < 12; ++b) {
    rr[b * 4 + 0] = aT[b][0]; rr[b * 4 + 1] = aT[b][1];
    rr[b * 4 + 2] = aU[b][0]; rr[b * 4 + 3] = aU[b][1];
  }
  __syncthreads();
  // 256 threads store 64 pairs x 12 bins x 2 tensors: thread -> (pair, 3 bins)
  const size_t P_ = (size_t)N * h;
  for (int e = threadIdx.x; e < 64 * 12; e += 256) {
    const int pr = e & 63, b = e >> 6;
    float t0 = 0.f, t1 = 0.f, u0 = 0.f, u1 = 0.f;
#pragma unroll
    for (int sg = 0; sg < 4; ++sg) {
      t0 += red[sg][pr][b * 4 + 0]; t1 += red[sg][pr][b * 4 + 1];
      u0 += red[sg][pr][b * 4 + 2]; u1 += red[sg][pr][b * 4 + 3];
    }
    const size_t o0 = (ny * 12 + b) * C + cbase + 2 * pr;
    *reinterpret_cast<float2*>(rowacc + o0) = make_float2(t0, t1);
    *reinterpret_cast<float2*>(rowacc + P_ * 12 * C + o0) = make_float2(u0, u1);
  }
}

// dW2_S[c][k] = beta * dW2_S[c][k] + tmp[4c + si][k]: the interleaved rows of the linearised weight gradient
// (W2cat = rows 4c + si) back into the four conv{S}_2 weights
__global__ void __launch_bounds__(256) ctx_w2_scatter_kernel(const float4* __restrict__ tmp, float* d0, float* d1,
                                                             float* d2, float* d3, int C, float beta) {
  const int C4 = C >> 2;
  const size_t total = (size_t)4 * C * C4;
  for (size_t t = blockIdx.x * 256 + threadIdx.x; t < total; t += (size_t)gridDim.x * 256) {
    const int k4 = (int)(t % C4);
    const size_t row = t / C4;                      // 4c + si
    const int si = (int)(row & 3), c = (int)(row >> 2);
    float* d = (si == 0) ? d0 : (si == 1) ? d1 : (si == 2) ? d2 : d3;
    float4* o = reinterpret_cast<float4*>(d + (size_t)c * C) + k4;
    float4 v = tmp[t];
    if (beta != 0.f) {
      const float4 q = *o;
      v.x += beta * q.x; v.y += beta * q.y; v.z += beta * q.z; v.w += beta * q.w;
    }
    *o = v;
  }
}

// ---------------------------------------------------------------------------
// conv{S}_1 (1x1, 512->512, no bias) on the pooled S x S grids, all four
// scales in ONE launch (blockIdx.z = scale), fp32 (model/CANNet.py:43,52,61,72;
// SURVEY §2.5 X2).  Cells are [N][50][C] fp32 (scale S at cell offset
// {0,1,5,14}, S*S cells per image); weights are the fp32 masters [C][C]
// (out, in).  Three GEMM shapes, out[m][n] = sum_k X(m,k) Y(k,n):
//   MODE 0 forward        table[r][o] = sum_k ave[r][k] * W[o][k]       (m = cell row r)
//   MODE 1 data gradient  dave[r][i]  = sum_o dA[r][o]  * W[o][i]
//   MODE 2 weight grad    dW[o][i]    = sum_r dA[r][o]  * ave[r][i]     (k = cell row r)
// 32 x 64 output tiles, 256 threads x (2 x 4) outputs, K tiles of 32 staged in
// LDS; fixed summation order (deterministic).  M <= 288 rows at batch 8: the
// whole context GEMM work is ~0.2 GFLOP, so this is a launch-count kernel
// (replaces 12 hipBLASLt GEMMs + 4 copies per step), not an MFMA one.
struct CtxGemmArgs {
  const float* x;        // MODE 0/1: cells (ave / dA); MODE 2: dA
  const float* y;        // MODE 2: ave
  const float* w[4];     // MODE 0/1: W1 per scale
  float* out;            // MODE 0/1: cells (table / dave)
  float* gw[4];          // MODE 2: dW1 per scale
  int N, C;
  float beta, scale;
  const float* dscale;
};

__device__ __forceinline__ int ctx_cell_row(int r, int k2, int off) { return (r / k2) * 50 + off + (r % k2); }

// One K tile (32 deep) of X (32 x 32) and Y (32 x 64) in registers, 16-B loads: every load of the tile is
// issued before any is consumed (the first version stored each element to LDS right after its load, which
// serialised ~12 memory latencies per K step).
template <int MODE>
struct CtxTile {
  float4 x, y0, y1;
};

template <int MODE>
__device__ __forceinline__ CtxTile<MODE> ctx_load(const CtxGemmArgs& a, const float* W, int m0, int n0, int k0,
                                                  int M, int K, int k2, int off, int tid) {
  const int C = a.C;
  const float4 z = make_float4(0.f, 0.f, 0.f, 0.f);
  CtxTile<MODE> t;
  if (MODE == 2) {
    // X(m,k) = dA[row(k)][m]: m contiguous; tile element (k = tid/8, m4 = tid%8)
    const int k = k0 + (tid >> 3), m = m0 + (tid & 7) * 4;
    t.x = (k < K) ? *reinterpret_cast<const float4*>(a.x + (size_t)ctx_cell_row(k, k2, off) * C + m) : z;
  } else {
    // X(m,k) = cells[row(m)][k]: k contiguous; (m = tid/8, k4 = tid%8)
    const int m = m0 + (tid >> 3), k = k0 + (tid & 7) * 4;
    t.x = (m < M) ? *reinterpret_cast<const float4*>(a.x + (size_t)ctx_cell_row(m, k2, off) * C + k) : z;
  }
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = tid + 256 * i;
    float4 v;
    if (MODE == 0) {
      // Y(k,n) = W[n][k]: k contiguous; (n = e/8, k4 = e%8)
      const int n = n0 + (e >> 3), k = k0 + (e & 7) * 4;
      v = *reinterpret_cast<const float4*>(W + (size_t)n * C + k);
    } else {
      // Y(k,n) = W[k][n] (MODE 1) / ave[row(k)][n] (MODE 2): n contiguous; (k = e/16, n4 = e%16)
      const int k = k0 + (e >> 4), n = n0 + (e & 15) * 4;
      if (MODE == 1) v = *reinterpret_cast<const float4*>(W + (size_t)k * C + n);
      else v = (k < K) ? *reinterpret_cast<const float4*>(a.y + (size_t)ctx_cell_row(k, k2, off) * C + n) : z;
    }
    if (i == 0) t.y0 = v; else t.y1 = v;
  }
  return t;
}

template <int MODE>
__global__ void __launch_bounds__(256) ctx_gemm_kernel(CtxGemmArgs a) {
  constexpr int TM = 32, TN = 64, TK = 32;
  __shared__ __attribute__((aligned(16))) float Xs[TK][TM + 4];
  __shared__ __attribute__((aligned(16))) float Ys[TK][TN + 4];
  const int si = blockIdx.z;
  const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
  const int off = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 5 : 14;
  const int k2 = S * S, R = a.N * k2, C = a.C;
  const int M = (MODE == 2) ? C : R, K = (MODE == 2) ? R : C;
  const int m0 = blockIdx.y * TM, n0 = blockIdx.x * TN;
  if (m0 >= M) return;
  const float* W = a.w[si];
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  float acc[2][4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
  CtxTile<MODE> cur = ctx_load<MODE>(a, W, m0, n0, 0, M, K, k2, off, tid);
  for (int k0 = 0; k0 < K; k0 += TK) {
    // registers -> LDS
    if (MODE == 2) {
      *reinterpret_cast<float4*>(&Xs[tid >> 3][(tid & 7) * 4]) = cur.x;
    } else {
      const int mm = tid >> 3, kk = (tid & 7) * 4;
      Xs[kk][mm] = cur.x.x; Xs[kk + 1][mm] = cur.x.y; Xs[kk + 2][mm] = cur.x.z; Xs[kk + 3][mm] = cur.x.w;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + 256 * i;
      const float4 v = i ? cur.y1 : cur.y0;
      if (MODE == 0) {
        const int nn = e >> 3, kk = (e & 7) * 4;
        Ys[kk][nn] = v.x; Ys[kk + 1][nn] = v.y; Ys[kk + 2][nn] = v.z; Ys[kk + 3][nn] = v.w;
      } else {
        *reinterpret_cast<float4*>(&Ys[e >> 4][(e & 15) * 4]) = v;
      }
    }
    __syncthreads();
    if (k0 + TK < K) cur = ctx_load<MODE>(a, W, m0, n0, k0 + TK, M, K, k2, off, tid);   // next tile in flight
#pragma unroll 8
    for (int kk = 0; kk < TK; ++kk) {
      const float x0 = Xs[kk][ty * 2], x1 = Xs[kk][ty * 2 + 1];
      const float4 y4 = *reinterpret_cast<const float4*>(&Ys[kk][tx * 4]);
      acc[0][0] = fmaf(x0, y4.x, acc[0][0]); acc[0][1] = fmaf(x0, y4.y, acc[0][1]);
      acc[0][2] = fmaf(x0, y4.z, acc[0][2]); acc[0][3] = fmaf(x0, y4.w, acc[0][3]);
      acc[1][0] = fmaf(x1, y4.x, acc[1][0]); acc[1][1] = fmaf(x1, y4.y, acc[1][1]);
      acc[1][2] = fmaf(x1, y4.z, acc[1][2]); acc[1][3] = fmaf(x1, y4.w, acc[1][3]);
    }
    __syncthreads();
  }
  const float sc = a.scale * ((a.dscale != nullptr) ? a.dscale[0] : 1.f);
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + ty * 2 + i;
    if (m >= M) continue;
    const int n = n0 + tx * 4;
    if (MODE == 2) {
      float* g = a.gw[si] + (size_t)m * C + n;
      float4 o = make_float4(acc[i][0] * sc, acc[i][1] * sc, acc[i][2] * sc, acc[i][3] * sc);
      if (a.beta != 0.f) {
        const float4 p = *reinterpret_cast<const float4*>(g);
        o.x += a.beta * p.x; o.y += a.beta * p.y; o.z += a.beta * p.z; o.w += a.beta * p.w;
      }
      *reinterpret_cast<float4*>(g) = o;
    } else {
      float* o = a.out + (size_t)ctx_cell_row(m, k2, off) * C + n;
      float4 v = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
      if (a.beta != 0.f) {
        const float4 p = *reinterpret_cast<const float4*>(o);
        v.x += a.beta * p.x; v.y += a.beta * p.y; v.z += a.beta * p.z; v.w += a.beta * p.w;
      }
      *reinterpret_cast<float4*>(o) = v;
    }
  }
}

// ctx_mm_kernel: the same three cell GEMMs on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: f32 in, exact f32
// FMA chain).  These GEMMs are latency-bound, not FLOP-bound (<= 0.3 GFLOP per launch): the 32 x 64-tile kernel
// above ran ~1 wave per SIMD through 16 dependent K steps (34-47 us per launch).  Here a block of 8 waves owns one
// 16 x 16 output tile of one scale and splits K 8 ways (each wave <= 16 MFMAs over 4-deep K chunks whose operands
// are all loaded before the first MFMA); the 8 partial tiles are summed in LDS in a fixed order (deterministic).
// The K order inside a 16-chunk is permuted (step s, lane group q -> k = 16c + 4q + s) identically for A and B, so
// K-contiguous operands load as one float4 per lane per chunk.
template <int MODE>
__global__ void __launch_bounds__(512) ctx_mm_kernel(CtxGemmArgs a) {
  __shared__ f32x4 red[8][64];
  const int si = blockIdx.z;
  const int S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
  const int off = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 5 : 14;
  const int k2 = S * S, R = a.N * k2, C = a.C;
  const int M = (MODE == 2) ? C : R, K = (MODE == 2) ? R : C;
  const int m0 = blockIdx.y * 16, n0 = blockIdx.x * 16;
  if (m0 >= M) return;
  const float* W = a.w[si];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i = lane & 15, q = lane >> 4;
  // this wave's K range, whole 16-chunks
  const int nch = (K + 15) / 16;
  const int cpw = (nch + 7) / 8;
  const int c0 = wave * cpw, c1 = min(nch, c0 + cpw);
  constexpr int MAXC = 4;                           // K <= 8 * 4 * 16 = 512 (C = 512; R <= 8 * 36 = 288)
  float av[MAXC][4], bv[MAXC][4];
#pragma unroll
  for (int cc = 0; cc < MAXC; ++cc) {
    const int ch = c0 + cc;
#pragma unroll
    for (int s = 0; s < 4; ++s) { av[cc][s] = 0.f; bv[cc][s] = 0.f; }
    if (ch >= c1) continue;
    const int kb = ch * 16 + 4 * q;                 // this lane's 4 k values: kb .. kb + 3
    const int m = m0 + i, n = n0 + i;
    if (MODE == 0) {
      // A(m,k) = cells[row(m)][k], B(k,n) = W[n][k]: both k-contiguous
      if (m < M) {
        const float4 v = *reinterpret_cast<const float4*>(a.x + (size_t)ctx_cell_row(m, k2, off) * C + kb);
        av[cc][0] = v.x; av[cc][1] = v.y; av[cc][2] = v.z; av[cc][3] = v.w;
      }
      const float4 v = *reinterpret_cast<const float4*>(W + (size_t)n * C + kb);
      bv[cc][0] = v.x; bv[cc][1] = v.y; bv[cc][2] = v.z; bv[cc][3] = v.w;
    } else if (MODE == 1) {
      // A(m,k) = cells[row(m)][k] (k-contiguous), B(k,n) = W[k][n]
      if (m < M) {
        const float4 v = *reinterpret_cast<const float4*>(a.x + (size_t)ctx_cell_row(m, k2, off) * C + kb);
        av[cc][0] = v.x; av[cc][1] = v.y; av[cc][2] = v.z; av[cc][3] = v.w;
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) bv[cc][s] = W[(size_t)(kb + s) * C + n];
    } else {
      // A(m,k) = dA[row(k)][m], B(k,n) = ave[row(k)][n] (k = cell row r < R)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = kb + s;
        if (k < K) {
          const size_t rr = (size_t)ctx_cell_row(k, k2, off) * C;
          av[cc][s] = a.x[rr + m];
          bv[cc][s] = a.y[rr + n];
        }
      }
    }
  }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int cc = 0; cc < MAXC; ++cc)
#pragma unroll
    for (int s = 0; s < 4; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[cc][s], bv[cc][s], acc, 0, 0, 0);
  red[wave][lane] = acc;
  __syncthreads();
  if (wave != 0) return;
  f32x4 t = red[0][lane];
#pragma unroll
  for (int w8 = 1; w8 < 8; ++w8) t += red[w8][lane];
  // D layout: column n0 + (lane & 15), rows m0 + 4 * (lane >> 4) + v
  const int n = n0 + i;
  const float sc = (MODE == 2) ? a.scale * ((a.dscale != nullptr) ? a.dscale[0] : 1.f) : 1.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int m = m0 + 4 * q + v;
    if (m >= M) continue;
    float* o = (MODE == 2) ? a.gw[si] + (size_t)m * C + n : a.out + (size_t)ctx_cell_row(m, k2, off) * C + n;
    float val = t[v] * sc;
    if (a.beta != 0.f) val += a.beta * *o;
    *o = val;
  }
}

static inline int gridn(size_t n, int cap = 8192) {
  size_t g = (n + 255) / 256;
  if (g > (size_t)cap) g = cap;
  return g < 1 ? 1 : (int)g;
}

}  // namespace can

using namespace can;

// mode 0: POOL(fv -> ave cells); mode 1: BILINEAR^T(sdir+dc -> dA cells).  dt: element type of the
// 16-bit inputs (DT_BF16 = 0, DT_F16 = 1); rowacc / cells are fp32.
template <int DT>
static int ctx_reduce_impl(int mode, const void* in0, const void* sdir, const void* dc, float* rowacc, float* cells,
                           int N, int h, int w, int C, hipStream_t s) {
  const int nb = N * h * ((C / 8 + 63) / 64);
  const size_t lds = (size_t)12 * w * sizeof(float);
  if (mode == 0)
    hipLaunchKernelGGL((ctx_rows_kernel<DT, true>), dim3(nb), dim3(256), lds, s, (const uint4*)in0, nullptr, nullptr,
                       rowacc, N, h, w, C);
  else
    hipLaunchKernelGGL((ctx_rows_kernel<DT, false>), dim3(nb), dim3(256), lds, s, nullptr, (const uint4*)sdir,
                       (const uint4*)dc, rowacc, N, h, w, C);
  const size_t tc = (size_t)N * 50 * C;
  if (mode == 0)
    hipLaunchKernelGGL(ctx_cells_kernel<true>, dim3(gridn(tc)), dim3(256), 0, s, rowacc, cells, N, h, C);
  else
    hipLaunchKernelGGL(ctx_cells_kernel<false>, dim3(gridn(tc)), dim3(256), 0, s, rowacc, cells, N, h, C);
  return (int)hipGetLastError();
}

extern "C" int can_ctx_reduce(int mode, const void* in0, const void* sdir, const void* dc, float* rowacc, float* cells,
                              int N, int h, int w, int C, int dt, void* stream) {
  if (C & 7) return -2;
  if (w > 2048) return -3;                       // LDS bin-weight table [12][w]
  CAN_DT_DISPATCH(dt, ctx_reduce_impl<DT>(mode, in0, sdir, dc, rowacc, cells, N, h, w, C, (hipStream_t)stream));
}

static inline dim3 ctx_grid(int N, int h, int C) { return dim3(N * h * ((C / 8 + 63) / 64) * 2); }

extern "C" int can_ctx_bwd_lin(const void* dcat, const void* wts, const float* U, void* dg, float* rowacc, int N,
                               int h, int w, int C, int dt, void* stream) {
  if (C % 128) return -2;
  CAN_LAUNCH_DT(dt, ctx_bwd_lin_kernel, dim3(N * h * (C / 128)), dim3(256), 0, (hipStream_t)stream,
                (const uint32_t*)dcat, (const uint4*)wts, U, (uint4*)dg, rowacc, N, h, w, C);
  return (int)hipGetLastError();
}

// y pass of the separable bilinear adjoint only: rowacc [N][h][12][C] -> cells [N][50][C]
extern "C" int can_ctx_cells(const float* rowacc, float* cells, int N, int h, int C, void* stream) {
  const size_t tc = (size_t)N * 50 * C;
  hipLaunchKernelGGL(ctx_cells_kernel<false>, dim3(gridn(tc)), dim3(256), 0, (hipStream_t)stream, rowacc, cells, N, h,
                     C);
  return (int)hipGetLastError();
}

extern "C" int can_ctx_w2_scatter(const float* tmp, float* const* dst, int C, float beta, void* stream) {
  if (C % 4) return -2;
  const size_t total = (size_t)C * C;             // float4 items = 4C rows x C/4
  hipLaunchKernelGGL(ctx_w2_scatter_kernel, dim3(gridn(total, 2048)), dim3(256), 0, (hipStream_t)stream,
                     (const float4*)tmp, dst[0], dst[1], dst[2], dst[3], C, beta);
  return (int)hipGetLastError();
}

extern "C" int can_ctx_expand(const void* fv, const float* T, void* cs, int N, int h, int w, int C, int dt,
                              void* stream) {
  if (C & 7) return -2;
  CAN_LAUNCH_DT(dt, ctx_expand_kernel, ctx_grid(N, h, C), dim3(256), 0, (hipStream_t)stream, (const uint4*)fv, T,
                (uint4*)cs, N, h, w, C);
  return (int)hipGetLastError();
}

extern "C" int can_ctx_fuse(const void* fv, const void* ws, const float* T, void* cat, int N, int h, int w, int C,
                            int dt, void* stream) {
  if (C & 7) return -2;
  CAN_LAUNCH_DT(dt, ctx_fuse_kernel, ctx_grid(N, h, C), dim3(256), 0, (hipStream_t)stream, (const uint4*)fv,
                (const uint4*)ws, T, (uint4*)cat, N, h, w, C);
  return (int)hipGetLastError();
}

extern "C" int can_ctx_bwd_e1(const void* dcat, const void* ws, const float* T, void* dz, void* sdir, int N, int h,
                              int w, int C, int dt, void* stream) {
  if (C & 7) return -2;
  CAN_LAUNCH_DT(dt, ctx_bwd_e1_kernel, ctx_grid(N, h, C), dim3(256), 0, (hipStream_t)stream, (const uint4*)dcat,
                (const uint4*)ws, T, (uint4*)dz, (uint4*)sdir, N, h, w, C);
  return (int)hipGetLastError();
}

extern "C" int can_ctx_bwd_final(const void* dcat, const void* dc, const float* dave, const void* fv, void* dfv,
                                 int N, int h, int w, int C, int dt, void* stream) {
  if (C & 7) return -2;
  CAN_LAUNCH_DT(dt, ctx_bwd_final_kernel, ctx_grid(N, h, C), dim3(256), 0, (hipStream_t)stream, (const uint4*)dcat,
                (const uint4*)dc, dave, (const uint4*)fv, (uint4*)dfv, N, h, w, C);
  return (int)hipGetLastError();
}

// conv{S}_1 GEMMs of all four scales in one launch.  mode 0: out = table (fwd), mode 1: out = dave,
// mode 2: gw = dW1 per scale (beta: accumulate, scale/dscale: gradient scaling of the fp16 step).
extern "C" int can_ctx_gemm(int mode, const float* x, const float* y, const float* const* w, float* out,
                            float* const* gw, int N, int C, float beta, float scale, const float* dscale,
                            void* stream) {
  if (C % 64 != 0 || N < 1) return -2;   // 16-B rows, 64-column tiles
  CtxGemmArgs a{};
  a.x = x; a.y = y; a.out = out; a.N = N; a.C = C; a.beta = beta; a.scale = scale; a.dscale = dscale;
  for (int i = 0; i < 4; ++i) {
    a.w[i] = w ? w[i] : nullptr;
    a.gw[i] = gw ? gw[i] : nullptr;
  }
  const int M = (mode == 2) ? C : N * 36;
  hipStream_t s = (hipStream_t)stream;
  if (C <= 512 && N * 36 <= 512) {
    // matrix-core form (K <= 512 on both sides): 16 x 16 tiles, K split over 8 waves
    const dim3 grid(C / 16, (M + 15) / 16, 4);
    if (mode == 0) hipLaunchKernelGGL(ctx_mm_kernel<0>, grid, dim3(512), 0, s, a);
    else if (mode == 1) hipLaunchKernelGGL(ctx_mm_kernel<1>, grid, dim3(512), 0, s, a);
    else if (mode == 2) hipLaunchKernelGGL(ctx_mm_kernel<2>, grid, dim3(512), 0, s, a);
    else return -3;
    return (int)hipGetLastError();
  }
  const dim3 grid(C / 64, (M + 31) / 32, 4);
  if (mode == 0) hipLaunchKernelGGL(ctx_gemm_kernel<0>, grid, dim3(256), 0, s, a);
  else if (mode == 1) hipLaunchKernelGGL(ctx_gemm_kernel<1>, grid, dim3(256), 0, s, a);
  else if (mode == 2) hipLaunchKernelGGL(ctx_gemm_kernel<2>, grid, dim3(256), 0, s, a);
  else return -3;
  return (int)hipGetLastError();
}
