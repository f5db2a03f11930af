// MFMA weight-gradient kernel for the NHWC implicit-GEMM convolutions (gfx950).
//
// Replaces cuDNN/MIOpen's backward-filter of every nn.Conv2d in the reference
// (model/CANNet.py:14-25; SURVEY §2.5 "convolution_backward x25").
//
//   dW[co][k] = sum_m dY[m][co] * Xcol[m][k],   k = tap*Cin + ci
//   db[co]    = sum_m dY[m][co]
//
// The reduction runs over output pixels m (up to N*H*W = 6.3M at batch 8,
// 768x1024), i.e. along the OUTER (strided) dimension of both NHWC operands.
// Both tiles are staged in LDS exactly as they sit in memory ([pixel][channel]
// rows, coalesced 16-B loads, zero-filled outside the image) and the MFMA
// fragments, which need 8 consecutive PIXELS per lane, are read with the
// gfx950 hardware-transpose LDS read ds_read_b64_tr_b16 (2 reads per
// fragment).  The 8-B chunk index of each LDS row is XOR-swizzled so that the
// 32 addresses of each transposed read hit 32 distinct 8-B bank slots.
//
// Work split: block = (co tile, k tile, pixel slice).  Slices write fp32
// partial slabs ws[slice][k][co] (4 consecutive co per lane -> 16-B stores);
// wgrad_reduce sums the slabs in a fixed order (deterministic, no atomics)
// and scatters the result into the PyTorch weight layout [co][ci][kh][kw] of
// the flat fp32 gradient arena (optionally accumulating).  The bias gradient
// rides along: blocks of k-tile 0 run one extra MFMA per co tile against a
// ones operand.
//
// Wave layouts (4 waves / 256 threads):
//   <2,2,1>: 128 co x 128 k tile, 64-pixel stages, each wave 64x64 x 2 k-steps
//   <1,1,4>: 64 co x 64 k tile, 128-pixel stages, each wave a 32-pixel quarter
//            of every stage; the 4 partial tiles are summed through LDS.
#include "common.h"
#include "fastdiv.h"
#include <stdlib.h>
#include <type_traits>

namespace can {

typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;

struct WgradArgs {
  const bf16_t* dy;   // [M][Cout]
  const bf16_t* x;    // [N][H][W][Cin] (FIRST: Cin = 4)
  float* ws;          // [S][Ktot][Cout] partial slabs
  float* wsb;         // [S][Cout] bias partials (or nullptr)
  int N, H, W, Cin, Cout, ksize, dil, M;
  int Ktot, S, mslice;
};

// 8-byte-chunk swizzle of an LDS row (row bytes = 2*RW): see file header.
template <int RW>
__device__ __forceinline__ int swz8(int row, int c8) {
  if (RW == 128) return c8 ^ (((row & 3) | (((row >> 3) & 1) << 2)) << 2);
  else return c8 ^ (((((row >> 1) & 1)) | (((row >> 3) & 1) << 1)) << 2);
}

template <int DT, int WC, int WK, int WM, bool FIRST>
__global__ void __launch_bounds__(256) conv_wgrad_kernel(WgradArgs a) {
  constexpr int TCo = 64 * WC;
  constexpr int TK = 64 * WK;
  constexpr int KSUB = (WM == 1) ? 2 : 1;
  constexpr int BKM = 32 * KSUB * WM;            // pixels per stage
  constexpr int CA = TCo / 8, CB = TK / 8;        // 16-B chunks per row
  constexpr int NA = BKM * CA / 256, NB = BKM * CB / 256;
  static_assert(WC * WK * WM == 4, "4 waves");
  static_assert(NA >= 1 && NB >= 1, "");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  bf16_t* As = reinterpret_cast<bf16_t*>(smem);            // [2][BKM][TCo]
  bf16_t* Bs = As + 2 * BKM * TCo;                          // [2][BKM][TK]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wc = wave % WC, wk = (wave / WC) % WK, wm = wave / (WC * WK);

  const int nco = a.Cout / TCo, nkt = a.Ktot / TK;
  const int ntile = nco * nkt;
  const int bid = xcd_remap(blockIdx.x, ntile * a.S);
  const int tile = bid % ntile;                  // slices of one tile are spread, tiles adjacent
  const int slice = bid / ntile;
  const int cot = tile % nco, kt = tile / nco;
  const int co0 = cot * TCo;
  const int k0 = kt * TK;
  int tap = 0, ci0 = 0;
  if (!FIRST) { tap = k0 / a.Cin; ci0 = k0 - tap * a.Cin; }
  const int kh = (a.ksize == 3) ? tap / 3 : 1, kw = (a.ksize == 3) ? tap % 3 : 1;
  const int dh = (kh - 1) * a.dil, dw = (kw - 1) * a.dil;
  const bool do_bias = (a.wsb != nullptr) && (kt == 0);

  const int mbeg = slice * a.mslice;
  const int mend = min(a.M, mbeg + a.mslice);
  const int nstage = (mend > mbeg) ? (mend - mbeg + BKM - 1) / BKM : 0;
  const int HW = a.H * a.W;

  // per-thread rows (fixed offsets within a stage)
  int arow[NA], ac[NA], brow[NB], bc[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) { const int id = tid + 256 * i; arow[i] = id / CA; ac[i] = id % CA; }
#pragma unroll
  for (int i = 0; i < NB; ++i) { const int id = tid + 256 * i; brow[i] = id / CB; bc[i] = id % CB; }
  // incremental (oh, ow) of each B row
  int boh[NB], bow[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int m = mbeg + brow[i];
    const int r = m % HW;
    boh[i] = r / a.W; bow[i] = r % a.W;
  }

  uint4 ra[NA], rb[NB];
  auto load_stage = [&](int st) {
    const int m0 = mbeg + st * BKM;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int m = m0 + arow[i];
      uint4 v = make_uint4(0, 0, 0, 0);
      if (m < mend) v = *reinterpret_cast<const uint4*>(a.dy + (size_t)m * a.Cout + co0 + ac[i] * 8);
      ra[i] = v;
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int m = m0 + brow[i];
      uint4 v = make_uint4(0, 0, 0, 0);
      if (!FIRST) {
        const int ih = boh[i] + dh, iw = bow[i] + dw;
        if (m < mend && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
          v = *reinterpret_cast<const uint4*>(a.x + (size_t)(m + dh * a.W + dw) * a.Cin + ci0 + bc[i] * 8);
      } else {
        uint2 h2[2] = {make_uint2(0, 0), make_uint2(0, 0)};
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int t = bc[i] * 2 + h;
          if (t < 9 && m < mend) {
            const int ddh = (t / 3 - 1) * a.dil, ddw = (t % 3 - 1) * a.dil;
            const int ih = boh[i] + ddh, iw = bow[i] + ddw;
            if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
              h2[h] = *reinterpret_cast<const uint2*>(a.x + (size_t)(m + ddh * a.W + ddw) * 4);
          }
        }
        v = make_uint4(h2[0].x, h2[0].y, h2[1].x, h2[1].y);
      }
      rb[i] = v;
      // advance this row by BKM pixels for the next stage
      int ow = bow[i] + BKM, oh = boh[i];
      while (ow >= a.W) { ow -= a.W; ++oh; }
      while (oh >= a.H) oh -= a.H;
      bow[i] = ow; boh[i] = oh;
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      bf16_t* row = As + (buf * BKM + arow[i]) * TCo;
      *reinterpret_cast<uint4*>(row + swz8<TCo>(arow[i], ac[i] * 2) * 4) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      bf16_t* row = Bs + (buf * BKM + brow[i]) * TK;
      *reinterpret_cast<uint4*>(row + swz8<TK>(brow[i], bc[i] * 2) * 4) = rb[i];
    }
  };

  f32x4 acc[4][4];
  f32x4 accb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    accb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const frag8_t ones = ones_frag<DT>();

  // transposed fragment read: 8 consecutive pixels (rows) of one column
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  auto read_frag = [&](const bf16_t* base, int rw_is128, int prow0, int col0) -> frag8_t {
    s16x4 lo, hi;
    const int r0 = prow0 + 8 * g + q;
    const int c8 = (col0 >> 2) + p;
    if (rw_is128) {
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + r0 * 128 + swz8<128>(r0, c8) * 4));
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (r0 + 4) * 128 + swz8<128>(r0 + 4, c8) * 4));
    } else {
      lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + r0 * 64 + swz8<64>(r0, c8) * 4));
      hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (r0 + 4) * 64 + swz8<64>(r0 + 4, c8) * 4));
    }
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(frag8_t, v);
  };

  if (nstage > 0) {
    load_stage(0);
    store_stage(0);
  }
  __syncthreads();
  for (int st = 0; st < nstage; ++st) {
    const int buf = st & 1;
    if (st + 1 < nstage) load_stage(st + 1);
    const bf16_t* Ab = As + buf * BKM * TCo;
    const bf16_t* Bb = Bs + buf * BKM * TK;
#pragma unroll
    for (int kk = 0; kk < KSUB; ++kk) {
      const int prow0 = wm * (32 * KSUB) + kk * 32;
      frag8_t af[4], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) af[j] = read_frag(Ab, TCo == 128, prow0, wc * 64 + j * 16);
#pragma unroll
      for (int i = 0; i < 4; ++i) bfr[i] = read_frag(Bb, TK == 128, prow0, wk * 64 + i * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = mfma16<DT>(af[j], bfr[i], acc[j][i]);
      // bias gradient: sum over pixels = MFMA against a ones operand.  Static
      // indices only (a runtime-indexed accumulator array spills to VGPR copies).
      if (do_bias && (WM != 1 || wk == 0)) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          accb[j] = mfma16<DT>(af[j], ones, accb[j]);
      }
    }
    if (st + 1 < nstage) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue.  D layout: col = lane&15 -> k, rows (lane>>4)*4 + r -> co
  const int fr = lane & 15, fq = lane >> 4;
  float* slab = a.ws + (size_t)slice * a.Ktot * a.Cout;
  if (WM == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int k = k0 + wk * 64 + i * 16 + fr;
        const int co = co0 + wc * 64 + j * 16 + fq * 4;
        *reinterpret_cast<f32x4*>(slab + (size_t)k * a.Cout + co) = acc[j][i];
      }
    if (do_bias && wk == 0 && fr == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + wc * 64 + j * 16 + fq * 4;
        *reinterpret_cast<f32x4*>(a.wsb + (size_t)slice * a.Cout + co) = accb[j];
      }
    }
  } else {
    // sum the 4 pixel-quarter partials through LDS (staging buffers are free now)
    float* red = reinterpret_cast<float*>(smem);   // [4 waves][16 tiles][64 lanes][4]
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<f32x4*>(red + ((wave * 16 + j * 4 + i) * 64 + lane) * 4) = acc[j][i];
    float* redb = red + 4 * 16 * 64 * 4;          // [4 waves][4][64][4]
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4*>(redb + ((wave * 4 + j) * 64 + lane) * 4) = accb[j];
    }
    __syncthreads();
    // wave w reduces tiles j = w (4 i-tiles each)
    const int j = wave;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < 4; ++w) s += *reinterpret_cast<const f32x4*>(red + ((w * 16 + j * 4 + i) * 64 + lane) * 4);
      const int k = k0 + i * 16 + fr;
      const int co = co0 + j * 16 + fq * 4;
      *reinterpret_cast<f32x4*>(slab + (size_t)k * a.Cout + co) = s;
    }
    if (do_bias && fr == 0) {
      f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int w = 0; w < 4; ++w) s += *reinterpret_cast<const f32x4*>(redb + ((w * 4 + j) * 64 + lane) * 4);
      const int co = co0 + j * 16 + fq * 4;
      *reinterpret_cast<f32x4*>(a.wsb + (size_t)slice * a.Cout + co) = s;
    }
  }
}

// ===========================================================================
// LDS-DMA pipelined variant (all layers except the Cin=3 first layer).
//
// Same math and output as conv_wgrad_kernel, restructured for latency:
//  * both tiles are staged by global_load_lds_dwordx4 (LDS-DMA, no VGPR
//    round trip); zero padding = lanes pointed at a zero page;
//  * NBUF-deep ring of stages, NBUF-1 stages in flight, counted
//    s_waitcnt vmcnt(N) + raw s_barrier (never a vmcnt(0) drain in the loop);
//  * the swizzle that makes the transposed reads conflict-free is applied to
//    the per-lane SOURCE address (the LDS destination of an LDS-DMA is
//    lane-linear), and the same XOR is used on the read side;
//  * k tiles may straddle taps (Cin = 64 layers): each 16-B chunk computes
//    its own (tap, ci); k >= K chunks read zeros and are not stored;
//  * pixel -> (oh, ow) by multiply-high division (no integer divide).
// Waves: WC x WK x WM, each 64 co x 64 k over 64 pixels of every stage
// (WM > 1: the waves split the stage's pixels, partial tiles summed in LDS).
// ===========================================================================
struct WgradArgs2 {
  const bf16_t* dy;
  const bf16_t* x;
  const bf16_t* zero;   // >= 16 B of zeros
  float* ws;
  float* wsb;
  int H, W, Cin, Cout, ksize, dil, M, K, S, mslice;
  FastDiv fdW, fdH, fdC;
  // batched GEMMs (wgrad_glds2 only): nb independent problems of the same shape,
  // operands nb apart by these element strides, slabs by S*K*Cout (default 1 / 0)
  int nb = 1;
  long long dy_bs = 0, x_bs = 0;
  // wgrad_glds2 on a ragged width (W % 64 != 0): the pixel index is VIRTUAL — every image row padded to
  // tx64 = ceil(W / 64) 64-pixel stages (M, mslice count virtual pixels); the padding pixels' activations come from
  // the zero page, so they add nothing.  tx64 = W / 64 and fdTX = fdiv by it on an aligned width (the same stages)
  int tx64 = 0;
  FastDiv fdTX;
  int Mreal = 0;        // real pixel count (the dY descriptor's range); M is virtual on a ragged width
};

template <int RB>   // row bytes
__device__ __forceinline__ int swz8b(int row, int c8) {
  if (RB >= 256) return c8 ^ (((row & 3) | (((row >> 3) & 1) << 2)) << 2);
  else return c8 ^ (((((row >> 1) & 1)) | (((row >> 3) & 1) << 1)) << 2);
}

template <int DT, int WC, int WK, int WM, int NBUF, int KW, int KK>
__global__ void __launch_bounds__(64 * WC * WK * WM, (WC * WK * WM >= 8) ? 1 : 2) wgrad_glds_kernel(WgradArgs2 a) {
  constexpr int NW = WC * WK * WM;
  constexpr int TCo = 64 * WC, TK = 64 * WK * KW;
  constexpr int BKM = 32 * KK * WM;              // pixels per stage (KK 32-deep MFMA steps per wave)
  constexpr int RBA = TCo * 2, RBB = TK * 2;
  constexpr int A_BYTES = BKM * RBA, B_BYTES = BKM * RBB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NIA = A_BYTES / 1024, NIB = B_BYTES / 1024;
  constexpr int G = (NIA + NIB) / NW;            // LDS-DMA instructions per wave per stage
  static_assert((NIA + NIB) % NW == 0, "instruction split");
  constexpr int D = NBUF - 1;                     // stages in flight

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wk = (wave / WC) % WK, wm = wave / (WC * WK);

  const int nco = a.Cout / TCo, nkt = (a.K + TK - 1) / TK;
  const int ntile = nco * nkt;
  const int bid = xcd_remap(blockIdx.x, ntile * a.S);
  const int tile = bid % ntile, slice = bid / ntile;
  const int co0 = (tile % nco) * TCo, k0 = (tile / nco) * TK;
  const bool do_bias = (a.wsb != nullptr) && (k0 == 0);
  const int mbeg = slice * a.mslice;
  const int mend = min(a.M, mbeg + a.mslice);
  const int nstage = (mend > mbeg) ? (mend - mbeg + BKM - 1) / BKM : 0;

  // ---- LDS-DMA issue of one stage.  Per-lane source addresses are
  // recomputed from (wave, instruction, lane) each time: keeping G
  // descriptors live would cost ~40 VGPRs and push the accumulators out of
  // the AGPR file (hipcc then copies them around every MFMA).
  auto issue = [&](int st, int buf) {
    const int m0 = mbeg + st * BKM;
    unsigned char* sbase = smem + buf * STAGE;
    int lane = tid & 63;
    // small tiles issue many LDS-DMA per stage: keep the compiler from
    // hoisting G address sets out of the loop (they would spill)
    if constexpr (G > 8 || KW > 1) asm volatile("" : "+v"(lane));
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int gi = wave + NW * i;          // wave-uniform
      const void* src = a.zero;
      unsigned char* dst;
      if (gi < NIA) {
        const int byte = gi * 1024 + lane * 16;
        const int row = byte / RBA;
        const int lc16 = swz8b<RBA>(row, ((byte % RBA) / 16) * 2) >> 1;
        const int m = m0 + row;
        if (m < mend) src = a.dy + (size_t)m * a.Cout + co0 + lc16 * 8;
        dst = sbase + gi * 1024;
      } else {
        const int byte = (gi - NIA) * 1024 + lane * 16;
        const int row = byte / RBB;
        const int lc16 = swz8b<RBB>(row, ((byte % RBB) / 16) * 2) >> 1;
        const int m = m0 + row;
        const int k = k0 + lc16 * 8;
        if (k < a.K && m < mend) {
          const int tap = (int)fdiv((uint32_t)k, a.fdC);
          const int ci = k - tap * a.Cin;
          int dh = 0, dw = 0;
          if (a.ksize == 3) {
            const int kh = (tap * 11) >> 5;        // tap / 3 for tap < 9
            dh = (kh - 1) * a.dil;
            dw = (tap - kh * 3 - 1) * a.dil;
          }
          const uint32_t qq = fdiv((uint32_t)m, a.fdW);
          const int ow = m - (int)qq * a.W;
          const int oh = (int)qq - (int)fdiv(qq, a.fdH) * a.H;
          const int ih = oh + dh, iw = ow + dw;
          if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
            src = a.x + (size_t)(m + dh * a.W + dw) * a.Cin + ci;
        }
        dst = sbase + A_BYTES + (gi - NIA) * 1024;
      }
      glds16(src, lds_addr(dst));
    }
  };

  f32x4 acc[4][4 * KW];
  f32x4 accb[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    accb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4 * KW; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const frag8_t ones = ones_frag<DT>();

  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  auto rd = [&](const unsigned char* base, int rb_is_wide, int rb, int prow0, int col0) -> frag8_t {
    const int r0 = prow0 + 8 * g + q;
    const int c8 = (col0 >> 2) + p;
    const int s0 = rb_is_wide ? swz8b<256>(r0, c8) : swz8b<128>(r0, c8);
    const int s1 = rb_is_wide ? swz8b<256>(r0 + 4, c8) : swz8b<128>(r0 + 4, c8);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + r0 * rb + s0 * 8));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (r0 + 4) * rb + s1 * 8));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(frag8_t, v);
  };

  // prologue: D stages in flight
#pragma unroll
  for (int s = 0; s < D; ++s)
    if (s < nstage) issue(s, s);

  for (int st = 0; st < nstage; ++st) {
    if (nstage - 1 - st >= D - 1) {
      if constexpr (D >= 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"((D - 1) * G) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (st + D < nstage) issue(st + D, (st + D) % NBUF);
    const unsigned char* Ab = smem + (st % NBUF) * STAGE;
    const unsigned char* Bb = Ab + A_BYTES;
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      const int prow0 = wm * 32 * KK + kk * 32;
      frag8_t af[4], bfr[4 * KW];
#pragma unroll
      for (int j = 0; j < 4; ++j) af[j] = rd(Ab, RBA >= 256, RBA, prow0, wc * 64 + j * 16);
#pragma unroll
      for (int i = 0; i < 4 * KW; ++i) bfr[i] = rd(Bb, RBB >= 256, RBB, prow0, wk * 64 * KW + i * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4 * KW; ++i)
          acc[j][i] = mfma16<DT>(af[j], bfr[i], acc[j][i]);
      if (do_bias && wk == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) accb[j] = mfma16<DT>(af[j], ones, accb[j]);
      }
    }
  }

  // ---- epilogue
  const int fr = lane & 15, fq = lane >> 4;
  float* slab = a.ws + (size_t)slice * a.K * a.Cout;
  if constexpr (WM == 1) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4 * KW; ++i) {
        const int k = k0 + wk * 64 * KW + i * 16 + fr;
        const int co = co0 + wc * 64 + j * 16 + fq * 4;
        if (k < a.K) *reinterpret_cast<f32x4*>(slab + (size_t)k * a.Cout + co) = acc[j][i];
      }
    if (do_bias && wk == 0 && fr == 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int co = co0 + wc * 64 + j * 16 + fq * 4;
        *reinterpret_cast<f32x4*>(a.wsb + (size_t)slice * a.Cout + co) = accb[j];
      }
    }
  } else {
    static_assert(KW == 1, "pixel-split waves use 64x64 wave tiles");
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);   // [NW][16][64][4] (+ bias [NW][4][64][4])
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        *reinterpret_cast<f32x4*>(red + ((wave * 16 + j * 4 + i) * 64 + lane) * 4) = acc[j][i];
    float* redb = red + NW * 16 * 64 * 4;
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 4; ++j) *reinterpret_cast<f32x4*>(redb + ((wave * 4 + j) * 64 + lane) * 4) = accb[j];
    }
    __syncthreads();
    if (wm == 0) {
      // waves of the first pixel group reduce and store their own (wc, wk) tile
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int w2 = 0; w2 < WM; ++w2) {
            const int wv = wave + w2 * WC * WK;
            s += *reinterpret_cast<const f32x4*>(red + ((wv * 16 + j * 4 + i) * 64 + lane) * 4);
          }
          const int k = k0 + wk * 64 + i * 16 + fr;
          const int co = co0 + wc * 64 + j * 16 + fq * 4;
          if (k < a.K) *reinterpret_cast<f32x4*>(slab + (size_t)k * a.Cout + co) = s;
        }
      if (do_bias && wk == 0 && fr == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f32x4 s = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int w2 = 0; w2 < WM; ++w2) {
            const int wv = wave + w2 * WC * WK;
            s += *reinterpret_cast<const f32x4*>(redb + ((wv * 4 + j) * 64 + lane) * 4);
          }
          const int co = co0 + wc * 64 + j * 16 + fq * 4;
          *reinterpret_cast<f32x4*>(a.wsb + (size_t)slice * a.Cout + co) = s;
        }
      }
    }
  }
}

template <int DT, int WC, int WK, int WM, int NBUF, int KW, int KK>
static int launch_wgrad2(const WgradArgs2& a, hipStream_t s) {
  constexpr int NW = WC * WK * WM;
  constexpr int STAGE = 32 * KK * WM * (64 * WC + 64 * WK * KW) * 2;
  size_t lds = (size_t)NBUF * STAGE;
  if (WM > 1) lds = std::max(lds, (size_t)(NW * 16 * 64 * 4 + NW * 4 * 64 * 4) * 4);
  auto kfn = wgrad_glds_kernel<DT, WC, WK, WM, NBUF, KW, KK>;
  static bool attr = false;
  if (!attr) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int ntile = (a.Cout / (64 * WC)) * ((a.K + 64 * WK * KW - 1) / (64 * WK * KW));
  hipLaunchKernelGGL(kfn, dim3(ntile * a.S), dim3(64 * NW), lds, s, a);
  return (int)hipGetLastError();
}

// ===========================================================================
// v2 of the LDS-DMA weight-gradient kernel for row-aligned layers
// (W % 64 == 0, K % TK == 0): every 64-pixel stage lies inside ONE image row,
// so a stage is (n, oh, ow0..ow0+63) and every per-lane quantity of the DMA
// addressing — the lane's (tap, ci) and its row inside the stage — is a
// loop invariant.  Per stage the wave computes (oh, ow0) once (scalar) and
// each B (activation) DMA costs two range compares and a select; the dY
// DMA is a pure pointer add.  Fragment reads are software-pipelined across
// the barrier exactly like conv_glds2_kernel (second K half read under the
// first half's MFMAs, the next stage's first half read right after the
// barrier under the other half).
// ===========================================================================
template <int DT, int WC, int WK, int KW, bool RW = false>
__global__ void __launch_bounds__(64 * WC * WK, 1) wgrad_glds2_kernel(WgradArgs2 a) {
  constexpr int NW = WC * WK;
  constexpr int TCo = 64 * WC, TK = 64 * WK * KW;
  constexpr int BKM = 64;                          // pixels per stage (2 MFMA K steps)
  constexpr int RBA = TCo * 2, RBB = TK * 2;
  constexpr int A_BYTES = BKM * RBA, B_BYTES = BKM * RBB;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NIA = A_BYTES / 1024, NIB = B_BYTES / 1024;
  constexpr int GA = NIA / NW, GB = NIB / NW;
  static_assert(NIA % NW == 0 && NIB % NW == 0, "instruction split");
  static_assert(RBB == 512 || RBB == 256, "B row = 256 or 128 k (2 or 4 pixel rows per 1-KiB DMA)");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wk = wave / WC;

  const int nco = a.Cout / TCo, nkt = a.K / TK;
  const int ntile = nco * nkt;
  const int bid = xcd_remap(blockIdx.x, ntile * a.S * a.nb);
  const int tile = bid % ntile, slice = (bid / ntile) % a.S, bt = bid / (ntile * a.S);
  const int co0 = (tile % nco) * TCo, k0 = (tile / nco) * TK;
  const int mbeg = slice * a.mslice;
  const int mend = min(a.M, mbeg + a.mslice);
  const int nstage = (mend > mbeg) ? (mend - mbeg) / BKM : 0;   // M, mslice multiples of 64
  const bf16_t* gdy = a.dy + bt * a.dy_bs;
  const bf16_t* gx = a.x + bt * a.x_bs;

  // dY tile through a buffer resource: per-lane 32-bit offsets, stage base in soffset.  DMA piece j of a
  // wave lands NW * 1024 / RB rows after piece 0 (a multiple of 16 rows: the same XOR swizzle), so one
  // per-lane base offset + a wave-uniform stride per piece replaces the per-piece offset arrays (they
  // pushed this kernel to 256 VGPRs with spills)
  const __amdgpu_buffer_rsrc_t dy_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)gdy, (short)0, a.Mreal * a.Cout * 2, 0x00020000);
  constexpr int ASTEP = NW * 1024 / RBA, BSTEP = NW * 1024 / RBB;    // rows between pieces
  static_assert(ASTEP % 16 == 0 && BSTEP % 16 == 0, "piece stride must keep the row swizzle");
  unsigned aoff0;
  int arow0;
  {
    const int byte = wave * 1024 + lane * 16;
    const int row = byte / RBA;
    arow0 = row;
    const int lc16 = swz8b<RBA>(row, ((byte % RBA) / 16) * 2) >> 1;
    aoff0 = (unsigned)(row * a.Cout + co0 + lc16 * 8) * 2u;
  }
  const unsigned astride = (unsigned)(ASTEP * a.Cout * 2);
  // Cin % TK == 0: the whole k tile is ONE tap -> (dh, dw) are block-uniform
  const int tap = k0 / a.Cin;
  int dh = 0, dw = 0;
  if (a.ksize == 3) {
    const int kh = (tap * 11) >> 5;
    dh = (kh - 1) * a.dil;
    dw = (tap - kh * 3 - 1) * a.dil;
  }
  const int ci0 = k0 - tap * a.Cin;
  int boff0, brow0;
  {
    const int byte = wave * 1024 + lane * 16;
    const int row = byte / RBB;
    brow0 = row;
    const int lc16 = swz8b<RBB>(row, ((byte % RBB) / 16) * 2) >> 1;
    boff0 = (row + dh * a.W + dw) * a.Cin + ci0 + lc16 * 8;
  }
  const int bstride = BSTEP * a.Cin;

  // DMA of one stage, in 4 parts (part p = pieces [p*GA/4 ...) of dY then [p*GB/4 ...) of X) so that the
  // issue cost of the 8 LDS-DMA pieces (~60-100 cycles each beside MFMAs) is spread between MFMA groups
  // instead of stalling both waves of a SIMD in one burst after the barrier (-DCANNET_DMA_BURST at build
  // time: the burst form)
  struct StageAddr {
    unsigned soff;
    const bf16_t* xs;
    int ow0;
    bool row_ok;
    unsigned char* sbase;
  };
  auto stage_addr = [&](int st, int buf) -> StageAddr {
    StageAddr sa;
    const int g = (mbeg + st * BKM) >> 6;             // virtual 64-pixel stage = (image row q, column block)
    const uint32_t q = fdiv((uint32_t)g, a.fdTX);
    sa.ow0 = (g - (int)q * a.tx64) * 64;
    const int m0 = (int)q * a.W + sa.ow0;             // its first real pixel
    const int oh = (int)q - (int)fdiv(q, a.fdH) * a.H;
    sa.row_ok = (unsigned)(oh + dh) < (unsigned)a.H;     // stage-uniform
    sa.sbase = smem + buf * STAGE;
    sa.soff = (unsigned)m0 * (unsigned)a.Cout * 2u;
    sa.xs = gx + (size_t)m0 * a.Cin;
    return sa;
  };
  auto issue_part = [&](const StageAddr& sa, int p, int parts) {
#if defined(CAN_WPROBE) && (CAN_WPROBE & 1)
    return;                                         // diagnostic build (scripts/probe): no DMA
#endif
#pragma unroll
    for (int j = p * GA / parts; j < (p + 1) * GA / parts; ++j) {
      if constexpr (RW) {
        // ragged width: the stage's padding pixels (>= W) are pixels of the next row (or past the end of dY): their
        // lanes get an offset beyond the descriptor's range (the range check on the per-lane offset returns zeros);
        // the stage base travels in the per-lane offset, not in soffset
        const bool okA = sa.ow0 + arow0 + j * ASTEP < a.W;
        blds16(dy_rsrc, okA ? aoff0 + j * astride + sa.soff : 0xFFFFFFF0u, 0u,
               lds_addr(sa.sbase + (wave + NW * j) * 1024));
      } else {
        blds16(dy_rsrc, aoff0 + j * astride, sa.soff, lds_addr(sa.sbase + (wave + NW * j) * 1024));
      }
    }
#pragma unroll
    for (int j = p * GB / parts; j < (p + 1) * GB / parts; ++j) {
      const int ow = sa.ow0 + brow0 + j * BSTEP;      // this piece row's output pixel (>= W: ragged padding)
      const int iw = ow + dw;
      const bool ok = sa.row_ok && ((unsigned)iw < (unsigned)a.W) && ow < a.W;
      const void* src = ok ? (const void*)(sa.xs + boff0 + j * bstride) : (const void*)a.zero;
      glds16(src, lds_addr(sa.sbase + A_BYTES + (wave + NW * j) * 1024));
    }
  };
  auto issue = [&](int st, int buf) { issue_part(stage_addr(st, buf), 0, 1); };
  constexpr int PARTS = (GA % 4 == 0 && GB % 4 == 0) ? 4 : 1;   // 2 parts measured slower (F5: +3..8%)

  f32x4 acc[4][4 * KW];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4 * KW; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, qd = (lane & 15) >> 2, p = lane & 3;
  auto rd = [&](const unsigned char* base, int rb_wide, int rb, int prow0, int col0) -> frag8_t {
#if defined(CAN_WPROBE) && (CAN_WPROBE & 2)
    return __builtin_bit_cast(frag8_t, make_uint4(prow0 + lane, col0, rb, 1));   // diagnostic: no LDS reads
#endif
    const int r0 = prow0 + 8 * g + qd;
    const int c8 = (col0 >> 2) + p;
    const int s0 = rb_wide ? swz8b<256>(r0, c8) : swz8b<128>(r0, c8);
    const int s1 = rb_wide ? swz8b<256>(r0 + 4, c8) : swz8b<128>(r0 + 4, c8);
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + r0 * rb + s0 * 8));
    const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (r0 + 4) * rb + s1 * 8));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(frag8_t, v);
  };
  auto read = [&](int buf, int kk, frag8_t (&af)[4], frag8_t (&bfr)[4 * KW]) {
    const unsigned char* Ab = smem + buf * STAGE;
    const unsigned char* Bb = Ab + A_BYTES;
    const int prow0 = kk * 32;
#pragma unroll
    for (int j = 0; j < 4; ++j) af[j] = rd(Ab, RBA >= 256, RBA, prow0, wc * 64 + j * 16);
#pragma unroll
    for (int i = 0; i < 4 * KW; ++i) bfr[i] = rd(Bb, RBB >= 256, RBB, prow0, wk * 64 * KW + i * 16);
  };
  auto mma = [&](const frag8_t (&af)[4], const frag8_t (&bfr)[4 * KW], int i0, int i1) {
#pragma unroll
    for (int i = i0; i < i1; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[j][i] = mfma16<DT>(af[j], bfr[i], acc[j][i]);
  };

  if (nstage > 0) {
    frag8_t a0[4], b0[4 * KW], a1[4], b1[4 * KW];
    issue(0, 0);
    if (nstage > 1) {
      issue(1, 1);
      asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(GA + GB) : "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
    }
    read(0, 0, a0, b0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    for (int st = 0; st < nstage - 1; ++st) {
      const int buf = st & 1;
      read(buf, 1, a1, b1);
      __builtin_amdgcn_sched_barrier(0);
      mma(a0, b0, 0, 4 * KW);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0x0070);
      asm volatile("s_barrier" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
#ifndef CANNET_DMA_BURST
      if constexpr (PARTS > 1) {
        // DMA parts interleaved with the four MFMA groups of the second K half; the reads of stage s+1's
        // first half after the second group
        const bool more = st + 2 < nstage;
        StageAddr sa;
        if (more) sa = stage_addr(st + 2, buf);
        constexpr int ord = CANNET_DMA_ORDER_WG;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          if (ord == 0 && more) issue_part(sa, g, PARTS);
          __builtin_amdgcn_sched_barrier(0);
          mma(a1, b1, g * KW, (g + 1) * KW);
          __builtin_amdgcn_sched_barrier(0);
          if (ord != 0 && more && (ord == 1 || g < 3)) {
            issue_part(sa, g, PARTS);
            if (ord == 2 && g == 2) issue_part(sa, 3, PARTS);
          }
          __builtin_amdgcn_sched_barrier(0);
          if (g == 1) read(buf ^ 1, 0, a0, b0);
          __builtin_amdgcn_sched_barrier(0);
        }
        __builtin_amdgcn_s_waitcnt(0xC07F);
        continue;
      }
#endif
      if (st + 2 < nstage) issue(st + 2, buf);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1, 0, 2 * KW);
      __builtin_amdgcn_sched_barrier(0);
      read(buf ^ 1, 0, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1, 2 * KW, 4 * KW);
      __builtin_amdgcn_sched_barrier(0);
      __builtin_amdgcn_s_waitcnt(0xC07F);
    }
    read((nstage - 1) & 1, 1, a1, b1);
    mma(a0, b0, 0, 4 * KW);
    mma(a1, b1, 0, 4 * KW);
  }

  const int fr = lane & 15, fq = lane >> 4;
  float* slab = a.ws + ((size_t)bt * a.S + slice) * a.K * a.Cout;
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4 * KW; ++i) {
      const int k = k0 + wk * 64 * KW + i * 16 + fr;
      const int co = co0 + wc * 64 + j * 16 + fq * 4;
      *reinterpret_cast<f32x4*>(slab + (size_t)k * a.Cout + co) = acc[j][i];
    }
}

// Bias gradient partials for the v2 path: part[b][co] = sum of dY rows of
// chunk b (SB chunks, fixed order; wgrad_reduce sums the SB partials).  A
// separate short launch with many blocks, so the GEMM grid stays whole rounds.
template <int DT>
__global__ void __launch_bounds__(256) bias_colsum_kernel(const bf16_t* __restrict__ dy, float* __restrict__ part,
                                                          int M, int Cout, int SB) {
  __shared__ float red[256 * 8];
  const int C8 = Cout >> 3;
  const int groups = 256 / C8;                    // row groups (C8 <= 256 -> >= 1)
  const int cg = threadIdx.x % C8, rg = threadIdx.x / C8;
  const int rows = (M + SB - 1) / SB;
  const int m0 = blockIdx.x * rows, m1 = min(M, m0 + rows);
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (rg < groups) {
    const bf16_t* base = dy + cg * 8;
    int m = m0 + rg;
    for (; m + 3 * groups < m1; m += 4 * groups) {
      uint4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const uint4*>(base + (size_t)(m + u * groups) * Cout);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const unsigned w4[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          s[2 * e2] += h2f<DT>((unsigned short)(w4[e2] & 0xffffu));
          s[2 * e2 + 1] += h2f<DT>((unsigned short)(w4[e2] >> 16));
        }
      }
    }
    for (; m < m1; m += groups) {
      const uint4 v = *reinterpret_cast<const uint4*>(base + (size_t)m * Cout);
      const unsigned w4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e2 = 0; e2 < 4; ++e2) {
        s[2 * e2] += h2f<DT>((unsigned short)(w4[e2] & 0xffffu));
        s[2 * e2 + 1] += h2f<DT>((unsigned short)(w4[e2] >> 16));
      }
    }
  }
#pragma unroll
  for (int e2 = 0; e2 < 8; ++e2) red[threadIdx.x * 8 + e2] = s[e2];
  __syncthreads();
  if (rg == 0) {
#pragma unroll
    for (int e2 = 0; e2 < 8; ++e2) {
      float t = 0.f;
      for (int r = 0; r < groups; ++r) t += red[(r * C8 + cg) * 8 + e2];
      part[(size_t)blockIdx.x * Cout + cg * 8 + e2] = t;
    }
  }
}

template <int DT, int WC, int WK, int KW, bool RW = false>
static int launch_wgrad3(const WgradArgs2& a, hipStream_t s) {
  constexpr int STAGE = 64 * (64 * WC + 64 * WK * KW) * 2;
  const size_t lds = 2 * (size_t)STAGE;
  auto kfn = wgrad_glds2_kernel<DT, WC, WK, KW, RW>;
  static bool attr = false;
  if (!attr) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int ntile = (a.Cout / (64 * WC)) * (a.K / (64 * WK * KW));
  hipLaunchKernelGGL(kfn, dim3(ntile * a.S * a.nb), dim3(64 * WC * WK), lds, s, a);
  return (int)hipGetLastError();
}

#include "wgrad_tap.inc"

// ===========================================================================
// Halo-tiled weight gradient for 3x3 / dilation-1 layers with Cin % 64 == 0 and
// Cout in {64, 128} (the high-resolution VGG layers conv1_2, conv2_1, conv2_2).
//
// The generic kernel re-streams dY once per k-tile and X once per co-tile
// from HBM (dY/X of conv1_2 are 0.8 GB each at batch 8) and its 64-wide tiles
// are L2-bound.  Here one block stages an output tile of TH x 64 pixels of dY
// plus the (TH+2) x 66 input halo of one 64-channel slice of X ONCE, and its 9
// waves - one per tap - read their shifted windows of the same halo with
// transposed LDS reads: every byte is fetched once per block-stage and feeds
// 9 taps.  Out tile per block = Cout x (9 taps x 64 ci); partial slabs and the
// deterministic reduction are shared with the generic kernel.
// ===========================================================================
struct HaloArgs {
  const bf16_t* dy;
  const bf16_t* x;
  const bf16_t* zero;
  float* ws;
  float* wsb;
  int N, H, W, Cin, Cout, K, S;
  int tiles_y, tiles_x, ntiles, tiles_per_slice;
};

template <int DT, int CO, int TH>
__global__ void __launch_bounds__(576, 1) wgrad_halo_kernel(HaloArgs a) {
  constexpr int TW = 64;
  constexpr int HW_ = TW + 2;                       // halo width
  constexpr int HH = TH + 2;                        // halo height
  constexpr int NPIX = TH * TW;
  constexpr int RBD = CO * 2;                       // dY row bytes
  constexpr int DY_BYTES = NPIX * RBD;
  constexpr int X_BYTES = ((HH * HW_ * 128 + 1023) / 1024) * 1024;
  constexpr int STAGE = DY_BYTES + X_BYTES;
  constexpr int NID = DY_BYTES / 1024;              // LDS-DMA instructions per stage
  constexpr int NIX = X_BYTES / 1024;
  constexpr int NT = CO / 16;                       // co tiles of 16

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);     // = tap
  const int kh = wave / 3, kw = wave % 3;
  const int nci = a.Cin >> 6, nco = a.Cout / CO;
  const int ci_t = blockIdx.x % nci;
  const int co0 = ((blockIdx.x / nci) % nco) * CO;
  const int slice = blockIdx.x / (nci * nco);
  const int ci0 = ci_t * 64;
  const int t_beg = slice * a.tiles_per_slice;
  const int t_end = min(a.ntiles, t_beg + a.tiles_per_slice);
  const int nstage = max(0, t_end - t_beg);
  const bool do_bias = (a.wsb != nullptr) && ci_t == 0 && wave == 4;

  // i_lo .. i_hi: the stage's DMA pieces to issue (dY pieces [0, NID), X pieces [NID, NID + NIX))
  auto issue = [&](int st, int buf, int i_lo = 0, int i_hi = -1) {
    if (i_hi < 0) i_hi = NID + NIX;
    const int t = t_beg + st;
    const int n = t / (a.tiles_y * a.tiles_x);
    const int rem = t - n * a.tiles_y * a.tiles_x;
    const int y0 = (rem / a.tiles_x) * TH, x0 = (rem % a.tiles_x) * TW;
    unsigned char* sbase = smem + buf * STAGE;
    for (int i = i_lo + (wave + 9 - i_lo % 9) % 9; i < i_hi; i += 9) {
      const void* src = a.zero;
      unsigned char* dst;
      if (i < NID) {
        const int byte = i * 1024 + lane * 16;
        const int p = byte / RBD;
        const int lc16 = swz8b<RBD>(p, ((byte % RBD) / 16) * 2) >> 1;
        const int yy = y0 + p / TW, xx = x0 + p % TW;
        if (yy < a.H && xx < a.W) src = a.dy + ((size_t)(n * a.H + yy) * a.W + xx) * a.Cout + co0 + lc16 * 8;
        dst = sbase + i * 1024;
      } else {
        const int byte = (i - NID) * 1024 + lane * 16;
        const int q = byte / 128;
        const int lc16 = swz8b<128>(q, ((byte % 128) / 16) * 2) >> 1;
        const int yy = y0 - 1 + q / HW_, xx = x0 - 1 + q % HW_;
        if (q < HH * HW_ && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
          src = a.x + ((size_t)(n * a.H + yy) * a.W + xx) * a.Cin + ci0 + lc16 * 8;
        dst = sbase + DY_BYTES + (i - NID) * 1024;
      }
      glds16(src, lds_addr(dst));
    }
  };
  f32x4 acc[NT][4];
  f32x4 accb[NT];
#pragma unroll
  for (int j = 0; j < NT; ++j) {
    accb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const frag8_t ones = ones_frag<DT>();
  const int g = lane >> 4, q = (lane & 15) >> 2, p = lane & 3;
  // transposed read of 8 consecutive rows r0.. (pixels) at column col0 of an LDS image with RB-byte rows
  auto rd = [&](const unsigned char* base, auto rbc, int prow0, int col0) -> frag8_t {
    constexpr int RB = decltype(rbc)::value;
    const int r0 = prow0 + 8 * g + q;
    const int c8 = (col0 >> 2) + p;
    const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + r0 * RB + swz8b<RB>(r0, c8) * 8));
    const s16x4 hi =
        __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)(base + (r0 + 4) * RB + swz8b<RB>(r0 + 4, c8) * 8));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(frag8_t, v);
  };
  using RBdy = std::integral_constant<int, RBD>;
  using RBx = std::integral_constant<int, 128>;

  if (nstage > 0) issue(0, 0);
  for (int st = 0; st < nstage; ++st) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (st + 1 < nstage) issue(st + 1, (st + 1) & 1);
    const unsigned char* Db = smem + (st & 1) * STAGE;
    const unsigned char* Xb = Db + DY_BYTES;
#pragma unroll
    for (int r = 0; r < TH; ++r) {
#pragma unroll
      for (int gg = 0; gg < TW / 32; ++gg) {
        const int prow_d = r * TW + gg * 32;
        const int prow_x = (r + kh) * HW_ + gg * 32 + kw;
        frag8_t af[NT], bfr[4];
#pragma unroll
        for (int j = 0; j < NT; ++j) af[j] = rd(Db, RBdy{}, prow_d, j * 16);
#pragma unroll
        for (int i = 0; i < 4; ++i) bfr[i] = rd(Xb, RBx{}, prow_x, i * 16);
#pragma unroll
        for (int j = 0; j < NT; ++j)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            acc[j][i] = mfma16<DT>(af[j], bfr[i], acc[j][i]);
        if (do_bias) {
#pragma unroll
          for (int j = 0; j < NT; ++j) accb[j] = mfma16<DT>(af[j], ones, accb[j]);
        }
      }
    }
  }
  // epilogue: slab[slice][k = tap*Cin + ci][co]
  const int fr = lane & 15, fq = lane >> 4;
  float* slab = a.ws + (size_t)slice * a.K * a.Cout;
#pragma unroll
  for (int j = 0; j < NT; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int k = wave * a.Cin + ci0 + i * 16 + fr;
      const int co = co0 + j * 16 + fq * 4;
      *reinterpret_cast<f32x4*>(slab + (size_t)k * a.Cout + co) = acc[j][i];
    }
  if (do_bias && fr == 0) {
#pragma unroll
    for (int j = 0; j < NT; ++j)
      *reinterpret_cast<f32x4*>(a.wsb + (size_t)slice * a.Cout + co0 + j * 16 + fq * 4) = accb[j];
  }
}

template <int DT, int CO, int TH>
static int launch_halo(HaloArgs& a, hipStream_t s) {
  constexpr int TW = 64;
  constexpr int DY_BYTES = TH * TW * CO * 2;
  constexpr int X_BYTES = (((TH + 2) * (TW + 2) * 128 + 1023) / 1024) * 1024;
  const size_t lds = 2 * (size_t)(DY_BYTES + X_BYTES);
  auto kfn = wgrad_halo_kernel<DT, CO, TH>;
  static bool attr = false;
  if (!attr) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL(kfn, dim3((a.Cin / 64) * (a.Cout / CO) * a.S), dim3(576), lds, s, a);
  return (int)hipGetLastError();
}

#include "wgrad_ring.inc"

template <int DT, int WC, int WK, int WM, bool FIRST>
static int launch_wgrad(const WgradArgs& a, hipStream_t s) {
  constexpr int TCo = 64 * WC, TK = 64 * WK;
  constexpr int KSUB = (WM == 1) ? 2 : 1;
  constexpr int BKM = 32 * KSUB * WM;
  size_t lds = 2 * BKM * (TCo + TK) * 2;
  if (WM != 1) lds = std::max(lds, (size_t)(4 * 16 * 64 * 4 + 4 * 4 * 64 * 4) * 4);
  auto kfn = conv_wgrad_kernel<DT, WC, WK, WM, FIRST>;
  static bool attr = false;
  if (!attr) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int ntile = (a.Cout / TCo) * (a.Ktot / TK);
  hipLaunchKernelGGL(kfn, dim3(ntile * a.S), dim3(256), lds, s, a);
  return (int)hipGetLastError();
}

}  // namespace can

// Tile configs of the pipelined kernel: 1 = 128co x 128k (4 waves, 4 bufs),
// 2 = 256co x 128k (8 waves, 3 bufs), 3 = 64co x 128k (4 waves, pixel-split 2,
// 3 bufs), 4 = 64co x 64k (2 waves, pixel-split 2, 4 bufs); 0 = first layer
// (register-staged kernel).
namespace can {
// Sum S slabs [S][K][Cout] in a fixed order and write dW in the PyTorch layout
// [Cout][Cin][kh][kw] (first layer: Cin = 3 real channels of the k = tap*4 + c
// packing); beta = 0 overwrites, 1 accumulates.
// Grid-stride slab reduction (v2): SG slice groups x (256/SG) elements per
// block, grid capped at 4096 blocks (the element-per-block form was bound by
// block dispatch for S ~ 7 and planes of millions of elements).  Each group
// sums slices sl = g, g+SG, ... in order with 4 accumulators; groups combine in
// LDS in a fixed order: deterministic.  The last Cout/16 blocks reduce the bias parts.
// bias: block = 16 channels x 16 part groups (group g sums parts g, g+16, ...), fixed order
__device__ __forceinline__ void reduce_bias_block(const float* __restrict__ wsb, float* __restrict__ db, int Sb,
                                                  int Cout, float beta, float scale, int bb, float (&bpart)[16][16]) {
  const int c = bb * 16 + (threadIdx.x & 15), g = threadIdx.x >> 4;
  float t0 = 0.f, t1 = 0.f;
  if (c < Cout) {
    int sl = g;
    for (; sl + 16 < Sb; sl += 32) {
      t0 += wsb[(size_t)sl * Cout + c];
      t1 += wsb[(size_t)(sl + 16) * Cout + c];
    }
    if (sl < Sb) t0 += wsb[(size_t)sl * Cout + c];
  }
  bpart[g][threadIdx.x & 15] = t0 + t1;
  __syncthreads();
  if (g == 0 && c < Cout) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) v += bpart[q][threadIdx.x & 15];
    v *= scale;
    db[c] = (beta != 0.f) ? db[c] * beta + v : v;
  }
}

template <int SG>
__global__ void __launch_bounds__(256) wgrad_reduce2_kernel(const float* __restrict__ ws, const float* __restrict__ wsb,
                                                            float* __restrict__ dw, float* __restrict__ db, int S,
                                                            int Sb, int Ktot, int Cout, int Cin, int taps, int first,
                                                            float beta, float scale,
                                                            const float* __restrict__ dscale) {
  constexpr int EPB = 256 / SG;
  if (dscale != nullptr) scale *= dscale[0];          // device-side factor (1 / loss scale)
  __shared__ float part[SG][EPB];
  __shared__ float bpart[16][16];
  const int e = threadIdx.x % EPB, grp = threadIdx.x / EPB;
  const size_t plane = (size_t)Ktot * Cout;
  const int nbias = (db != nullptr) ? (Cout + 15) / 16 : 0;
  const int nmain = gridDim.x - nbias;
  if ((int)blockIdx.x >= nmain) {
    reduce_bias_block(wsb, db, Sb, Cout, beta, scale, (int)blockIdx.x - nmain, bpart);
    return;
  }
  const int cin_t = first ? 3 : Cin;
  for (size_t base = (size_t)blockIdx.x * EPB; base < plane; base += (size_t)nmain * EPB) {
    const size_t idx = base + e;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
    if (idx < plane) {
      int sl = grp;
      for (; sl + 3 * SG < S; sl += 4 * SG) {
        s0 += ws[(size_t)sl * plane + idx];
        s1 += ws[(size_t)(sl + SG) * plane + idx];
        s2 += ws[(size_t)(sl + 2 * SG) * plane + idx];
        s3 += ws[(size_t)(sl + 3 * SG) * plane + idx];
      }
      for (; sl < S; sl += SG) s0 += ws[(size_t)sl * plane + idx];
    }
    float v = (s0 + s1) + (s2 + s3);
    if (SG > 1) {
      part[grp][e] = v;
      __syncthreads();
      v = 0.f;
      if (grp == 0)
#pragma unroll
        for (int g = 0; g < SG; ++g) v += part[g][e];
      __syncthreads();
    }
    if (grp == 0 && idx < plane) {
      v *= scale;
      const unsigned ui = (unsigned)idx;                 // plane < 2^31 (host-checked)
      const int co = (int)(ui % (unsigned)Cout), k = (int)(ui / (unsigned)Cout);
      int ci, tap;
      bool valid = true;
      if (first) { tap = k >> 2; ci = k & 3; valid = (tap < 9) && (ci < 3); }
      else { tap = k / Cin; ci = k - tap * Cin; }
      if (valid) {
        float* o = dw + ((size_t)co * cin_t + ci) * taps + tap;
        *o = (beta != 0.f) ? (*o * beta + v) : v;
      }
    }
  }
}

// Tiled form for 3x3 layers with few slabs (S <= 16): block = 64 output channels x RCI input channels x 9 taps.
// Slab rows (tap, ci) are read as 256-B runs of 64 co, summed over the slabs in order, transposed through LDS
// and written as 64 contiguous runs of RCI*9 floats of dW[co][ci][tap] (the grid-stride form writes dW with a
// Cin*9-float stride between neighbouring lanes: one 4-B store per 64-B line).
constexpr int RCI = 8;
__global__ void __launch_bounds__(256) wgrad_reduce_tiled_kernel(const float* __restrict__ ws,
                                                                 const float* __restrict__ wsb,
                                                                 float* __restrict__ dw, float* __restrict__ db,
                                                                 int S, int Sb, int Cout, int Cin, float beta,
                                                                 float scale, const float* __restrict__ dscale) {
  constexpr int ROWS = 9 * RCI, LD = 68;          // (tap, ci) rows of 64 co, padded to 68 floats
  __shared__ __attribute__((aligned(16))) float tile[ROWS * LD];
  __shared__ float bpart[16][16];
  if (dscale != nullptr) scale *= dscale[0];
  const int nco = Cout >> 6, nci = Cin / RCI;
  const int nmain = nco * nci;
  if ((int)blockIdx.x >= nmain) {
    reduce_bias_block(wsb, db, Sb, Cout, beta, scale, (int)blockIdx.x - nmain, bpart);
    return;
  }
  const int co0 = ((int)blockIdx.x % nco) * 64, ci0 = ((int)blockIdx.x / nco) * RCI;
  const size_t plane = (size_t)9 * Cin * Cout;
  const int c4 = threadIdx.x & 15, rg = threadIdx.x >> 4;
  for (int row = rg; row < ROWS; row += 16) {
    const int t = row / RCI, ci = row - t * RCI;
    const float* src = ws + ((size_t)(t * Cin + ci0 + ci) * Cout + co0 + c4 * 4);
    // same summation order as wgrad_reduce2_kernel<1> (4 accumulators over slabs sl, sl+1, sl+2, sl+3)
    float4 acc[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
    int sl = 0;
    for (; sl + 3 < S; sl += 4) {
      float4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(src + (size_t)(sl + u) * plane);
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
      }
    }
    for (; sl < S; ++sl) {
      const float4 v = *reinterpret_cast<const float4*>(src + (size_t)sl * plane);
      acc[0].x += v.x; acc[0].y += v.y; acc[0].z += v.z; acc[0].w += v.w;
    }
    *reinterpret_cast<float4*>(tile + row * LD + c4 * 4) =
        make_float4(((acc[0].x + acc[1].x) + (acc[2].x + acc[3].x)) * scale,
                    ((acc[0].y + acc[1].y) + (acc[2].y + acc[3].y)) * scale,
                    ((acc[0].z + acc[1].z) + (acc[2].z + acc[3].z)) * scale,
                    ((acc[0].w + acc[1].w) + (acc[2].w + acc[3].w)) * scale);
  }
  __syncthreads();
  // dW[co][ci0 .. ci0 + RCI)[0 .. 9) is RCI*9 contiguous floats per co
  for (int e = threadIdx.x; e < 64 * ROWS; e += 256) {
    const int co = e / ROWS, rem = e - co * ROWS;
    const int ci = rem / 9, t = rem - ci * 9;
    const float v = tile[(t * RCI + ci) * LD + co];
    float* o = dw + ((size_t)(co0 + co) * Cin + ci0) * 9 + rem;
    *o = (beta != 0.f) ? (*o * beta + v) : v;
  }
}

// Bias partials produced by the data-gradient epilogue that wrote dY (conv_igemm.hip, EPI_MASK /
// EPI_POOLBWD: one row per wave's pixel slice, up to ~10^5 rows): [R][C] -> [G][C], block g sums rows
// [g*RPB, (g+1)*RPB) in order (deterministic), so the reduce kernels' bias blocks see <= 512 rows.
__global__ void __launch_bounds__(256) bias_rows_reduce_kernel(const float* __restrict__ in, float* __restrict__ out,
                                                               int R, int C, int RPB) {
  __shared__ float4 red[256];
  const int C4 = C >> 2;                       // C % 64 == 0, C <= 1024
  const int groups = 256 / C4;
  const int col = threadIdx.x % C4, rg = threadIdx.x / C4;
  const int r0 = blockIdx.x * RPB, r1 = min(R, r0 + RPB);
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (rg < groups) {
    for (int r = r0 + rg; r < r1; r += groups) {
      const float4 v = reinterpret_cast<const float4*>(in + (size_t)r * C)[col];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  if (rg == 0) {
    for (int g = 1; g < groups; ++g) {
      const float4 v = red[g * C4 + col];
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    reinterpret_cast<float4*>(out + (size_t)blockIdx.x * C)[col] = acc;
  }
}

static int launch_reduce2(const float* ws, const float* wsb, float* dw, float* db, int S, int Sb, int K, int Cout,
                          int Cin, int taps, int first, float beta, float scale, const float* dscale, hipStream_t s) {
  const size_t plane = (size_t)K * Cout;
  const int nbias = (db != nullptr) ? (Cout + 15) / 16 : 0;
  auto grid = [&](int epb) { return (int)std::min<size_t>((plane + epb - 1) / epb, 4096) + nbias; };
  if (g_dispatch.reduce_tiled && !first && taps == 9 && S <= 16 && Cout % 64 == 0 && Cin % RCI == 0 &&
      (Cout / 64) * (Cin / RCI) >= 256) {
    hipLaunchKernelGGL(wgrad_reduce_tiled_kernel, dim3((Cout / 64) * (Cin / RCI) + nbias), dim3(256), 0, s, ws, wsb,
                       dw, db, S, Sb, Cout, Cin, beta, scale, dscale);
  } else if (S <= 16)
    hipLaunchKernelGGL(wgrad_reduce2_kernel<1>, dim3(grid(256)), dim3(256), 0, s, ws, wsb, dw, db, S, Sb, K, Cout,
                       Cin, taps, first, beta, scale, dscale);
  else if (S <= 128)
    hipLaunchKernelGGL(wgrad_reduce2_kernel<4>, dim3(grid(64)), dim3(256), 0, s, ws, wsb, dw, db, S, Sb, K, Cout,
                       Cin, taps, first, beta, scale, dscale);
  else
    hipLaunchKernelGGL(wgrad_reduce2_kernel<16>, dim3(grid(16)), dim3(256), 0, s, ws, wsb, dw, db, S, Sb, K, Cout,
                       Cin, taps, first, beta, scale, dscale);
  return (int)hipGetLastError();
}
}  // namespace can
using namespace can;

// bias partial count of the v2 path (workspace: max(S, kBiasParts) x Cout floats)
static constexpr int kBiasParts = 512;

static void wgrad_tile(int cfg, int* TCo, int* TK, int* BKM) {
  switch (cfg) {
    case 1: *TCo = 128; *TK = 128; *BKM = 64; break;
    case 2: *TCo = 256; *TK = 128; *BKM = 64; break;
    case 3: *TCo = 64; *TK = 128; *BKM = 128; break;
    case 4: *TCo = 64; *TK = 64; *BKM = 128; break;
    case 5: *TCo = 256; *TK = 256; *BKM = 32; break;
    case 6: *TCo = 128; *TK = 256; *BKM = 64; break;
    case 7: *TCo = 256; *TK = 256; *BKM = 64; break;
    case 9: *TCo = 256; *TK = 256; *BKM = 64; break;   // v2 (row-aligned layers), falls back to 7
    case 10: *TCo = 256; *TK = 128; *BKM = 64; break;  // v2 256co x 128k (Cin = 128), falls back to 2
    case 11: *TCo = 128; *TK = 256; *BKM = 64; break;  // v2 128co x 256k (Cout = 128), falls back to 6
    case 8: *TCo = 0; *TK = 0; *BKM = 128; break;   // halo kernel: tiles of 2x64 pixels
    default: *TCo = 64; *TK = 64; *BKM = 128; break;
  }
}

extern "C" int can_wgrad_plan(int M, int Cin, int Cout, int ksize, int first, int target_blocks, int* S_out,
                              int* mslice_out, int* cfg_out, int dil, int W) {
  const int K = first ? 64 : ksize * ksize * Cin;
  int cfg;
  // the halo weight-gradient kernel is dilation-1 only (B5: 256 -> 128, dil 2, reaches M >= 262144 at batch 32)
  const bool halo_ok = !first && ksize == 3 && dil == 1 && (Cout == 64 || Cout == 128) && Cin % 64 == 0;
  if (first) cfg = 0;
  else if (halo_ok && M >= 262144) cfg = 8;
  else if (Cout % 256 == 0 && K >= 2048) cfg = (K % 256 == 0) ? 9 : 7;
  else if (Cout % 256 == 0 && ksize == 1 && K % 256 == 0 && K >= 512)
    cfg = 9;   // 1x1 with many output rows (the linearised context module's dW2cat: 2048 x 512)
  else if (Cout % 256 == 0 && K >= 1024)
    cfg = (Cin % 128 == 0) ? 10 : 2;
  else if (Cout == 128 && Cin % 256 == 0 && K >= 2048)
    cfg = 11;
  else if (Cout % 128 == 0 && K >= 2048) cfg = 6;
  else if (Cout % 128 == 0) cfg = 1;
  else if (K >= 128) cfg = 3;
  else cfg = 4;
  // the tap-ring kernel (wgrad_tap.inc) for the layers the v2 GEMM takes (dispatch wgrad_tap >= 1) and the Cout = 128
  // ones of the full-resolution ring kernel (>= 2); it needs the map width (W = 0: unknown, not chosen)
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0)
      ncu = 256;
  }
  // the smallest slice count that fills whole rounds of one-block-per-CU launches to >= 90 %
  auto whole_rounds = [&](int ntile) {
    for (int R = 1; R <= 8; ++R) {
      const int s = (ncu * R) / ntile;
      if (s >= 1 && (long long)ntile * s * 10 >= 9LL * ncu * R) return s;
    }
    return 0;
  };
  const int tco = wgrad_tap_tco(Cout);
  if (!first && W > 0 && M % W == 0 && wgrad_tap_ok(1, M / W, W, Cin, Cout, ksize, dil) && cfg != 0 &&
      g_dispatch.wgrad_tap >= (tco == 64 ? 3 : cfg == 8 ? 2 : 1)) {
    // one block per CU (TCO 128) or two (TCO 64)
    const int ntile = (Cin / 64) * (Cout / tco);
    const int stages = (M / W) * ((W + 63) / 64);
    const int slots_per_cu = (tco == 128) ? 1 : 2;
    int S = 0;
    for (int R = 1; R <= 8 && !S; ++R) {
      const int s = (ncu * slots_per_cu * R) / ntile;
      if (s >= 1 && (long long)ntile * s * 10 >= 9LL * ncu * slots_per_cu * R) S = s;
    }
    if (S < 1) S = max(1, ncu * slots_per_cu / ntile);
    if (S > stages) S = stages;
    *S_out = S; *mslice_out = 0; *cfg_out = 12;
    return 0;
  }
  int TCo, TK, BKM;
  wgrad_tile(cfg, &TCo, &TK, &BKM);
  if (cfg == 8) {
    // slices of whole 2x64-pixel tiles; the Python side passes N,H,W to the launcher,
    // here only the slice count matters: ~2 blocks per CU worth of (ci tile, slice) pairs.
    const int nci = (Cin / 64) * (Cout / 64);
    int S = 512 / nci;
    if (S < 1) S = 1;
    *S_out = S; *mslice_out = 0; *cfg_out = cfg;
    return 0;
  }
  const int ntile = (Cout / TCo) * ((K + TK - 1) / TK);
  // whole rounds of co-resident blocks (no half-empty last round)
  int S = target_blocks / ntile;
  if (cfg != 0 && cfg != 8) {
    // the pipelined kernels run one block per CU (LDS ring >= 128 KB): as few pixel slices as fill
    // whole rounds of the CUs to >= 90 % (fewer fp32 partial slabs to write and
    // reduce, longer K loops per block)
    const int wr = whole_rounds(ntile);
    if (wr) S = wr;
  }
  if (S < 1) S = 1;
  const int max_s = (M + BKM - 1) / BKM;
  if (S > max_s) S = max_s;
  if (S < 1) S = 1;
  int mslice = (M + S - 1) / S;
  mslice = ((mslice + BKM - 1) / BKM) * BKM;
  S = (M + mslice - 1) / mslice;
  *S_out = S; *mslice_out = mslice; *cfg_out = cfg;
  return 0;
}

static const can::bf16_t* zero_page() {
  static void* z = nullptr;
  if (!z) {
    if (hipMalloc(&z, 4096) != hipSuccess) return nullptr;
    if (hipMemset(z, 0, 4096) != hipSuccess) return nullptr;
  }
  return (const can::bf16_t*)z;
}

template <int DT>
static int conv_wgrad_impl(const void* dy, const void* x, float* ws, float* wsb, float* dw, float* db, int N, int H,
                           int W, int Cin, int Cout, int ksize, int dil, int first, int S, int mslice, int cfg,
                           float beta, float scale, const float* dscale, void* stream, const float* bext,
                           int bext_rows) {
  using namespace can;
  hipStream_t s = (hipStream_t)stream;
  const int K = first ? 64 : ksize * ksize * Cin;
  if ((long long)K * Cout >= 0x7fffffffLL) return -9;   // 32-bit plane indexing in the reduction
  // external bias partials (the dgrad epilogue that produced dY summed it): no bias work in the GEMM /
  // column-sum kernels, only a rows pre-reduction into the workspace's bias area (<= kBiasParts rows)
  const bool ext = (db != nullptr) && (bext != nullptr) && bext_rows > 0;
  if (ext && (Cout % 64 || Cout > 1024)) return -15;
  float* wsb_used = (db != nullptr && !ext) ? wsb : nullptr;
  int rc;
  int Sb = S;                       // bias partials summed by the reduce kernel
  int Sb_ext = 0;
  const float* bsrc = wsb;          // bias partial rows the reduce kernel sums (external: bext itself when short)
  // long external lists are folded to <= kBiasParts rows by a short launch queued AFTER the GEMM on this (weight-
  // gradient) stream: it then takes the CUs the GEMM's last blocks release.  Queued on the data-gradient stream (the
  // producer) it waited 85-345 us for CUs behind this stream's one-block-per-CU GEMM, on the critical path
  // (profiles/r3/ab_bias_prereduce.txt)
  int bias_rpb = 0;
  if (ext) {
    if (bext_rows <= kBiasParts) {
      bsrc = bext;
      Sb_ext = bext_rows;
    } else {
      bias_rpb = (bext_rows + kBiasParts - 1) / kBiasParts;
      Sb_ext = (bext_rows + bias_rpb - 1) / bias_rpb;
    }
  }
  auto bias_pre = [&]() {
    if (bias_rpb)
      hipLaunchKernelGGL(bias_rows_reduce_kernel, dim3(Sb_ext), dim3(256), 0, s, bext, wsb, bext_rows, Cout, bias_rpb);
  };
  if (first || cfg == 0) {
    if (Cin != 4 || Cout % 64) return -2;
    WgradArgs a;
    a.dy = (const bf16_t*)dy; a.x = (const bf16_t*)x; a.ws = ws; a.wsb = wsb_used;
    a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.ksize = ksize; a.dil = dil; a.M = N * H * W;
    a.Ktot = 64; a.S = S; a.mslice = mslice;
    rc = launch_wgrad<DT, 1, 1, 4, true>(a, s);
  } else {
    if (Cin % 64 || Cout % 64 || ((H < 2 || W < 2) && cfg != 12)) return -3;
    WgradArgs2 a;
    a.dy = (const bf16_t*)dy; a.x = (const bf16_t*)x; a.zero = zero_page(); a.ws = ws; a.wsb = wsb_used;
    if (!a.zero) return -7;
    a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.ksize = ksize; a.dil = dil; a.M = N * H * W; a.K = K;
    a.S = S; a.mslice = mslice;
    a.fdW = make_fastdiv((uint32_t)W); a.fdH = make_fastdiv((uint32_t)H); a.fdC = make_fastdiv((uint32_t)Cin);
    a.Mreal = a.M;
    a.tx64 = (W + 63) / 64; a.fdTX = make_fastdiv((uint32_t)a.tx64);
    // v2 on a ragged width: virtual pixels (every row padded to whole 64-pixel stages), the same slice count
    const bool rw = (W % 64) != 0 && ksize == 3;
    WgradArgs2 gv = a;
    if (rw) {
      gv.M = N * H * a.tx64 * 64;
      gv.mslice = ((gv.M + S - 1) / S + 63) / 64 * 64;   // slices past the end run no stage and write zero slabs
    }
    if (cfg == 12) {
      if (!wgrad_tap_ok(N, H, W, Cin, Cout, ksize, dil)) return -6;
      if (wsb_used) {
        Sb = kBiasParts;
        hipLaunchKernelGGL(bias_colsum_kernel<DT>, dim3(Sb), dim3(256), 0, s, a.dy, wsb_used, a.M, Cout, Sb);
      }
      TapArgs t;
      t.dy = a.dy; t.x = a.x; t.ws = ws;
      t.N = N; t.H = H; t.W = W; t.Cin = Cin; t.Cout = Cout;
      t.tx64 = (W + 63) / 64;
      t.total = N * H * t.tx64;
      t.S = S;
      t.spb = (t.total + S - 1) / S;
      t.dy_bytes = (unsigned)((long long)a.M * Cout * 2);
      t.x_bytes = (unsigned)((long long)a.M * Cin * 2);
      const bool adb = g_dispatch.wgrad_tap_adb != 0;
      if (wgrad_tap_tco(Cout) == 128) {
        if (adb) rc = (dil == 1) ? launch_wgrad_tap<DT, 1, 128, true>(t, s) : launch_wgrad_tap<DT, 2, 128, true>(t, s);
        else rc = (dil == 1) ? launch_wgrad_tap<DT, 1, 128, false>(t, s) : launch_wgrad_tap<DT, 2, 128, false>(t, s);
      } else {
        if (adb) rc = (dil == 1) ? launch_wgrad_tap<DT, 1, 64, true>(t, s) : launch_wgrad_tap<DT, 2, 64, true>(t, s);
        else rc = (dil == 1) ? launch_wgrad_tap<DT, 1, 64, false>(t, s) : launch_wgrad_tap<DT, 2, 64, false>(t, s);
      }
      if (rc) return rc;
      bias_pre();
      return ext ? launch_reduce2(ws, bsrc, dw, db, S, Sb_ext, K, Cout, Cin, 9, 0, beta, scale, dscale, s)
                 : launch_reduce2(ws, wsb_used, dw, db, S, Sb, K, Cout, Cin, 9, 0, beta, scale, dscale, s);
    }
    if (cfg == 8) {
      if (ksize != 3 || dil != 1 || (Cout != 64 && Cout != 128) || Cin % 64) return -6;
      HaloArgs h;
      h.dy = a.dy; h.x = a.x; h.zero = a.zero; h.ws = ws; h.wsb = wsb_used;
      h.N = N; h.H = H; h.W = W; h.Cin = Cin; h.Cout = Cout; h.K = K; h.S = S;
      // Cout = 128 runs as two 64-channel co tiles.  Default: the row-ring kernel (4-row tiles walked
      // down 64-column strips, each input row fetched once per strip); dispatch wgrad_halo_ring = 0: 2-row tiles
      // with a full halo per tile
      const bool ring = g_dispatch.wgrad_halo_ring != 0;
      const int th = ring ? 4 : 2;
      h.tiles_y = (H + th - 1) / th; h.tiles_x = (W + 63) / 64; h.ntiles = N * h.tiles_y * h.tiles_x;
      h.tiles_per_slice = (h.ntiles + S - 1) / S;
      rc = ring ? launch_halo_ring<DT, 64, 4>(h, s) : launch_halo<DT, 64, 2>(h, s);
      if (rc) return rc;
      bias_pre();
      return ext ? launch_reduce2(ws, bsrc, dw, db, S, Sb_ext, K, Cout, Cin, 9, 0, beta, scale, dscale, s)
                 : launch_reduce2(ws, wsb_used, dw, db, S, S, K, Cout, Cin, 9, 0, beta, scale, dscale, s);
    }
    switch (cfg) {
      case 1: if (Cout % 128) return -4; rc = launch_wgrad2<DT, 2, 2, 1, 4, 1, 2>(a, s); break;
      case 2: if (Cout % 256) return -4; rc = launch_wgrad2<DT, 4, 2, 1, 3, 1, 2>(a, s); break;
      case 3: rc = launch_wgrad2<DT, 1, 2, 2, 3, 1, 2>(a, s); break;
      case 4: rc = launch_wgrad2<DT, 1, 1, 2, 4, 1, 2>(a, s); break;
      case 5: if (Cout % 256) return -4; rc = launch_wgrad2<DT, 4, 2, 1, 4, 2, 1>(a, s); break;
      case 6: if (Cout % 128) return -4; rc = launch_wgrad2<DT, 2, 2, 1, 3, 2, 2>(a, s); break;
      case 7: if (Cout % 256) return -4; rc = launch_wgrad2<DT, 4, 2, 1, 2, 2, 2>(a, s); break;
      case 9:
        if (Cout % 256) return -4;
        if ((W % 64 == 0 || rw) && Cin % 256 == 0 && gv.mslice % 64 == 0 && (long long)a.M * Cout * 2 < 0x7fffffffLL &&
            Cout <= 2048) {
          if (wsb_used) {
            Sb = kBiasParts;
            hipLaunchKernelGGL(bias_colsum_kernel<DT>, dim3(Sb), dim3(256), 0, s, a.dy, wsb_used, a.M, Cout, Sb);
          }
          WgradArgs2 g = gv;
          g.wsb = nullptr;
          rc = rw ? launch_wgrad3<DT, 4, 2, 2, true>(g, s) : launch_wgrad3<DT, 4, 2, 2>(g, s);
        } else
          rc = launch_wgrad2<DT, 4, 2, 1, 2, 2, 2>(a, s);   // same tiles / slicing as cfg 7
        break;
      case 10:   // 256co x 128k v2 (k tile = one tap of a Cin % 128 layer); fallback = cfg 2 tiles
      case 11: { // 128co x 256k v2 (Cout = 128); fallback = cfg 6 tiles
        const int tk = (cfg == 10) ? 128 : 256;
        if (Cout % (cfg == 10 ? 256 : 128)) return -4;
        if ((W % 64 == 0 || rw) && Cin % tk == 0 && K % tk == 0 && gv.mslice % 64 == 0 &&
            (long long)a.M * Cout * 2 < 0x7fffffffLL && Cout <= 2048) {
          if (wsb_used) {
            Sb = kBiasParts;
            hipLaunchKernelGGL(bias_colsum_kernel<DT>, dim3(Sb), dim3(256), 0, s, a.dy, wsb_used, a.M, Cout, Sb);
          }
          WgradArgs2 g = gv;
          g.wsb = nullptr;
          if (rw) rc = (cfg == 10) ? launch_wgrad3<DT, 4, 2, 1, true>(g, s) : launch_wgrad3<DT, 2, 4, 1, true>(g, s);
          else rc = (cfg == 10) ? launch_wgrad3<DT, 4, 2, 1>(g, s) : launch_wgrad3<DT, 2, 4, 1>(g, s);
        } else {
          rc = (cfg == 10) ? launch_wgrad2<DT, 4, 2, 1, 3, 1, 2>(a, s) : launch_wgrad2<DT, 2, 2, 1, 3, 2, 2>(a, s);
        }
        break;
      }
      default: return -5;
    }
  }
  if (rc) return rc;
  bias_pre();
  if (ext) return launch_reduce2(ws, bsrc, dw, db, S, Sb_ext, K, Cout, first ? 4 : Cin, ksize * ksize, first, beta,
                                 scale, dscale, s);
  return launch_reduce2(ws, wsb_used, dw, db, S, Sb, K, Cout, first ? 4 : Cin, ksize * ksize, first, beta, scale, dscale,
                        s);
}

// dt: element type of dy / x (DT_BF16 = 0, DT_F16 = 1); the gradients are fp32.  The result is
// multiplied by scale and, when dscale is not null, by the device scalar dscale[0] (1 / loss scale).
// bext (optional): [bext_rows][Cout] fp32 bias partials of dy already summed by its producer (the data-gradient
// epilogue): db comes from them, the kernels here do no bias work
extern "C" int can_bias_rows_reduce(const float* in, float* out, int R, int C, int rows_out, void* stream) {
  if (C % 64 || C > 1024 || R < 1 || rows_out < 1) return -2;
  const int rpb = (R + rows_out - 1) / rows_out;
  const int g = (R + rpb - 1) / rpb;
  hipLaunchKernelGGL(can::bias_rows_reduce_kernel, dim3(g), dim3(256), 0, (hipStream_t)stream, in, out, R, C, rpb);
  if (hipGetLastError() != hipSuccess) return -3;
  return g;                                   // rows written
}

extern "C" int can_conv_wgrad(const void* dy, const void* x, float* ws, float* wsb, float* dw, float* db, int N,
                              int H, int W, int Cin, int Cout, int ksize, int dil, int first, int S, int mslice,
                              int cfg, float beta, float scale, const float* dscale, int dt, void* stream,
                              const float* bext, int bext_rows) {
  CAN_DT_DISPATCH(dt, conv_wgrad_impl<DT>(dy, x, ws, wsb, dw, db, N, H, W, Cin, Cout, ksize, dil, first, S, mslice,
                                          cfg, beta, scale, dscale, stream, bext, bext_rows));
}

// Batched 1x1 weight gradient without bias: nb problems dW_b[Cout][Cin] = sum_m dY_b[m][co] X_b[m][ci]
// (the four conv{S}_2 layers of the context module, one launch instead of four half-filled ones).
// dY_b = dy + b*dy_bs, X_b = x + b*x_bs (elements), dW_b = dw + b*dw_bs (floats); ws holds nb*S slabs.
template <int DT>
static int conv_wgrad_1x1_batched_impl(const void* dy, const void* x, float* ws, float* dw, int M, int W, int Cin,
                                       int Cout, int nb, long long dy_bs, long long x_bs, long long dw_bs, int S,
                                       int mslice, float beta, float scale, const float* dscale, hipStream_t s) {
  using namespace can;
  if (Cout % 256 || Cin % 256 || W % 64 || mslice % 64 || M % 64 || (long long)M * Cout * 2 >= 0x7fffffffLL) return -3;
  WgradArgs2 a;
  a.dy = (const bf16_t*)dy; a.x = (const bf16_t*)x; a.zero = zero_page(); a.ws = ws; a.wsb = nullptr;
  if (!a.zero) return -7;
  a.H = M / W; a.W = W; a.Cin = Cin; a.Cout = Cout; a.ksize = 1; a.dil = 1; a.M = M; a.K = Cin;
  a.S = S; a.mslice = mslice;
  a.fdW = make_fastdiv((uint32_t)W); a.fdH = make_fastdiv((uint32_t)(M / W)); a.fdC = make_fastdiv((uint32_t)Cin);
  a.Mreal = M; a.tx64 = W / 64; a.fdTX = make_fastdiv((uint32_t)a.tx64);
  a.nb = nb; a.dy_bs = dy_bs; a.x_bs = x_bs;
  int rc = launch_wgrad3<DT, 4, 2, 2>(a, s);
  if (rc) return rc;
  const size_t slabs = (size_t)S * Cin * Cout;
  for (int b = 0; b < nb; ++b) {
    rc = launch_reduce2(ws + b * slabs, nullptr, dw + b * dw_bs, nullptr, S, S, Cin, Cout, Cin, 1, 0, beta, scale,
                        dscale, s);
    if (rc) return rc;
  }
  return 0;
}

extern "C" int can_conv_wgrad_1x1_batched(const void* dy, const void* x, float* ws, float* dw, int M, int W, int Cin,
                                          int Cout, int nb, long long dy_bs, long long x_bs, long long dw_bs, int S,
                                          int mslice, float beta, float scale, const float* dscale, int dt,
                                          void* stream) {
  CAN_DT_DISPATCH(dt, conv_wgrad_1x1_batched_impl<DT>(dy, x, ws, dw, M, W, Cin, Cout, nb, dy_bs, x_bs, dw_bs, S,
                                                      mslice, beta, scale, dscale, (hipStream_t)stream));
}

// first-layer slab reduction: ws [S][36][64] (k = tap*4 + c), wsb [S][64] -> dW [64][3][3][3], db [64]
extern "C" int can_wgrad_reduce_first(const float* ws, const float* wsb, float* dw, float* db, int S, float beta,
                                      float scale, const float* dscale, void* stream) {
  return launch_reduce2(ws, wsb, dw, db, S, S, 36, 64, 4, 9, 1, beta, scale, dscale, (hipStream_t)stream);
}
