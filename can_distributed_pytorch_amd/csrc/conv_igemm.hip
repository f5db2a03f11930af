// MFMA implicit-GEMM convolution for gfx950 (forward and data-gradient).
//
// Replaces the cuDNN/MIOpen convolutions the reference gets implicitly from
// nn.Conv2d (model/CANNet.py:14-17,114-115): 3x3 dilation 1 (VGG frontend),
// 3x3 dilation 2 (backend), 1x1 (context module / head).  SURVEY §2.5 F1-B6.
//
// GEMM view (NHWC activations, K-contiguous packed weights):
//   Y[m][co] = sum_k  Wp[co][k] * Xcol[m][k],   k = tap*Cin + ci,
//   m = flattened output pixel (n, oh, ow), Xcol gathered on the fly with
//   zero padding (no im2col buffer).
// The data gradient is the same GEMM with the flipped/transposed weight pack
// (Wd[ci][tap'][co] = W[co][8-tap'][ci]) applied to dY, so one kernel serves
// both; the epilogue multiplies by the ReLU mask of the previous layer.
//
// CDNA4 mapping:
//   * wave64, MFMA v_mfma_f32_16x16x32_bf16, fp32 accumulation;
//   * each wave owns a 64(ch) x 64(pix) tile = 4x4 MFMA tiles (64 acc VGPRs);
//     the weight tile is the MFMA A operand (rows = channels), the pixel tile
//     the B operand (cols = pixels).  Weight rows are loaded into LDS in a
//     permuted order so that every lane ends up holding 16 CONSECUTIVE output
//     channels of one pixel -> two 16-byte global stores per 16x16 tile with no
//     LDS round trip in the epilogue;
//   * LDS tiles are [rows][64 bf16] (128-B rows) with the 16-B chunk index
//     XOR-swizzled by (row & 7): conflict-free for the ds_read_b128 lane
//     groups of gfx950 (checked exhaustively for the fragment read pattern);
//   * K loop in 64-deep steps, register-staged double buffer: the next tile's
//     global loads are issued before the MFMAs of the current tile and written
//     to the other LDS buffer after them (one barrier per K step);
//   * 1-D grid with a bijective XCD-aware remap so that the channel tiles
//     sharing one pixel tile (and its halo) run on the same XCD / L2.
#include "common.h"
#include "fastdiv.h"
#include <stdlib.h>

namespace can {


struct ConvArgs {
  const bf16_t* x;     // NHWC [N][H][W][Cin] bf16 (FIRST: Cin = 4, channel 3 zero)
  const bf16_t* w;     // packed [Cout][Ktot] bf16
  const float* bias;   // [Cout] fp32 (EPI_BIAS*) or nullptr
  const bf16_t* mask;  // [M][Cout] bf16, output multiplied by (mask > 0) (EPI_MASK)
  bf16_t* y;           // [M][Cout] bf16
  int N, H, W, Cin, Cout, ksize, dil, M;
};

// Max-pool codes: the forward pool epilogues record, per pooled pixel and channel, a 4-bit one-hot of the
// FIRST max of its 2x2 window (ATen scan order (0,0),(0,1),(1,0),(1,1) = bit 0..3), or 0 when that max is
// not > 0 (the ReLU mask of the pool input).  uint32 codes[N][H/2][W/2][C/8], channel c in word c/8,
// nibble c%8.  That is everything the backward needs, so the full-resolution pre-pool activation
// (805 MB for conv1_2 at batch 8 x 768 x 1024) is never written nor re-read.
// EPI_POOLBWD (LDS-DMA kernels only): the GEMM output is the gradient of a 2x2/s2 max-pool output; the
// epilogue scatters it straight into the pool INPUT gradient through the codes (a.pcodes, pooled
// resolution) into a.y [N][2H][2W][Cout].
// EPI_POOLFWD (LDS-DMA v2 kernel only, H even, W % (TP/2) == 0): bias + ReLU like EPI_BIAS_RELU, and
// the 2x2/s2 max-pool of the result is written to a.yp [N][H/2][W/2][Cout] in the same epilogue.  A pixel
// tile is then 2 image rows x TP/2 columns with the rows interleaved inside each 16-pixel MFMA fragment
// (fragment f, row fr: column f*8 + fr/2, row fr&1), so every pool window sits in 4 adjacent lanes and is
// reduced with two DPP quad permutes (the pooled map is never re-read from HBM by a separate pass).
// EPI_F32 (LDS-DMA kernels only): the raw GEMM result (+ bias when a.bias is given) stored as fp32 into
// a.y reinterpreted as float [M][Cout] — the split-bf16 fp32 path (ops/fp32.py) sums hi*hi + hi*lo + lo*hi
// in one K-concatenated GEMM and needs the fp32 accumulator, not its 16-bit rounding.
// EPI_CTXF / EPI_CTXB (LDS-DMA v2 kernel, 256 x 256 tiles, 1x1): the context module as ONE GEMM each way,
// see "Linearised context module" below.
enum { EPI_BIAS_RELU = 0, EPI_MASK = 1, EPI_NONE = 2, EPI_BIAS = 3, EPI_SIGMOID = 4, EPI_POOLBWD = 5,
       EPI_POOLFWD = 6, EPI_F32 = 7, EPI_CTXF = 8, EPI_CTXB = 9 };
enum { LOAD_GENERIC = 0, LOAD_FIRST = 1 };


__device__ __forceinline__ int swz(int row, int chunk) { return (chunk ^ (row & 7)); }

template <int DT, int WC, int WP, int LOAD, int EPI>
__global__ void __launch_bounds__(64 * WC * WP)
conv_igemm_kernel(ConvArgs a) {
  constexpr int NT = 64 * WC * WP;
  constexpr int TC = 64 * WC;          // output channels per block
  constexpr int TP = 64 * WP;          // output pixels per block
  constexpr int NA = TC * 8 / NT;      // 16-B weight chunks per thread per stage
  constexpr int NB = TP * 8 / NT;      // 16-B pixel chunks per thread per stage
  static_assert(NA >= 1 && NB >= 1, "tile too small");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint4* As = reinterpret_cast<uint4*>(smem);                 // [2][TC][8]
  uint4* Bs = As + 2 * TC * 8;                                // [2][TP][8]

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wc = wave % WC;
  const int wp = wave / WC;

  const int nct = a.Cout / TC;
  const int npt = (a.M + TP - 1) / TP;
  const int tile = xcd_remap(blockIdx.x, nct * npt);
  const int ct = tile % nct;
  const int pt = tile / nct;

  const int Ktot = (LOAD == LOAD_FIRST) ? 64 : a.ksize * a.ksize * a.Cin;
  const int cchunks = (LOAD == LOAD_FIRST) ? 1 : a.Cin / 64;
  const int nk = (LOAD == LOAD_FIRST) ? 1 : a.ksize * a.ksize * cchunks;
  const int HW = a.H * a.W;

  // ---- per-thread fixed rows -------------------------------------------
  const bf16_t* wrow[NA];
  int achunk[NA], arow[NA];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int id = tid + NT * i;
    arow[i] = id >> 3;
    achunk[i] = id & 7;
    wrow[i] = a.w + (size_t)(ct * TC + perm_row(arow[i])) * Ktot + achunk[i] * 8;
  }
  int bm[NB], boh[NB], bow[NB], brow[NB], bchunk[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i) {
    const int id = tid + NT * i;
    brow[i] = id >> 3;
    bchunk[i] = id & 7;
    const int m = pt * TP + brow[i];
    bm[i] = m;
    const int r = m % HW;
    boh[i] = (m < a.M) ? r / a.W : -100000;   // invalid rows never pass the bounds test
    bow[i] = r % a.W;
  }

  uint4 ra[NA], rb[NB];

  auto load_stage = [&](int ks) {
    int tap = 0, c0 = 0;
    if (LOAD == LOAD_GENERIC) {
      tap = ks / cchunks;
      c0 = (ks - tap * cchunks) * 64;
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) ra[i] = *reinterpret_cast<const uint4*>(wrow[i] + ks * 64);
    if (LOAD == LOAD_GENERIC) {
      const int kh = (a.ksize == 3) ? tap / 3 : 1;
      const int kw = (a.ksize == 3) ? tap - kh * 3 : 1;
      const int dh = (kh - 1) * a.dil, dw = (kw - 1) * a.dil;
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        const int ih = boh[i] + dh, iw = bow[i] + dw;
        const bool ok = (ih >= 0) && (ih < a.H) && (iw >= 0) && (iw < a.W);
        uint4 v = make_uint4(0, 0, 0, 0);
        if (ok) v = *reinterpret_cast<const uint4*>(a.x + (size_t)(bm[i] + dh * a.W + dw) * a.Cin + c0 + bchunk[i] * 8);
        rb[i] = v;
      }
    } else {
      // first layer: Cin = 4 (8 B per pixel); chunk j = taps 2j, 2j+1
#pragma unroll
      for (int i = 0; i < NB; ++i) {
        uint2 lo = make_uint2(0, 0), hi = make_uint2(0, 0);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int tap = bchunk[i] * 2 + h;
          if (tap < 9) {
            const int dh = (tap / 3 - 1) * a.dil, dw = (tap % 3 - 1) * a.dil;
            const int ih = boh[i] + dh, iw = bow[i] + dw;
            if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) {
              const uint2 v = *reinterpret_cast<const uint2*>(a.x + (size_t)(bm[i] + dh * a.W + dw) * 4);
              if (h == 0) lo = v; else hi = v;
            }
          }
        }
        rb[i] = make_uint4(lo.x, lo.y, hi.x, hi.y);
      }
    }
  };
  auto store_stage = [&](int buf) {
#pragma unroll
    for (int i = 0; i < NA; ++i) As[(buf * TC + arow[i]) * 8 + swz(arow[i], achunk[i])] = ra[i];
#pragma unroll
    for (int i = 0; i < NB; ++i) Bs[(buf * TP + brow[i]) * 8 + swz(brow[i], bchunk[i])] = rb[i];
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  load_stage(0);
  store_stage(0);
  __syncthreads();

  const int fr = lane & 15;
  const int fq = lane >> 4;
  for (int ks = 0; ks < nk; ++ks) {
    const int buf = ks & 1;
    if (ks + 1 < nk) load_stage(ks + 1);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + fq;
      frag8_t af[4], bfr[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wc * 64 + j * 16 + fr;
        af[j] = __builtin_bit_cast(frag8_t, As[(buf * TC + row) * 8 + swz(row, chunk)]);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int row = wp * 64 + i * 16 + fr;
        bfr[i] = __builtin_bit_cast(frag8_t, Bs[(buf * TP + row) * 8 + swz(row, chunk)]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i)
          acc[j][i] = mfma16<DT>(af[j], bfr[i], acc[j][i]);
    }
    if (ks + 1 < nk) store_stage(buf ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane owns channels [chb, chb+16) of one pixel per tile i
  const int chb = ct * TC + wc * 64 + fq * 16;
  float bias[16];
  if (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_POOLFWD) {
#pragma unroll
    for (int c = 0; c < 16; c += 4) {
      const float4 b4 = *reinterpret_cast<const float4*>(a.bias + chb + c);
      bias[c] = b4.x; bias[c + 1] = b4.y; bias[c + 2] = b4.z; bias[c + 3] = b4.w;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = pt * TP + wp * 64 + i * 16 + fr;
    if (m >= a.M) continue;
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j * 4 + r] = acc[j][i][r];
    if (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_POOLFWD) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        v[c] += bias[c];
        if (EPI != EPI_BIAS) v[c] = fmaxf(v[c], 0.f);
      }
    }
    if (EPI == EPI_SIGMOID) {
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = 1.f / (1.f + __expf(-v[c]));
    }
    const size_t off = (size_t)m * a.Cout + chb;
    if (EPI == EPI_MASK) {
      const uint4 m0 = *reinterpret_cast<const uint4*>(a.mask + off);
      const uint4 m1 = *reinterpret_cast<const uint4*>(a.mask + off + 8);
      const unsigned mw[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const unsigned short bits = (unsigned short)(mw[c >> 1] >> ((c & 1) * 16));
        const bool pos = pos_bits(bits);
        v[c] = pos ? v[c] : 0.f;
      }
    }
    uint4 o0 = make_uint4(pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]), pack2<DT>(v[6], v[7]));
    uint4 o1 = make_uint4(pack2<DT>(v[8], v[9]), pack2<DT>(v[10], v[11]), pack2<DT>(v[12], v[13]), pack2<DT>(v[14], v[15]));
    *reinterpret_cast<uint4*>(a.y + off) = o0;
    *reinterpret_cast<uint4*>(a.y + off + 8) = o1;
  }
}

template <int DT, int WC, int WP, int LOAD, int EPI>
static int launch_conv(const ConvArgs& a, hipStream_t s) {
  constexpr int NT = 64 * WC * WP;
  constexpr int TC = 64 * WC, TP = 64 * WP;
  const size_t lds = 2 * (TC + TP) * 128;
  auto kfn = conv_igemm_kernel<DT, WC, WP, LOAD, EPI>;
  static bool attr_set = false;
  if (!attr_set) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_set = true;
  }
  const int nct = a.Cout / TC;
  const int npt = (a.M + TP - 1) / TP;
  hipLaunchKernelGGL(kfn, dim3(nct * npt), dim3(NT), lds, s, a);
  return (int)hipGetLastError();
}

template <int DT, int LOAD, int EPI>
static int dispatch_tiles(const ConvArgs& a, int tile_cfg, hipStream_t s) {
  // tile_cfg: 0 = auto, 1 = 128ch x 128pix, 2 = 64ch x 256pix, 3 = 128ch x 256pix, 4 = 256ch x 128pix
  int cfg = tile_cfg;
  if (cfg == 0) {
    if (a.Cout % 128 != 0) cfg = 2;
    else if (a.Cout % 256 == 0 && a.M >= 65536) cfg = 4;
    else cfg = 1;
  }
  switch (cfg) {
    case 1: return launch_conv<DT, 2, 2, LOAD, EPI>(a, s);
    case 2: return launch_conv<DT, 1, 4, LOAD, EPI>(a, s);
    case 3: return launch_conv<DT, 2, 4, LOAD, EPI>(a, s);
    case 4: return launch_conv<DT, 4, 2, LOAD, EPI>(a, s);
  }
  return -1;
}


// ===========================================================================
// 8-wave LDS-DMA pipelined variant (every layer except the Cin=3 first one).
//  * tiles TC x TP = (64*WC) channels x (64*PW*WP) pixels, 8 waves, each
//    wave 64 ch x 64*PW pix (PW=2: 128 fp32 accumulators per lane);
//    256x256 for Cout % 256 == 0, 128x256 for Cout % 128, 64x512 for Cout=64;
//  * global_load_lds_dwordx4 staging (no VGPR round trip), 2 LDS buffers,
//    the next stage's DMA overlaps the current stage's MFMAs, raw s_barrier
//    + explicit vmcnt (no __syncthreads vmcnt drain);
//  * zero padding / tail rows: lanes pointed at a zero page;
//  * swizzle applied on the DMA source address (LDS image lane-linear).
// ===========================================================================
struct ConvArgs2 {
  const bf16_t* x;
  const bf16_t* w;
  const float* bias;
  const bf16_t* mask;
  bf16_t* y;
  const bf16_t* zero;
  int H, W, Cin, Cout, ksize, dil, M;
  FastDiv fdW, fdH;
  bf16_t* yp = nullptr;   // EPI_POOLFWD: pooled output [N][H/2][W/2][Cout]
  uint32_t* codes = nullptr;         // EPI_POOLFWD: max-pool codes (optional); a.y optional too
  const uint32_t* pcodes = nullptr;  // EPI_POOLBWD: max-pool codes of the pool this gradient goes through
  // EPI_MASK / EPI_POOLBWD (data gradient = the next layer's dY): bias-gradient partials of that dY,
  // [npt * WP][Cout] fp32, row = pixel tile * WP + wave's pixel slot (optional)
  float* bpart = nullptr;
  // batched launch (v2 kernel): item blockIdx.y reads x + y*xbs, w + y*wbs and writes y + y*ybs (elements)
  long long xbs = 0, wbs = 0, ybs = 0;
  // EPI_CTXF / EPI_CTXB: context-module cell tables [N][50][cC] fp32 (CTXF: ctab0 = t = W2 u, ctab1 = u = W1 ave;
  // CTXB: ctab0 = dave), the concat buffer [M][2 cC] (CTXF: written; CTXB: read, = dcat) and fv [M][cC] (CTXF)
  const float* ctab0 = nullptr;
  const float* ctab1 = nullptr;
  bf16_t* cat = nullptr;
  const bf16_t* fvp = nullptr;
  int cC = 0;
  int ctx_prologue = 0;    // 1: the launch reserved LDS for the row tables beside the staging ring
  // row-ring kernel (conv_rring_kernel): 128-column blocks per image row (ceil(W / 128)), RT-row tile rows per image
  // (ceil(H / RT)) and the pixel-tile count N * rr_ty * rr_tx; a ragged last block / tile row is masked
  int rr_tx = 0, rr_ty = 0, rr_np = 0;
};

// pixel m of row r of pixel tile pt; EPI_POOLFWD tiles are 2 rows x TP/2 columns, rows interleaved per
// 16-pixel fragment (see EPI_POOLFWD), the other epilogues take TP consecutive pixels
// RT (row-ring kernel, conv_rring_kernel): a tile is RT image rows x 128 columns, tile pt = (n, row group, 128-column
// block) with the column block fastest; r = row * 128 + column.  RG (ragged map: W % 128 != 0 or H % RT != 0): the
// tiles are per image (rr_ty tile rows of rr_tx column blocks) and pixels of a ragged last column block or tile row
// map to a.M (= skipped by the epilogue); otherwise (W % 128 == 0, H % RT == 0) tile rows run across images
template <int TP, int EPI, int RT = 0, bool RG = false>
__device__ __forceinline__ int tile_pix(const ConvArgs2& a, int pt, int r) {
  if constexpr (RT != 0 && EPI != EPI_POOLFWD && RG) {
    const int tx = a.rr_tx, q = pt / tx, cb = pt - q * tx;
    const int n = q / a.rr_ty, oh = RT * (q - n * a.rr_ty) + (r >> 7), ow = cb * 128 + (r & 127);
    return (oh < a.H && ow < a.W) ? (n * a.H + oh) * a.W + ow : a.M;
  } else if constexpr (RT != 0 && EPI != EPI_POOLFWD) {
    const int tx = a.W >> 7, q = pt / tx, cb = pt - q * tx;
    return (RT * q + (r >> 7)) * a.W + cb * 128 + (r & 127);
  } else if constexpr (RT != 0 && EPI == EPI_POOLFWD) {
    // row ring, 2 x 128 tiles: fragment f = r / 16 holds columns 8f .. 8f + 7 of both rows, lanes 0-7 row 0 and
    // 8-15 row 1 (the ds_read_b128 lane groups then see 8 distinct pixels per chunk: conflict-free)
    const int ncb = a.W >> 7;
    const int rp = pt / ncb, cb = pt - rp * ncb;
    return (2 * rp + ((r & 15) >> 3)) * a.W + cb * 128 + (r >> 4) * 8 + (r & 7);
  } else if constexpr (EPI == EPI_POOLFWD) {
    const int ncb = a.W / (TP / 2);
    const int rp = pt / ncb, cb = pt - rp * ncb;    // rp = n * H/2 + pooled row
    return (2 * rp + (r & 1)) * a.W + cb * (TP / 2) + (r >> 4) * 8 + ((r & 15) >> 1);
  } else {
    return pt * TP + r;
  }
}

// two 16-bit lanes per VGPR (the max-pool epilogue works on the stored bf16 / fp16 bit patterns: after the ReLU they
// are non-negative, where the unsigned order of the bits is the order of the values)
__device__ __forceinline__ unsigned pk_max_u16(unsigned a, unsigned b) {
  unsigned r;
  asm("v_pk_max_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ unsigned pk_min_u16(unsigned a, unsigned b) {
  unsigned r;
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ unsigned pk_sub_u16(unsigned a, unsigned b) {
  unsigned r;
  asm("v_pk_sub_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}
__device__ __forceinline__ unsigned pk_lshl_b16(unsigned v, unsigned sh) {
  unsigned r;
  asm("v_pk_lshlrev_b16 %0, %1, %2" : "=v"(r) : "v"(sh), "v"(v));
  return r;
}
__device__ __forceinline__ unsigned pk_mul_lo_u16(unsigned a, unsigned b) {
  unsigned r;
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
  return r;
}

// Shared epilogue of the LDS-DMA kernels: lane (fr, fq) of wave (wc, wp) owns
// 16 consecutive output channels of one pixel per 16x16 pixel fragment.
template <int DT, int WC, int WP, int PW, int EPI, int RT = 0, bool RG = false>
__device__ __forceinline__ void glds_epilogue(const ConvArgs2& a, f32x4 (&acc)[4][4 * PW], int ct, int pt,
                                              int wc, int wp, int fr, int fq) {
  constexpr int TC = 64 * WC, TP = 64 * PW * WP;
  const int chb = ct * TC + wc * 64 + fq * 16;
  float bias[16];
  if (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_POOLFWD || (EPI == EPI_F32 && a.bias != nullptr)) {
#pragma unroll
    for (int c = 0; c < 16; c += 4) {
      const float4 b4 = *reinterpret_cast<const float4*>(a.bias + chb + c);
      bias[c] = b4.x; bias[c + 1] = b4.y; bias[c + 2] = b4.z; bias[c + 3] = b4.w;
    }
  }
  constexpr bool BPART = (EPI == EPI_MASK || EPI == EPI_POOLBWD);
  float bs[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) bs[c] = 0.f;
  // the epilogue's global reads (ReLU mask / max-pool codes) for ALL pixel fragments, issued before the first
  // store: the compiler cannot move a load above a store that may alias it, so a per-fragment load was one
  // exposed memory round trip per fragment (4 * PW per tile).  The main loop's operand registers are dead here.
  constexpr int NF = 4 * PW;
  uint4 mk0[EPI == EPI_MASK ? NF : 1], mk1[EPI == EPI_MASK ? NF : 1];
  uint2 pcw[EPI == EPI_POOLBWD ? NF : 1];
  if constexpr (EPI == EPI_MASK || EPI == EPI_POOLBWD) {
#pragma unroll
    for (int i = 0; i < NF; ++i) {
      const int m = tile_pix<TP, EPI, RT, RG>(a, pt, wp * 64 * PW + i * 16 + fr);
      if constexpr (EPI == EPI_MASK) {
        mk0[i] = make_uint4(0u, 0u, 0u, 0u);
        mk1[i] = make_uint4(0u, 0u, 0u, 0u);
        if (m < a.M) {
          const size_t off = (size_t)m * a.Cout + chb;
          mk0[i] = *reinterpret_cast<const uint4*>(a.mask + off);
          mk1[i] = *reinterpret_cast<const uint4*>(a.mask + off + 8);
        }
      } else {
        pcw[i] = make_uint2(0u, 0u);
        if (m < a.M) pcw[i] = *reinterpret_cast<const uint2*>(a.pcodes + (size_t)m * (a.Cout >> 3) + (chb >> 3));
      }
    }
    // one wait for all of them here: with only stores outstanding afterwards, the per-fragment blocks below need
    // no vmcnt wait (the compiler otherwise waits for the previous fragment's stores at every block)
    __builtin_amdgcn_s_waitcnt(0x0F70);             // vmcnt(0), expcnt / lgkmcnt untouched
  }
#pragma unroll
  for (int i = 0; i < 4 * PW; ++i) {
    const int m = tile_pix<TP, EPI, RT, RG>(a, pt, wp * 64 * PW + i * 16 + fr);
    if (m >= a.M) continue;
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) v[j * 4 + r] = acc[j][i][r];
    if constexpr (EPI == EPI_POOLBWD) {
      // pooled pixel m = (n, ph, pw) -> window rows 2ph, 2ph+1, columns 2pw, 2pw+1 of the full map; the
      // window position w (ATen order) gets the gradient iff bit w of the channel's code is set
      const uint32_t q = fdiv((uint32_t)m, a.fdW);
      const int pw = m - (int)q * a.W;
      const uint32_t n = fdiv(q, a.fdH);
      const int ph = (int)q - (int)n * a.H;
      const size_t W2 = 2 * (size_t)a.W;
      const size_t b0 = (((size_t)n * 2 * a.H + 2 * ph) * W2 + 2 * pw) * a.Cout + chb;
      const size_t off[4] = {b0, b0 + a.Cout, b0 + W2 * a.Cout, b0 + W2 * a.Cout + a.Cout};
      const uint2 cw = pcw[i];
      float o[4][16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const unsigned nib = ((c < 8 ? cw.x : cw.y) >> (4 * (c & 7))) & 0xFu;
#pragma unroll
        for (int w = 0; w < 4; ++w) o[w][c] = ((nib >> w) & 1u) ? v[c] : 0.f;
        if (nib) bs[c] += v[c];
      }
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        *reinterpret_cast<uint4*>(a.y + off[w]) = pack8h<DT>(o[w]);
        *reinterpret_cast<uint4*>(a.y + off[w] + 8) = pack8h<DT>(o[w] + 8);
      }
      continue;
    }
    if (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_POOLFWD) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        v[c] += bias[c];
        if (EPI != EPI_BIAS) v[c] = fmaxf(v[c], 0.f);
      }
    }
    if (EPI == EPI_SIGMOID) {
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = 1.f / (1.f + __expf(-v[c]));
    }
    const size_t off = (size_t)m * a.Cout + chb;
    if constexpr (EPI == EPI_F32) {
      if (a.bias != nullptr) {
#pragma unroll
        for (int c = 0; c < 16; ++c) v[c] += bias[c];
      }
      float* yf = reinterpret_cast<float*>(a.y) + off;
#pragma unroll
      for (int c = 0; c < 16; c += 4) *reinterpret_cast<float4*>(yf + c) = make_float4(v[c], v[c + 1], v[c + 2], v[c + 3]);
      continue;
    }
    if constexpr (EPI == EPI_MASK) {
      const uint4 m0 = mk0[i], m1 = mk1[i];
      const unsigned mw[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const unsigned short bits = (unsigned short)(mw[c >> 1] >> ((c & 1) * 16));
        const bool pos = pos_bits(bits);
        v[c] = pos ? v[c] : 0.f;
        bs[c] += v[c];
      }
    }
    const uint4 o0 =
        make_uint4(pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]), pack2<DT>(v[6], v[7]));
    const uint4 o1 =
        make_uint4(pack2<DT>(v[8], v[9]), pack2<DT>(v[10], v[11]), pack2<DT>(v[12], v[13]), pack2<DT>(v[14], v[15]));
    if (EPI != EPI_POOLFWD || a.y != nullptr) {
      *reinterpret_cast<uint4*>(a.y + off) = o0;
      *reinterpret_cast<uint4*>(a.y + off + 8) = o1;
    }
    if constexpr (EPI == EPI_POOLFWD) {
      // lanes 4q .. 4q+3 hold the window (2 columns x 2 rows) of one pooled pixel: max of the stored
      // (rounded) values over quad_perm [1,0,3,2] then [2,3,0,1]; this lane's window position in ATen
      // order is p = row * 2 + column = (fr & 1) * 2 + ((fr >> 1) & 1).  Row ring (RT != 0): the window is
      // lanes 2q, 2q + 1, 2q + 8, 2q + 9 (quad_perm [1,0,3,2] then row_ror 8), p = (fr >> 3) * 2 + (fr & 1)
      constexpr int DPP2 = (RT != 0) ? 0x128 : 0x4E;
      // on the stored 16-bit patterns, two channels per VGPR (channel 2k low half, 2k + 1 high half of word k);
      // the sign bits are cleared so a -0 from the ReLU counts as +0
      const unsigned ow[8] = {o0.x & 0x7FFF7FFFu, o0.y & 0x7FFF7FFFu, o0.z & 0x7FFF7FFFu, o0.w & 0x7FFF7FFFu,
                              o1.x & 0x7FFF7FFFu, o1.y & 0x7FFF7FFFu, o1.z & 0x7FFF7FFFu, o1.w & 0x7FFF7FFFu};
      unsigned mx[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        mx[k] = pk_max_u16(ow[k], (unsigned)__builtin_amdgcn_mov_dpp((int)ow[k], 0xB1, 0xF, 0xF, false));
        mx[k] = pk_max_u16(mx[k], (unsigned)__builtin_amdgcn_mov_dpp((int)mx[k], DPP2, 0xF, 0xF, false));
      }
      uint32_t cw0 = 0u, cw1 = 0u;
      if (a.codes != nullptr) {
        const unsigned ps = (RT != 0) ? (unsigned)((fr >> 3) * 2 + (fr & 1)) : (unsigned)((fr & 1) * 2 + ((fr >> 1) & 1));
        const unsigned ps2 = ps | (ps << 16), one2 = 0x00010001u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // bit p of each half where this lane (window position p) holds the max, OR-ed over the window, the
          // lowest set bit kept (first max), zeroed where the max is not > 0 (ReLU mask)
          unsigned b = pk_lshl_b16(pk_sub_u16(one2, pk_min_u16(ow[k] ^ mx[k], one2)), ps2);
          b |= (unsigned)__builtin_amdgcn_mov_dpp((int)b, 0xB1, 0xF, 0xF, false);
          b |= (unsigned)__builtin_amdgcn_mov_dpp((int)b, DPP2, 0xF, 0xF, false);
          const unsigned nib = pk_mul_lo_u16(b & pk_sub_u16(0u, b), pk_min_u16(mx[k], one2));
          const unsigned byte = (nib & 0xFu) | ((nib >> 12) & 0xF0u);
          if (k < 4) cw0 |= byte << (8 * k); else cw1 |= byte << (8 * (k - 4));
        }
      }
      if ((fr & ((RT != 0) ? 9 : 3)) == 0) {
        const int ncb = a.W / (TP / 2);
        const int rp = pt / ncb, cb = pt - rp * ncb;
        const int pr = wp * 64 * PW + i * 16 + fr;
        const int pc = cb * (TP / 4) + (pr >> 4) * 4 + ((RT != 0) ? ((pr & 7) >> 1) : ((pr & 15) >> 2));
        const size_t pp = (size_t)rp * (a.W >> 1) + pc;
        bf16_t* yp = a.yp + pp * a.Cout + chb;
        *reinterpret_cast<uint4*>(yp) = make_uint4(mx[0], mx[1], mx[2], mx[3]);
        *reinterpret_cast<uint4*>(yp + 8) = make_uint4(mx[4], mx[5], mx[6], mx[7]);
        if (a.codes != nullptr) *reinterpret_cast<uint2*>(a.codes + pp * (a.Cout >> 3) + (chb >> 3)) = make_uint2(cw0, cw1);
      }
    }
  }
  if constexpr (BPART) {
    if (a.bpart != nullptr) store_bias_partials(bs, a.bpart + (size_t)(pt * WP + wp) * a.Cout + chb, fr);
  }
}

// ===========================================================================
// Linearised context module (model/CANNet.py:42-87).
// Per scale S, z_S = conv{S}_2(s_S - fv) with s_S = up(u_S) the bilinear
// (align_corners) upsample of the S x S cells u_S = conv{S}_1(ave_S).  Both
// the 1x1 conv and the upsample are linear per channel, so
//     z_S = up(t_S) - G_S,   t_S = W2_S u_S (S x S cells),  G_S = W2_S fv,
// and the four conv{S}_2 GEMMs over the 4 x [P x 512] expanded maps c_S
// become ONE GEMM over fv itself: G = fv . W2cat^T with the 2048 columns
// interleaved col' = 4c + si (W2cat[4c + si] = W2_S[c]), so every lane of the
// MFMA D layout holds the four scales of 4 consecutive channels of one pixel.
// EPI_CTXF (forward) then computes in registers
//     w_S = sigmoid(up(t_S) - G_S),  fi = sum_S w_S up(u_S) / (sum_S w_S + 1e-12)
// and writes w (a.y [M][4C], what the backward needs), fi and the fv copy into
// the concat buffer (a.cat [M][2C]): c_S, the sigmoid maps and the separate
// expand / fuse passes of the direct form (4 x 2 x 100 MB per 8 x 768 x 1024
// batch) are never materialised.
// EPI_CTXB (backward data gradient): x = dG = -dz [M][4C] (context.hip:
// ctx_bwd_lin), W = W2cat^T [C][4C]; the epilogue adds the concat's direct
// gradient dcat[:, :C], the adaptive-pool adjoint of dave and applies the
// ReLU mask of fv (a.mask) -> dfv.
// The up-sampling / pooling tables are separable: the block stages, for each
// image row its 256 pixels touch (<= 5 rows: W >= 64, checked on the host),
// the y-interpolated (CTXF) or y-pooled (CTXB) values of the 12 column bins
// of the four scales (bins 0 | 1-2 | 3-5 | 6-11) in LDS after the main loop;
// per pixel only the x weights remain.
// ===========================================================================
__device__ __forceinline__ void ctx_scale_of_bin(int bin, int& S, int& j, int& off) {
  const int si = (bin >= 6) ? 3 : (bin >= 3) ? 2 : (bin >= 1) ? 1 : 0;
  S = (si == 0) ? 1 : (si == 1) ? 2 : (si == 2) ? 3 : 6;
  const int bo = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 3 : 6;
  off = (si == 0) ? 0 : (si == 1) ? 1 : (si == 2) ? 5 : 14;
  j = bin - bo;
}
// bilinear taps (align_corners=True) of position x over length L at scale S
__device__ __forceinline__ void ctx_bil(int S, int x, int L, int& x0, int& x1, float& lam) {
  const float sc = (L > 1) ? (float)(S - 1) / (float)(L - 1) : 0.f;
  const float src = sc * (float)x;
  x0 = (int)src;
  x1 = x0 + ((x0 < S - 1) ? 1 : 0);
  lam = src - (float)x0;
}
// adaptive-pool bin [st, en) of index i at scale S over L (ATen: floor / ceil, overlapping when L % S != 0)
__device__ __forceinline__ void ctx_pool_bin(int i, int S, int L, int& st, int& en) {
  st = (i * L) / S;
  en = ((i + 1) * L + S - 1) / S;
}

// CTXF table: tab[((lr * 2 + tensor) * 12 + bin) * TCH + cl], tensor 0 = t, 1 = u, cl = channel in the
// TCH-channel tile (TCH = TC / 4), value = y-bilinear mix of the two cell rows of row rlo + lr.
// CTXB table: tab[(lr * 12 + bin) * TC + cl] = sum over the pool cells (i, j(bin)) whose row bin contains row
// rlo + lr of dave[cell][c] / cell area (cl = channel in the TC-channel tile).
// Both are built in the kernel's prologue into LDS beside the staging ring when they fit (every global load of a
// thread's items is issued before its first LDS write; the main loop's first barrier makes them visible), else
// (CTXB, 256 x 256 tiles) after the main loop in the freed staging LDS.
__host__ __device__ constexpr int ctx_tab_row_bytes(int EPI_, int TC) {
  return EPI_ == EPI_CTXF ? 2 * 12 * (TC / 4) * 4 : 12 * TC * 4;
}
__host__ __device__ constexpr int ctx_max_rows(int TP, int W) { return (TP - 1) / W + 2; }

// adaptive-pool bins of scale S containing x (over L): jA always, jB (or -1) when two bins overlap at x
__device__ __forceinline__ void ctx_pool_cols(int S, int x, int L, int& jA, int& jB) {
  jA = (x * S) / L;
  jB = -1;
  if (jA > 0 && ((jA * L + S - 1) / S) > x) jB = jA - 1;                 // end of bin jA - 1 reaches past x
  else if (jA + 1 < S && ((jA + 1) * L) / S <= x) jB = jA + 1;           // bin jA + 1 starts at or before x
}

template <int EPI, int TC, int NT, int Q>
__device__ __forceinline__ void ctx_build_tab(const ConvArgs2& a, float* tab, int ct, int rlo, int nr) {
  const int C = a.cC;
  constexpr int TCH = (EPI == EPI_CTXF) ? TC / 4 : TC;      // table channels
  constexpr int G4 = TCH / 4;                              // float4 groups per bin
  constexpr int NB = (EPI == EPI_CTXF) ? 24 : 12;          // (tensor,) bin rows per image row
  const int items = nr * NB * G4;
  float4 p0[Q], p1[Q];
  float l1[Q], l0[Q];
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int it = threadIdx.x + q * NT;
    p0[q] = p1[q] = make_float4(0.f, 0.f, 0.f, 0.f);
    l0[q] = l1[q] = 0.f;
    if (it < items) {
      const int c4 = it % G4, rest = it / G4, bin = rest % 12, lt = rest / 12;
      const int lr = (EPI == EPI_CTXF) ? (lt >> 1) : lt;
      const int r = rlo + lr;
      const int n = (int)fdiv((uint32_t)r, a.fdH), y = r - n * a.H;
      int S, j, off;
      ctx_scale_of_bin(bin, S, j, off);
      if constexpr (EPI == EPI_CTXF) {
        int y0, y1;
        float ly;
        ctx_bil(S, y, a.H, y0, y1, ly);
        const float* T = ((lt & 1) ? a.ctab1 : a.ctab0) + ((size_t)n * 50 + off) * C + ct * TCH + c4 * 4;
        p0[q] = *reinterpret_cast<const float4*>(T + (size_t)(y0 * S + j) * C);
        p1[q] = *reinterpret_cast<const float4*>(T + (size_t)(y1 * S + j) * C);
        l0[q] = 1.f - ly;
        l1[q] = ly;
      } else {
        int iA, iB, xs, xe;
        ctx_pool_cols(S, y, a.H, iA, iB);
        ctx_pool_bin(j, S, a.W, xs, xe);
        const float* D = a.ctab0 + ((size_t)n * 50 + off) * C + ct * TCH + c4 * 4;
        int ys, ye;
        ctx_pool_bin(iA, S, a.H, ys, ye);
        l0[q] = 1.f / (float)((ye - ys) * (xe - xs));
        p0[q] = *reinterpret_cast<const float4*>(D + (size_t)(iA * S + j) * C);
        if (iB >= 0) {
          ctx_pool_bin(iB, S, a.H, ys, ye);
          l1[q] = 1.f / (float)((ye - ys) * (xe - xs));
          p1[q] = *reinterpret_cast<const float4*>(D + (size_t)(iB * S + j) * C);
        }
      }
    }
  }
#pragma unroll
  for (int q = 0; q < Q; ++q) {
    const int it = threadIdx.x + q * NT;
    if (it < items) {
      const int c4 = it % G4, rest = it / G4;      // rest = lt * 12 + bin
      *reinterpret_cast<float4*>(tab + (size_t)rest * TCH + c4 * 4) =
          make_float4(l0[q] * p0[q].x + l1[q] * p1[q].x, l0[q] * p0[q].y + l1[q] * p1[q].y,
                      l0[q] * p0[q].z + l1[q] * p1[q].z, l0[q] * p0[q].w + l1[q] * p1[q].w);
    }
  }
}

template <int DT, int WC, int WP, int PW>
__device__ __forceinline__ void ctxf_epilogue(const ConvArgs2& a, f32x4 (&acc)[4][4 * PW], const float* tab, int ct,
                                              int pt, int rlo, int wc, int wp, int fr, int fq) {
  constexpr int TP = 64 * PW * WP, NF = 4 * PW, TCH = 16 * WC;   // TCH: channels of the tile (= TC / 4)
  const int C = a.cC;
  const int cl0 = wc * 16 + fq * 4;                 // this lane's first channel in the tile
  const int c0 = ct * TCH + cl0;
  const int chb = ct * 64 * WC + wc * 64 + fq * 16; // this lane's first GEMM column (= 4 * c0)
  uint2 fvw[NF];
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int m = pt * TP + wp * 64 * PW + i * 16 + fr;
    fvw[i] = make_uint2(0u, 0u);
    if (m < a.M) fvw[i] = *reinterpret_cast<const uint2*>(a.fvp + (size_t)m * C + c0);
  }
#pragma unroll
  for (int i = 0; i < NF; ++i) {
    const int m = pt * TP + wp * 64 * PW + i * 16 + fr;
    if (m >= a.M) continue;
    const int r = (int)fdiv((uint32_t)m, a.fdW), x = m - r * a.W;
    const float* tr = tab + (size_t)(r - rlo) * 2 * 12 * TCH + cl0;
    // T[si][j], U[si][j]: up(t), up(u) of the 4 scales at this pixel, channels c0 + j
    float T[4][4], U[4][4];
    {
      const float4 t = *reinterpret_cast<const float4*>(tr);
      const float4 u = *reinterpret_cast<const float4*>(tr + 12 * TCH);
      T[0][0] = t.x; T[0][1] = t.y; T[0][2] = t.z; T[0][3] = t.w;
      U[0][0] = u.x; U[0][1] = u.y; U[0][2] = u.z; U[0][3] = u.w;
    }
#pragma unroll
    for (int si = 1; si < 4; ++si) {
      const int S = (si == 1) ? 2 : (si == 2) ? 3 : 6, bo = (si == 1) ? 1 : (si == 2) ? 3 : 6;
      int x0, x1;
      float lx;
      ctx_bil(S, x, a.W, x0, x1, lx);
      const float l0 = 1.f - lx;
      const float4 t0 = *reinterpret_cast<const float4*>(tr + (bo + x0) * TCH);
      const float4 t1 = *reinterpret_cast<const float4*>(tr + (bo + x1) * TCH);
      const float4 u0 = *reinterpret_cast<const float4*>(tr + (12 + bo + x0) * TCH);
      const float4 u1 = *reinterpret_cast<const float4*>(tr + (12 + bo + x1) * TCH);
      T[si][0] = l0 * t0.x + lx * t1.x; T[si][1] = l0 * t0.y + lx * t1.y;
      T[si][2] = l0 * t0.z + lx * t1.z; T[si][3] = l0 * t0.w + lx * t1.w;
      U[si][0] = l0 * u0.x + lx * u1.x; U[si][1] = l0 * u0.y + lx * u1.y;
      U[si][2] = l0 * u0.z + lx * u1.z; U[si][3] = l0 * u0.w + lx * u1.w;
    }
    float wv[16], fi[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float num = 0.f, den = 0.f;
#pragma unroll
      for (int si = 0; si < 4; ++si) {
        const float z = T[si][j] - acc[j][i][si];
        const float w = __builtin_amdgcn_rcpf(1.f + __expf(-z));   // v_rcp_f32 (1 ulp): the output is 16-bit
        wv[j * 4 + si] = w;
        num += w * U[si][j];
        den += w;
      }
      fi[j] = num * __builtin_amdgcn_rcpf(den + 1e-12f);
    }
    bf16_t* yo = a.y + (size_t)m * a.Cout + chb;
    *reinterpret_cast<uint4*>(yo) = pack8h<DT>(wv);
    *reinterpret_cast<uint4*>(yo + 8) = pack8h<DT>(wv + 8);
    bf16_t* co = a.cat + (size_t)m * 2 * C + c0;
    *reinterpret_cast<uint2*>(co) = fvw[i];
    *reinterpret_cast<uint2*>(co + C) = make_uint2(pack2<DT>(fi[0], fi[1]), pack2<DT>(fi[2], fi[3]));
  }
}

template <int DT, int WC, int WP, int PW>
__device__ __forceinline__ void ctxb_epilogue(const ConvArgs2& a, f32x4 (&acc)[4][4 * PW], const float* tab, int ct,
                                              int pt, int rlo, int wc, int wp, int fr, int fq) {
  constexpr int TP = 64 * PW * WP, NF = 4 * PW, HALF = 2, TC = 64 * WC;
  const int C = a.cC;
  const int cl = wc * 64 + fq * 16;                 // this lane's first channel in the tile
  const int chb = ct * TC + cl;
  // groups of 2 pixel fragments: the dcat / mask loads of a group are issued before its first store (more in
  // flight spills: the 128 accumulators are live throughout)
#pragma unroll
  for (int h = 0; h < NF / HALF; ++h) {
    uint4 g0[HALF], g1[HALF], k0[HALF], k1[HALF];
#pragma unroll
    for (int ii = 0; ii < HALF; ++ii) {
      const int m = pt * TP + wp * 64 * PW + (h * HALF + ii) * 16 + fr;
      g0[ii] = g1[ii] = k0[ii] = k1[ii] = make_uint4(0u, 0u, 0u, 0u);
      if (m < a.M) {
        const bf16_t* gp = a.cat + (size_t)m * 2 * C + chb;
        const bf16_t* kp = a.mask + (size_t)m * C + chb;
        g0[ii] = *reinterpret_cast<const uint4*>(gp);
        g1[ii] = *reinterpret_cast<const uint4*>(gp + 8);
        k0[ii] = *reinterpret_cast<const uint4*>(kp);
        k1[ii] = *reinterpret_cast<const uint4*>(kp + 8);
      }
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);           // vmcnt(0): only stores are outstanding below
#pragma unroll
    for (int ii = 0; ii < HALF; ++ii) {
      const int i = h * HALF + ii;
      const int m = pt * TP + wp * 64 * PW + i * 16 + fr;
      if (m >= a.M) continue;
      const int r = (int)fdiv((uint32_t)m, a.fdW), x = m - r * a.W;
      const float* tr = tab + (size_t)(r - rlo) * 12 * TC + cl;
      float v[16];
      unpack8h<DT>(g0[ii], v);
      unpack8h<DT>(g1[ii], v + 8);
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) v[j * 4 + rr] += acc[j][i][rr];
      auto add_bin = [&](int bin, float wgt) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float4 t = *reinterpret_cast<const float4*>(tr + bin * TC + q * 4);
          v[q * 4 + 0] += wgt * t.x; v[q * 4 + 1] += wgt * t.y; v[q * 4 + 2] += wgt * t.z; v[q * 4 + 3] += wgt * t.w;
        }
      };
      add_bin(0, 1.f);
#pragma unroll 1
      for (int si = 1; si < 4; ++si) {          // not unrolled: the hoisted table reads of 7 bins spill
        const int S = (si == 1) ? 2 : (si == 2) ? 3 : 6, bo = (si == 1) ? 1 : (si == 2) ? 3 : 6;
        int jA, jB;
        ctx_pool_cols(S, x, a.W, jA, jB);
        add_bin(bo + jA, 1.f);
        add_bin(bo + (jB >= 0 ? jB : jA), jB >= 0 ? 1.f : 0.f);
      }
      const unsigned mw[8] = {k0[ii].x, k0[ii].y, k0[ii].z, k0[ii].w, k1[ii].x, k1[ii].y, k1[ii].z, k1[ii].w};
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const unsigned short bits = (unsigned short)(mw[c >> 1] >> ((c & 1) * 16));
        v[c] = pos_bits(bits) ? v[c] : 0.f;
      }
      bf16_t* yo = a.y + (size_t)m * a.Cout + chb;
      *reinterpret_cast<uint4*>(yo) = pack8h<DT>(v);
      *reinterpret_cast<uint4*>(yo + 8) = pack8h<DT>(v + 8);
    }
  }
}

template <int DT, int WC, int WP, int PW, int EPI>
__global__ void __launch_bounds__(64 * WC * WP, 1) conv_glds_kernel(ConvArgs2 a) {
  constexpr int NW = WC * WP;
  constexpr int TC = 64 * WC, TP = 64 * PW * WP;
  constexpr int A_BYTES = TC * 128, B_BYTES = TP * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NIA = A_BYTES / 1024, NIB = B_BYTES / 1024;
  constexpr int G = (NIA + NIB) / NW;
  static_assert((NIA + NIB) % NW == 0, "instruction split");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wp = wave / WC;

  const int nct = a.Cout / TC;
  const int npt = (a.M + TP - 1) / TP;
  const int tile = xcd_remap(blockIdx.x, nct * npt);
  const int ct = tile % nct, pt = tile / nct;
  const int Ktot = a.ksize * a.ksize * a.Cin;
  const int cchunks = a.Cin >> 6;
  const int nk = a.ksize * a.ksize * cchunks;

  auto issue = [&](int ks, int buf) {
    const int tap = ks / cchunks;
    const int c0 = (ks - tap * cchunks) * 64;
    int dh = 0, dw = 0;
    if (a.ksize == 3) {
      const int kh = (tap * 11) >> 5;
      dh = (kh - 1) * a.dil;
      dw = (tap - kh * 3 - 1) * a.dil;
    }
    unsigned char* sbase = smem + buf * STAGE;
#pragma unroll
    for (int i = 0; i < G; ++i) {
      const int gi = wave + NW * i;
      const void* src = a.zero;
      unsigned char* dst;
      if (gi < NIA) {
        const int r = gi * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ (r & 7);
        src = a.w + (size_t)(ct * TC + perm_row(r)) * Ktot + ks * 64 + lc * 8;
        dst = sbase + gi * 1024;
      } else {
        const int r = (gi - NIA) * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ (r & 7);
        const int m = pt * TP + r;
        if (m < a.M) {
          const uint32_t q = fdiv((uint32_t)m, a.fdW);
          const int ow = m - (int)q * a.W;
          const int oh = (int)q - (int)fdiv(q, a.fdH) * a.H;
          const int ih = oh + dh, iw = ow + dw;
          if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
            src = a.x + (size_t)(m + dh * a.W + dw) * a.Cin + c0 + lc * 8;
        }
        dst = sbase + A_BYTES + (gi - NIA) * 1024;
      }
      glds16(src, lds_addr(dst));
    }
  };

  f32x4 acc[4][4 * PW];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4 * PW; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  issue(0, 0);
  for (int ks = 0; ks < nk; ++ks) {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (ks + 1 < nk) issue(ks + 1, (ks + 1) & 1);
    const uint4* As = reinterpret_cast<const uint4*>(smem + (ks & 1) * STAGE);
    const uint4* Bs = reinterpret_cast<const uint4*>(smem + (ks & 1) * STAGE + A_BYTES);
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int chunk = kk * 4 + fq;
      frag8_t af[4], bfr[4 * PW];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = wc * 64 + j * 16 + fr;
        af[j] = __builtin_bit_cast(frag8_t, As[row * 8 + swz(row, chunk)]);
      }
#pragma unroll
      for (int i = 0; i < 4 * PW; ++i) {
        const int row = wp * 64 * PW + i * 16 + fr;
        bfr[i] = __builtin_bit_cast(frag8_t, Bs[row * 8 + swz(row, chunk)]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4 * PW; ++i)
          acc[j][i] = mfma16<DT>(af[j], bfr[i], acc[j][i]);
    }
  }

  glds_epilogue<DT, WC, WP, PW, EPI>(a, acc, ct, pt, wc, wp, fr, fq);
}

// ===========================================================================
// v2 of the LDS-DMA kernel (same tiles, LDS image and epilogue):
//  * per-lane DMA addressing hoisted out of the K loop: each B (pixel) DMA
//    row keeps a 32-bit element offset and a 9-bit "tap in range" mask, the
//    per-stage part (tap shift, channel chunk) is wave-uniform scalar math —
//    no division or bounds arithmetic per stage;
//  * the A (weight) and B DMA instructions are split at compile time (no
//    uniform branches between DMA issues);
//  * fragment reads are software-pipelined across the barrier: the second
//    K half of stage s is read while the first half's MFMAs run, and the
//    first half of stage s+1 is read (right after the barrier) while the
//    second half's MFMAs run, so LDS read latency is never exposed at the
//    head of an MFMA burst.
// (A 4-wave layout of 128-channel waves, 8 A fragments each, measured 14-27 % slower per layer and was removed:
// with one wave per SIMD nothing covers the DMA issue and the stage barrier, profiles/r3/ab_glds_four_wave.txt.)
// ===========================================================================
template <int DT, int WC, int WP, int PW, int EPI>
__global__ void __launch_bounds__(64 * WC * WP, 1) conv_glds2_kernel(ConvArgs2 a) {
  constexpr int JW = 4;                           // 64-channel waves: 4 A fragments
  if (blockIdx.y) {                               // batched launch: item blockIdx.y
    a.x += blockIdx.y * a.xbs;
    a.w += blockIdx.y * a.wbs;
    a.y += blockIdx.y * a.ybs;
  }
  constexpr int NW = WC * WP;
  constexpr int TC = 16 * JW * WC, TP = 64 * PW * WP;
  constexpr int A_BYTES = TC * 128, B_BYTES = TP * 128;
  constexpr int STAGE = A_BYTES + B_BYTES;
  constexpr int NIA = A_BYTES / 1024, NIB = B_BYTES / 1024;
  constexpr int GA = NIA / NW, GB = NIB / NW;
  constexpr int JH = 1;
  static_assert(NIA % NW == 0 && NIB % NW == 0, "instruction split");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wp = wave / WC;

  const int nct = a.Cout / TC;
  const int npt = (a.M + TP - 1) / TP;
  const int tile = xcd_remap(blockIdx.x, nct * npt);
  const int ct = tile % nct, pt = tile / nct;
  const int Ktot = a.ksize * a.ksize * a.Cin;
  const int nk = a.ksize * a.ksize * (a.Cin >> 6);
  const int lc8 = ((lane & 7) ^ (lane >> 3)) * 8;     // swizzled 16-B chunk, in elements

  int aoff[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int r = (wave + NW * j) * 8 + (lane >> 3);
    aoff[j] = (ct * TC + perm_row(r)) * Ktot + lc8;
  }
  int boff[GB];
  // 9-bit tap-validity masks, three per VGPR (the 128 x 512 tile's 8 pieces per wave otherwise push the
  // kernel past 256 VGPRs into scratch)
  constexpr int NBM = (GB + 2) / 3;
  unsigned bmask[NBM];
#pragma unroll
  for (int j = 0; j < NBM; ++j) bmask[j] = 0u;
#pragma unroll
  for (int j = 0; j < GB; ++j) {
    const int r = (wave + NW * j) * 8 + (lane >> 3);
    const int m = tile_pix<TP, EPI>(a, pt, r);
    unsigned msk = 0;
    if (m < a.M) {
      const uint32_t q = fdiv((uint32_t)m, a.fdW);
      const int ow = m - (int)q * a.W;
      const int oh = (int)q - (int)fdiv(q, a.fdH) * a.H;
      if (a.ksize == 3) {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int ih = oh + (t / 3 - 1) * a.dil, iw = ow + (t % 3 - 1) * a.dil;
          if (ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) msk |= 1u << t;
        }
      } else {
        msk = 1u;
      }
    }
    boff[j] = m * a.Cin + lc8;
    bmask[j / 3] |= msk << (9 * (j % 3));
  }

  // stage -> (channel chunk, tap) advanced incrementally (scalar).  Stages run
  // chunk-major / tap-minor: the 9 taps of one 64-channel chunk are 9
  // consecutive stages over the same few activation rows, so the shifted
  // re-reads hit L2 (tap-major order re-fetched every activation row once
  // per tap from beyond L2: measured 25% L2 misses on the 512-ch layers).
  const int ntap = a.ksize * a.ksize;
  int i_tap = 0, i_c0 = 0;
  // one stage's DMA in PARTS parts (part p = pieces [p*GA/PARTS ..) of the weights, [p*GB/PARTS ..) of the
  // activations), issued between MFMA groups so the ~60-100-cycle issue cost of each LDS-DMA piece does not
  // stall both waves of a SIMD in one burst after the barrier
  constexpr int PARTS = (GA % 4 == 0 && GB % 4 == 0) ? 4 : 1;   // 2 parts measured slower (F5: +3..8%)
  auto issue_part = [&](int buf, int p) {
    int sh = 0;
    if (a.ksize == 3) {
      const int kh = (i_tap * 11) >> 5;
      sh = ((kh - 1) * a.W + (i_tap - kh * 3 - 1)) * a.dil * a.Cin;
    }
    sh += i_c0;
    const int i_k = i_tap * a.Cin + i_c0;
    unsigned char* sbase = smem + buf * STAGE;
#if defined(CAN_PROBE) && CAN_PROBE >= 2
    if (p == PARTS - 1 && ++i_tap == ntap) { i_tap = 0; i_c0 += 64; }
    return;
#endif
#pragma unroll
    for (int j = p * GA / PARTS; j < (p + 1) * GA / PARTS; ++j)
      glds16((const void*)(a.w + aoff[j] + i_k), lds_addr((sbase + (wave + NW * j) * 1024)));
#if defined(CAN_PROBE) && CAN_PROBE == 1
    if (p == PARTS - 1 && ++i_tap == ntap) { i_tap = 0; i_c0 += 64; }
    return;
#endif
#pragma unroll
    for (int j = p * GB / PARTS; j < (p + 1) * GB / PARTS; ++j) {
      const void* src = ((bmask[j / 3] >> (9 * (j % 3) + i_tap)) & 1u) ? (const void*)(a.x + boff[j] + sh) : (const void*)a.zero;
      glds16(src, lds_addr((sbase + A_BYTES + (wave + NW * j) * 1024)));
    }
    if (p == PARTS - 1 && ++i_tap == ntap) { i_tap = 0; i_c0 += 64; }
  };
  auto issue = [&](int buf) {
    int sh = 0;
    if (a.ksize == 3) {
      const int kh = (i_tap * 11) >> 5;
      sh = ((kh - 1) * a.W + (i_tap - kh * 3 - 1)) * a.dil * a.Cin;
    }
    sh += i_c0;
    const int i_k = i_tap * a.Cin + i_c0;
    unsigned char* sbase = smem + buf * STAGE;
#if defined(CAN_PROBE) && CAN_PROBE >= 2
    if (++i_tap == ntap) { i_tap = 0; i_c0 += 64; }
    return;
#endif
#pragma unroll
    for (int j = 0; j < GA; ++j)
      glds16((const void*)(a.w + aoff[j] + i_k), lds_addr((sbase + (wave + NW * j) * 1024)));
#if defined(CAN_PROBE) && CAN_PROBE == 1
    if (++i_tap == ntap) { i_tap = 0; i_c0 += 64; }
    return;
#endif
#pragma unroll
    for (int j = 0; j < GB; ++j) {
      const void* src = ((bmask[j / 3] >> (9 * (j % 3) + i_tap)) & 1u) ? (const void*)(a.x + boff[j] + sh) : (const void*)a.zero;
      glds16(src, lds_addr((sbase + A_BYTES + (wave + NW * j) * 1024)));
    }
    if (++i_tap == ntap) { i_tap = 0; i_c0 += 64; }
  };

  f32x4 acc[JH][4][4 * PW];
#pragma unroll
  for (int h = 0; h < JH; ++h)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int i = 0; i < 4 * PW; ++i) acc[h][j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto read = [&](int buf, int kk, frag8_t (&af)[JW], frag8_t (&bfr)[4 * PW]) {
    const uint4* As = reinterpret_cast<const uint4*>(smem + buf * STAGE);
    const uint4* Bs = reinterpret_cast<const uint4*>(smem + buf * STAGE + A_BYTES);
    const int chunk = kk * 4 + fq;
#if defined(CAN_PROBE) && CAN_PROBE >= 3
    for (int j = 0; j < JW; ++j) af[j] = __builtin_bit_cast(frag8_t, make_uint4(buf + lane, kk, j, 1));
    for (int i = 0; i < 4 * PW; ++i) bfr[i] = __builtin_bit_cast(frag8_t, make_uint4(buf, kk + lane, i, 1));
    return;
#endif
#pragma unroll
    for (int j = 0; j < JW; ++j) {
      const int row = wc * (16 * JW) + j * 16 + fr;
      af[j] = __builtin_bit_cast(frag8_t, As[row * 8 + swz(row, chunk)]);
    }
#pragma unroll
    for (int i = 0; i < 4 * PW; ++i) {
      const int row = wp * 64 * PW + i * 16 + fr;
      bfr[i] = __builtin_bit_cast(frag8_t, Bs[row * 8 + swz(row, chunk)]);
    }
  };
  // MFMAs over pixel fragments [i0, i1) (so the B fragments die in halves)
  auto mma = [&](const frag8_t (&af)[JW], const frag8_t (&bfr)[4 * PW], int i0, int i1) {
#pragma unroll
    for (int i = i0; i < i1; ++i)
#pragma unroll
      for (int j = 0; j < JW; ++j)
        acc[j >> 2][j & 3][i] = mfma16<DT>(af[j], bfr[i], acc[j >> 2][j & 3][i]);
  };

  frag8_t a0[JW], b0[4 * PW], a1[JW], b1[4 * PW];
  issue(0);
  // context epilogues: row tables beside the staging ring when the launch reserved room for them (a.cC flag bit),
  // visible after the first barrier below
  constexpr bool CTX = (EPI == EPI_CTXF || EPI == EPI_CTXB);
  constexpr int CTX_Q = CTX ? (5 * (EPI == EPI_CTXF ? 24 : 12) * ((EPI == EPI_CTXF ? TC / 4 : TC) / 4) + NW * 64 - 1) /
                                  (NW * 64)
                            : 1;
  const bool ctx_pro = CTX && a.ctx_prologue;
  if constexpr (CTX) {
    if (ctx_pro) {
      const int rlo = (pt * TP) / a.W, rhi = (min(a.M, (pt + 1) * TP) - 1) / a.W;
      ctx_build_tab<EPI, TC, NW * 64, CTX_Q>(a, reinterpret_cast<float*>(smem + 2 * STAGE), ct, rlo, rhi - rlo + 1);
    }
  }
  if (nk > 1) {
    issue(1);
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" :: "n"(GA + GB) : "memory");
  } else {
    asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  }
  read(0, 0, a0, b0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  for (int s = 0; s < nk - 1; ++s) {
    const int buf = s & 1;
    read(buf, 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0, b0, 0, 4 * PW);
    // this wave's reads of stage s are in registers, stage s+1 has landed
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0x0070);
#if !defined(CAN_PROBE) || CAN_PROBE < 4
    asm volatile("s_barrier" ::: "memory");
#endif
    __builtin_amdgcn_sched_barrier(0);
#ifndef CANNET_DMA_BURST
    if constexpr (PARTS > 1) {
      // the four MFMA groups of the second K half, DMA parts of stage s+2 between them, the reads of stage
      // s+1's first half after the second group
      const bool more = s + 2 < nk;
      constexpr int ord = CANNET_DMA_ORDER_CONV;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        if (ord == 0 && more) issue_part(buf, g);
        __builtin_amdgcn_sched_barrier(0);
        mma(a1, b1, g * PW, (g + 1) * PW);
        __builtin_amdgcn_sched_barrier(0);
        if (ord != 0 && more && (ord == 1 || g < 3)) {
          issue_part(buf, g);
          if (ord == 2 && g == 2) issue_part(buf, 3);
        }
        __builtin_amdgcn_sched_barrier(0);
        if (g == 1) read(buf ^ 1, 0, a0, b0);
        __builtin_amdgcn_sched_barrier(0);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      continue;
    }
#endif
    if (s + 2 < nk) issue(buf);
    __builtin_amdgcn_sched_barrier(0);
    // half of the second-half MFMAs first (their operands are complete, so
    // any counter wait the compiler places here is free), then the reads of
    // stage s+1's first half, hidden behind the other half
    mma(a1, b1, 0, 2 * PW);
    __builtin_amdgcn_sched_barrier(0);
    read(buf ^ 1, 0, a0, b0);
    __builtin_amdgcn_sched_barrier(0);
    mma(a1, b1, 2 * PW, 4 * PW);
    // the first-half reads have long landed; a visible lgkmcnt(0) keeps the
    // compiler's counter model exact at the loop head
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  read((nk - 1) & 1, 1, a1, b1);
  mma(a0, b0, 0, 4 * PW);
  mma(a1, b1, 0, 4 * PW);
  if constexpr (CTX) {
    const int rlo = (pt * TP) / a.W;
    const int rhi = (min(a.M, (pt + 1) * TP) - 1) / a.W;
    float* tab = reinterpret_cast<float*>(smem + (ctx_pro ? 2 * STAGE : 0));
    if (!ctx_pro) {
      // the staging LDS is free once every wave's last fragment reads are done
      __syncthreads();
      ctx_build_tab<EPI, TC, NW * 64, CTX_Q>(a, tab, ct, rlo, rhi - rlo + 1);
      __syncthreads();
    }
    if constexpr (EPI == EPI_CTXF) ctxf_epilogue<DT, WC, WP, PW>(a, acc[0], tab, ct, pt, rlo, wc, wp, fr, fq);
    else ctxb_epilogue<DT, WC, WP, PW>(a, acc[0], tab, ct, pt, rlo, wc, wp, fr, fq);
    return;
  } else {
    glds_epilogue<DT, WC, WP, PW, EPI>(a, acc[0], ct, pt, wc, wp, fr, fq);
  }
}

template <int DT, int WC, int WP, int PW, int EPI>
static int launch_glds2(const ConvArgs2& a, hipStream_t s, int nb = 1) {
  constexpr int TC = 64 * WC, TP = 64 * PW * WP;
  size_t lds = 2 * (size_t)(TC + TP) * 128;
  ConvArgs2 b = a;
  if (EPI == EPI_CTXF || EPI == EPI_CTXB) {
    // room for the context row tables beside the ring when it fits one CU's LDS (else: built after the main loop)
    const size_t tab = (size_t)ctx_tab_row_bytes(EPI, TC) * ctx_max_rows(TP, a.W);
    b.ctx_prologue = (lds + tab <= 160 * 1024) ? 1 : 0;
    if (b.ctx_prologue) lds += tab;
    else if ((size_t)ctx_tab_row_bytes(EPI, TC) * ctx_max_rows(TP, a.W) > lds) return -15;
  }
  auto kfn = conv_glds2_kernel<DT, WC, WP, PW, EPI>;
  static size_t attr_lds = 0;
  if (lds > attr_lds) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr_lds = lds;
  }
  const int nct = a.Cout / TC, npt = (a.M + TP - 1) / TP;
  hipLaunchKernelGGL(kfn, dim3(nct * npt, nb), dim3(64 * WC * WP), lds, s, b);
  return (int)hipGetLastError();
}

// ===========================================================================
// Row-ring 3x3 conv (forward / data gradient; cfg 27): the 256 x 256 tile of conv_glds2 (8 waves of 64 channels x
// 128 pixels, same MFMA order, same epilogue) with the activation operand staged once per input ROW instead of once
// per tap.  A pixel tile is 2 image rows x 128 columns (a ragged last column block / tile row is masked: its DMA
// reads the zero page, its epilogue skips the pixels); for one 64-channel chunk its 9 taps
// read only 2 + 2 * dil input rows, each a 128-column row plus an 8-pixel guard on both sides.  The rows sit in a
// 4-slot LDS ring (18 KB each) beside the 2-stage weight ring: a row is DMA'd two stages ahead of its first tap
// (with that stage's weights) into the slot of the row whose last tap is already in registers, and every tap reads
// its shifted window from the row slots (chunk swizzle keyed on the slot pixel, conflict-free for any shift).
// LDS-DMA per 64-deep stage: 32 KB weights + 7.1 (dil 1) / 10.7 (dil 2) KB of rows instead of 32 + 32 KB; the
// weight and row pieces are issued between the MFMA groups like conv_glds2's.  Out-of-image rows and columns come
// from the zero page (guards of a one-block-wide map are zeroed once).  Results are bitwise those of cfg 21.
// ===========================================================================
constexpr int RR_SLOT = 144 * 128;                         // 8-px guard | 128 columns | 8-px guard, 64 channels
// LDS of a row-ring config: 2 weight stages + the row slots (TC = 256, 2-row tiles: 4 slots, 139,264 B; TC = 64,
// 4-row tiles: 8 slots, 163,840 B = all of a CU's LDS)
__host__ __device__ constexpr int rr_ring(int TR) { return TR == 2 ? 4 : 8; }
__host__ __device__ constexpr int rr_lds(int TC, int TR) { return 2 * TC * 128 + rr_ring(TR) * RR_SLOT; }

// TC x (TR x 128) tiles: (256, 2) = cfg 27 (the 256 x 256 conv_glds2 tile, bitwise cfg 21), (64, 4) = cfg 28 (the
// 64 x 512 tile of cfg 23, bitwise cfg 23: 8 waves of 64 channels x 64 pixels, two per tile row).  A 4-row tile's
// chunk needs 4 + 2 * dil rows and its rows 2, 3 stay live to the chunk's last tap, so it runs 8 slots and issues a
// row 2 stages ahead with a full drain per stage (LEAD = 2); the 2-row tile runs 4 slots, LEAD 3 or 4, counted waits.
// RG: a ragged map (W % 128 != 0 or H % TR != 0), its own instantiation so the aligned one keeps the cheaper
// cross-image tile decode (and its SGPR budget: the per-image decode of both in one kernel spilled SGPRs)
template <int DT, int EPI, int D, int LEAD = 3, int TC = 256, int TR = 2, bool RG = false>
__global__ void __launch_bounds__(512, 1) conv_rring_kernel(ConvArgs2 a) {
  static_assert(((TC == 256 || TC == 128) && TR == 2 && LEAD >= 3 && LEAD <= 4) || (TC == 64 && TR == 4 && LEAD == 2),
                "row-ring configs: 256 x (2 x 128) with a 3- or 4-stage row lead (counted barrier waits need >= 3, 4 slots "
                "allow <= 4); 64 x (4 x 128) with a 2-stage lead and a full drain");
  static_assert(D == 1 || D == 2, "dilation 1 or 2");
  static_assert(EPI != EPI_CTXF && EPI != EPI_CTXB, "row-ring epilogues");
  // EPI_POOLFWD: 2-row tiles of an aligned map, dilation 1; every wave computes both rows of its columns
  constexpr bool PL = (EPI == EPI_POOLFWD);
  static_assert(!PL || (TR == 2 && !RG && D == 1), "fused max-pool: aligned 2-row tiles");
  constexpr int NW = 8, WC = TC / 64, WP = NW / WC;
  constexpr int TP = 128 * TR, PW = TP / (64 * WP);  // pixel fragments per wave / 4
  constexpr int WPR = WP / TR;                       // waves per tile row
  constexpr int A_BYTES = TC * 128;
  constexpr int GA = A_BYTES / 1024 / NW;            // weight pieces per wave per stage (4 or 1)
  constexpr int NR = TR + 2 * D;                     // input rows of a tile per channel chunk
  constexpr int RING = rr_ring(TR);
  static_assert(PW >= 1 && WPR >= 1 && (GA == 4 || GA == 2 || GA == 1), "row-ring tile");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* ring = smem + 2 * A_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave % WC, wp = wave / WC;
  const int rt = wp / WPR;                           // the tile row this wave computes
  const int cbw = (wp - rt * WPR) * 64 * PW;         // and its first column in the tile

  const int tx = RG ? a.rr_tx : (a.W >> 7);                  // ceil(W / 128) column blocks
  const int nct = a.Cout / TC;
  const int npt = RG ? a.rr_np : a.M / TP;
  const int tile = xcd_remap(blockIdx.x, nct * npt);
  const int ct = tile % nct, pt = tile / nct;
  const int q = pt / tx, cb = pt - q * tx;
  int oh0, grow0;                                             // grow0 = n * H + oh0
  if constexpr (RG) {
    const int nimg = q / a.rr_ty;
    oh0 = TR * (q - nimg * a.rr_ty);
    grow0 = nimg * a.H + oh0;
  } else {
    grow0 = TR * q;
    oh0 = grow0 - (int)fdiv((uint32_t)grow0, a.fdH) * a.H;
  }
  const int col0 = cb * 128;
  // a ragged last column block (W % 128 != 0): interior / guard pixels at or beyond W come from the zero page
  const bool ragged_w = RG && (a.W & 127) != 0;
  const int Ktot = 9 * a.Cin;
  const int nc = a.Cin >> 6, nk = 9 * nc;
  const int lc8 = ((lane & 7) ^ (lane >> 3)) * 8;             // swizzled 16-B chunk (pieces are 8-pixel aligned)

  int aoff[GA];
#pragma unroll
  for (int j = 0; j < GA; ++j) {
    const int r = (wave + NW * j) * 8 + (lane >> 3);
    aoff[j] = (ct * TC + perm_row(r)) * Ktot + lc8;
  }
  const int boff = (lane >> 3) * a.Cin + lc8;                 // lane's pixel / chunk inside a row piece

  if (tx == 1) {
    // the guards of a one-block-wide map are always zero padding: written once (slots x 16 pixels x 8 chunks)
    for (int e = tid; e < RING * 128; e += NW * 64) {
      const int sl = e >> 7, g = (e >> 3) & 15;
      reinterpret_cast<uint4*>(ring + sl * RR_SLOT + ((g < 8) ? g : 128 + g) * 128)[e & 7] = make_uint4(0u, 0u, 0u, 0u);
    }
  }

  // stage s = 9 * chunk + tap (chunk-major, tap-minor: conv_glds2's k order).  The weights of stage s are issued two
  // stages ahead (in the stage-(s-2) MFMA gaps, like conv_glds2), the rows whose first tap is stage f LEAD stages
  // ahead, after that stage's weights: with LEAD >= 3 the barrier wait before stage s + 1 counts only the row pieces
  // just issued (vmcnt retires in order), so a row has LEAD - 1 stages to arrive (a first-touch row comes from beyond
  // L2; with LEAD = 2 and a full vmcnt drain per stage the 2-row kernel waited on them).  Row r of chunk c (input row
  // oh0 - D + r) is first read by tap 0 (rows 0 .. TR - 1), 3 (the next D) or 6 (the last D) and last read by the
  // last tap of the highest kh whose window holds it; with the ring sizes above every slot's previous row has had its
  // last tap at or before the issuing stage, whose fragments are in registers once its barrier passed.
  auto issue_A = [&](int st, int buf, int p) {
#if defined(CAN_PROBE) && CAN_PROBE == 5
    return;                                  // diagnostic build (scripts/probe): no weight DMA in the row ring
#endif
    const int c = st / 9, tap = st - 9 * c;
    glds16((const void*)(a.w + aoff[p] + tap * a.Cin + c * 64), lds_addr(smem + buf * A_BYTES + (wave + NW * p) * 1024));
  };
  auto rows_at = [&](int tap) -> int { return (tap == 0) ? TR : (tap == 3 || tap == 6) ? D : 0; };
  // row pieces this wave issues for the rows first read by stage f (0 when f is past the end)
  auto row_pieces = [&](int f) -> int {
    const int c = f / 9, tap = f - 9 * c;
    const int nr = (c >= nc) ? 0 : rows_at(tap);
    return nr * (2 + ((tx > 1 && wave < 2) ? 1 : 0));
  };
  auto issue_rows = [&](int f) {
#if defined(CAN_PROBE) && CAN_PROBE == 6
    return;                                  // diagnostic build (scripts/probe): no row DMA in the row ring
#endif
    const int c = f / 9, tap = f - 9 * c;
    const int nr = (c >= nc) ? 0 : rows_at(tap);
    for (int k = 0; k < nr; ++k) {
      const int r = ((tap == 0) ? 0 : (tap == 3) ? TR : TR + D) + k;
      const int ih = oh0 - D + r;
      const bool rv = (unsigned)ih < (unsigned)a.H;
      unsigned char* slot = ring + ((c * NR + r) & (RING - 1)) * RR_SLOT;
      const size_t rbase = ((size_t)(grow0 - D + r) * a.W + col0) * a.Cin + c * 64;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int j = wave + NW * h;                           // interior piece: pixels 8j .. 8j + 7
        // wave-uniform: a ragged width is a multiple of 8 (rring_width_ok), so a piece is wholly in or out.  Keep
        // it so: with a lane-divergent condition here hipcc (ROCm 7.2) merged the two sources of the select into
        // one wave-uniform base plus a per-lane offset, and masked lanes read x + rbase + 8 * lane instead of the
        // zero page (out of bounds on the first / last row of the map)
        const bool cv = !ragged_w || col0 + 8 * j < a.W;
        glds16((rv && cv) ? (const void*)(a.x + rbase + (size_t)(8 * j) * a.Cin + boff)
                          : (const void*)(a.zero + lane * 8),
               lds_addr(slot + (j + 1) * 1024));
      }
      if (tx > 1 && wave < 2) {
        // 8-pixel guards of an interior column block: real pixels of the neighbouring blocks (wave 0 left, 1 right;
        // a right neighbour block starts below W, and W % 8 == 0 puts its whole guard piece inside the map)
        const bool gv = rv && (wave == 0 ? cb > 0 : cb + 1 < tx);
        const long long gc = (wave == 0) ? -8 : 128;
        glds16(gv ? (const void*)(a.x + (long long)rbase + gc * a.Cin + boff) : (const void*)(a.zero + lane * 8),
               lds_addr(slot + (wave == 0 ? 0 : 17) * 1024));
      }
    }
  };
  // s_waitcnt vmcnt(n) for a wave-uniform run-time n (the row pieces issued after the weights)
  auto wait_vm = [&](int n) {
    switch (n) {
      case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
      case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
      case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
      case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
      case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
      case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
      default: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    }
  };

  f32x4 acc[4][4 * PW];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4 * PW; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fq = lane >> 4;
  auto read = [&](int st, int kk, frag8_t (&af)[4], frag8_t (&bfr)[4 * PW]) {
    const uint4* As = reinterpret_cast<const uint4*>(smem + (st & 1) * A_BYTES);
    const int chunk = kk * 4 + fq;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = wc * 64 + j * 16 + fr;
      af[j] = __builtin_bit_cast(frag8_t, As[row * 8 + swz(row, chunk)]);
    }
    const int c = st / 9, tap = st - 9 * c, kh = (tap * 11) >> 5, kw = tap - 3 * kh;
    if constexpr (PL) {
      // fragment i: columns 8 i .. 8 i + 7 of the wave's 32 PW, lanes 0-7 tile row 0, 8-15 row 1 (tile_pix)
      const int hp = 8 + wp * 32 * PW + (fr & 7) + (kw - 1) * D;
      const unsigned char* base =
          ring + ((c * NR + kh * D + (fr >> 3)) & (RING - 1)) * RR_SLOT + hp * 128 + ((chunk ^ (hp & 7)) << 4);
#pragma unroll
      for (int i = 0; i < 4 * PW; ++i)
        bfr[i] = __builtin_bit_cast(frag8_t, *reinterpret_cast<const uint4*>(base + i * 1024));
    } else {
      const int hp = 8 + cbw + fr + (kw - 1) * D;    // slot pixel of this lane's column in fragment 0
      const unsigned char* base =
          ring + ((c * NR + kh * D + rt) & (RING - 1)) * RR_SLOT + hp * 128 + ((chunk ^ (hp & 7)) << 4);
#pragma unroll
      for (int i = 0; i < 4 * PW; ++i)
        bfr[i] = __builtin_bit_cast(frag8_t, *reinterpret_cast<const uint4*>(base + i * 2048));
    }
  };
  auto mma = [&](const frag8_t (&af)[4], const frag8_t (&bfr)[4 * PW], int i0, int i1) {
#pragma unroll
    for (int i = i0; i < i1; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j][i] = mfma16<DT>(af[j], bfr[i], acc[j][i]);
  };

  frag8_t a0[4], b0[4 * PW], a1[4], b1[4 * PW];
  // prologue: every row first read before stage LEAD, the weights of stages 0 and 1, then a full drain
#pragma unroll
  for (int f = 0; f < LEAD; ++f) issue_rows(f);
#pragma unroll
  for (int p = 0; p < GA; ++p) issue_A(0, 0, p);
  if (nk > 1) {
#pragma unroll
    for (int p = 0; p < GA; ++p) issue_A(1, 1, p);
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  read(0, 0, a0, b0);
  __builtin_amdgcn_s_waitcnt(0xC07F);
  int rp_prev = 0;               // row pieces issued after the weights in the previous stage (still in flight)
  for (int s = 0; s < nk - 1; ++s) {
    const int buf = s & 1;
    read(s, 1, a1, b1);
    __builtin_amdgcn_sched_barrier(0);
    mma(a0, b0, 0, 4 * PW);
    // this wave's reads of stage s are in registers; stage s + 1 (weights, rows) has landed: everything but the
    // row pieces issued last stage (LEAD >= 3) / everything (LEAD = 2)
    __builtin_amdgcn_sched_barrier(0);
    wait_vm(rp_prev);
    __builtin_amdgcn_s_waitcnt(0xC07F);
    asm volatile("s_barrier" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const bool more = s + 2 < nk;
    constexpr int ord = CANNET_DMA_ORDER_RR;
    // part p = weight piece p (GA = 4; GA = 2 / 1: parts 0 .. GA - 1), the rows after part 3, placed per
    // CANNET_DMA_ORDER_RR (common.h)
    auto part = [&](int p) {
      if (more && p < GA) issue_A(s + 2, buf, p);
      if (p == 3) {
        issue_rows(s + LEAD);
        rp_prev = (LEAD >= 3) ? row_pieces(s + LEAD) : 0;
      }
    };
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      if (ord == 0) part(g);
      __builtin_amdgcn_sched_barrier(0);
      mma(a1, b1, g * PW, (g + 1) * PW);
      __builtin_amdgcn_sched_barrier(0);
      if (ord != 0 && (ord == 1 || g < 3)) {
        part(g);
        if (ord == 2 && g == 2) part(3);
      }
      __builtin_amdgcn_sched_barrier(0);
      if (g == 1) read(s + 1, 0, a0, b0);
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
  }
  read(nk - 1, 1, a1, b1);
  mma(a0, b0, 0, 4 * PW);
  mma(a1, b1, 0, 4 * PW);
  glds_epilogue<DT, WC, WP, PW, EPI, TR, RG>(a, acc, ct, pt, wc, wp, fr, fq);
}

// column-block utilisation of the row ring on a ragged width: W / (ceil(W / 128) * 128) >= 0.7 (W = 240, 480,
// 960: 94 %); below it (W = 135: 53 %) the per-tap LDS-DMA kernel, whose pixel tiles run across rows, wastes less.
// A ragged width must be a multiple of 8: the row DMA's validity is then uniform per 8-pixel piece (see issue_rows)
static bool rring_width_ok(int W) {
  if (W % 128 == 0) return true;
  const int tx = (W + 127) / 128;
  return W % 8 == 0 && W >= 96 && 10 * W >= 7 * 128 * tx;
}
// pixel tiles of the row ring: N * ceil(H / TR) * ceil(W / 128) (ragged last tile row / column block masked)
static int rr_np(int H, int W, int M, int TR) {
  return (M / (H * W)) * ((H + TR - 1) / TR) * ((W + 127) / 128);
}
// the row-ring kernel applies: 3x3, dilation 1 / 2, a width the column blocks cover well (rring_width_ok); Cout % 256
// == 0 (cfg 27, 2-row tiles), Cout % 128 (cfg 29) or Cout == 64 (cfg 28, 4-row tiles); 0 = not applicable
static int rring_cfg(int H, int W, int Cin, int Cout, int ksize, int dil, int epi) {
  if (ksize != 3 || (dil != 1 && dil != 2) || !rring_width_ok(W) || Cin % 64 || epi == EPI_POOLFWD ||
      epi == EPI_SIGMOID || epi == EPI_CTXF || epi == EPI_CTXB)
    return 0;
  if (Cout % 256 == 0) return 27;
  // cfg 29 (128 x (2 x 128), the wave tile of cfg 22): dispatch rring128 = 1 (default) for the dilation-1 cfg-22
  // layers (K > 1152: conv3_1's data gradient 0.270 -> 0.253 ms), = 2 also for the cfg-25 ones (128 x 512 tiles,
  // K <= 1152: conv2_2 +2 %), = 3 also dilation 2 (backend.8 forward +10 %); 0 = off (profiles/r3/ab_rring128.txt)
  const int m128 = g_dispatch.rring128;
  if (Cout % 128 == 0 && Cout % 256 != 0 && m128 >= ((9 * Cin > 1152) ? 1 : 2) && (dil == 1 || m128 >= 3))
    return 29;
  // cfg 28 (dispatch rring64 = 0: off): conv2_1's data gradient 0.435 -> 0.347 ms isolated, step 487.3 -> 489.9
  // img/s (profiles/r3/ab_dma_order.txt)
  if (Cout == 64 && g_dispatch.rring64) return 28;
  return 0;
}
// dispatch rring: 0 = off, 1 = dilation-1 layers, 2 (default) = every dilation.  With the after-group DMA placement
// (CANNET_DMA_ORDER_RR = 1) the dilation-2 layers gain too: step 497.0 -> 501.3 img/s (profiles/r3/ab_rring128.txt).
// Before that placement, per layer at batch 8 x 768 x 1024
// (profiles/r3/ab_rring.txt) -2..-6 % vs cfg 21 with the rows issued 3 stages ahead (issued 2 ahead with a full
// DMA drain per stage: dilation 1 -1..-4 %, dilation 2 +1..+7 %); the step: off 482.6, dilation 1 485.4, every
// dilation 484.9 img/s (medians of 4 interleaved rounds)
static int rring_mode() { return g_dispatch.rring; }

template <int DT, int EPI, int TC, int TR, int LEAD, int D, bool RG>
static int launch_rring_rg(const ConvArgs2& a, hipStream_t s) {
  auto kfn = conv_rring_kernel<DT, EPI, D, LEAD, TC, TR, RG>;
  static bool attr = false;
  if (!attr) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, rr_lds(TC, TR)));
    attr = true;
  }
  ConvArgs2 b = a;
  b.rr_tx = (a.W + 127) / 128;
  b.rr_ty = (a.H + TR - 1) / TR;
  b.rr_np = rr_np(a.H, a.W, a.M, TR);
  hipLaunchKernelGGL(kfn, dim3((a.Cout / TC) * b.rr_np), dim3(512), rr_lds(TC, TR), s, b);
  return (int)hipGetLastError();
}
template <int DT, int EPI, int TC, int TR, int LEAD, int D>
static int launch_rring_one(const ConvArgs2& a, hipStream_t s) {
  if (a.W % 128 == 0 && a.H % TR == 0) return launch_rring_rg<DT, EPI, TC, TR, LEAD, D, false>(a, s);
  return launch_rring_rg<DT, EPI, TC, TR, LEAD, D, true>(a, s);
}

template <int DT, int EPI>
static int launch_rring(const ConvArgs2& a, hipStream_t s, int cfg) {
  if constexpr (EPI == EPI_POOLFWD || EPI == EPI_SIGMOID || EPI == EPI_CTXF || EPI == EPI_CTXB) {
    return -16;
  } else {
    if (rring_cfg(a.H, a.W, a.Cin, a.Cout, a.ksize, a.dil, EPI) != cfg) return -16;
    if (cfg == 28)
      return a.dil == 1 ? launch_rring_one<DT, EPI, 64, 4, 2, 1>(a, s) : launch_rring_one<DT, EPI, 64, 4, 2, 2>(a, s);
    if (cfg == 29)
      return a.dil == 1 ? launch_rring_one<DT, EPI, 128, 2, 3, 1>(a, s) : launch_rring_one<DT, EPI, 128, 2, 3, 2>(a, s);
    // rows are issued 3 stages ahead of their first tap (per layer 0.4 % ahead of 4, profiles/r3/ab_rring.txt)
    if (a.dil == 1) return launch_rring_one<DT, EPI, 256, 2, 3, 1>(a, s);
    return launch_rring_one<DT, EPI, 256, 2, 3, 2>(a, s);
  }
}

// ===========================================================================
// Halo-tiled 3x3 / dilation-1 conv for Cin = 64 (conv1_2 fwd + dgrad, conv2_1
// fwd: the 768x1024 / 384x512 layers).  The generic kernel streams the
// activation once per tap (9x re-reads, ~7 GB of LDS-DMA for conv1_2 at
// batch 8); here a block stages the (4+2) x (128+2) input halo of its
// 4 x 128 output tile ONCE (97.5 KB, XOR-swizzled per pixel; conflict-free
// for any column shift) and every tap reads its shifted window from it.
// Weights stream per tap through a 3-slot LDS ring (tap t+2 loads while tap t
// computes).  Waves: CO = 64 -> 8 waves = 4 rows x 2 column halves (64 co x
// 64 px each); CO = 128 -> 8 waves = 4 rows x 2 channel halves (64 co x 128 px).
// ===========================================================================
struct HaloConvArgs {
  const bf16_t* x;
  const bf16_t* w;      // packed [CO][9*64] (fwd or dgrad pack)
  const float* bias;
  const bf16_t* mask;
  bf16_t* y;
  const bf16_t* zero;
  int N, H, W, tiles_x, tiles_y;
  // conv_ws64_kernel<.., EPI_MASK, W1G>: the NHWC4 network input
  const bf16_t* img = nullptr;
  // EPI_POOLFWD (CO = 64, TCOL = 64; H % 4 == 0, W % 64 == 0): the 2x2/s2 max-pool of the output tile
  // -> yp [N][H/2][W/2][64], its max-pool codes -> codes [N][H/2][W/2][8] (optional), y optional
  bf16_t* yp = nullptr;
  uint32_t* codes = nullptr;
  // EPI_MASK: bias-gradient partials of the produced dY, [ntile * rows per tile][CO] fp32
  float* bpart = nullptr;
  // conv_ws64_kernel<.., EPI_MASK, W1G>: conv1_1's weight gradient from the dY tile it just produced (from
  // img): per-block partial slabs w1slab [2 * grid][36][64] (k = tap*4 + c) and
  // w1bslab [2 * grid][64] (bias), reduced by the first-layer slab reduction; y may be null (dY not stored)
  float* w1slab = nullptr;
  float* w1bslab = nullptr;
};

template <int DT, int CO, int EPI, int TCOL>
__global__ void __launch_bounds__((CO == 64 && TCOL == 64) ? 256 : 512, (TCOL == 64) ? 2 : 1)
conv_halo64_kernel(HaloConvArgs a) {
  constexpr int TR = 4, HR = TR + 2, HC = TCOL + 2;
  constexpr int NW = (CO == 64 && TCOL == 64) ? 4 : 8; // waves
  constexpr int HPIX = HR * HC;                       // 780 halo pixels (TCOL 128)
  constexpr int NHI = (HPIX + 7) / 8;                 // 98 one-KiB DMA pieces
  constexpr int HALO_BYTES = NHI * 1024;
  constexpr int WTAP = CO * 128;                      // one tap of weights: CO rows x 64 ci
  constexpr int GW = WTAP / 1024 / NW;                // weight DMA pieces per wave per tap
  constexpr int PW = CO / 64;                         // pixel fragments per wave / 4
  static_assert(GW >= 1, "weights split");
  static_assert(TCOL == 128 || (TCOL == 64 && CO == 64), "tile");
  static_assert(EPI != EPI_POOLFWD || (CO == 64 && TCOL == 64), "fused pool: conv1_2 64-column tiles");

  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned char* halo = smem;
  unsigned char* wring = smem + HALO_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);

  const int ntile = a.N * a.tiles_y * a.tiles_x;
  const int tile = xcd_remap(blockIdx.x, ntile);
  const int tx = tile % a.tiles_x;
  const int ty = (tile / a.tiles_x) % a.tiles_y;
  const int n = tile / (a.tiles_x * a.tiles_y);
  const int oh0 = ty * TR, ow0 = tx * TCOL;

  // ---- halo DMA (once): piece i covers halo pixels 8i..8i+7
  for (int i = wave; i < NHI; i += NW) {
    const int hp = i * 8 + (lane >> 3);
    const int hr = hp / HC, hc = hp - hr * HC;
    const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
    const void* src = a.zero;
    if (hp < HPIX && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W)
      src = a.x + ((size_t)(n * a.H + ih) * a.W + iw) * 64 + (((lane & 7) ^ (hc & 7)) * 8);
    glds16(src, lds_addr((halo + i * 1024)));
  }
  auto issue_w = [&](int t) {
    unsigned char* dst = wring + (t % 3) * WTAP;
#pragma unroll
    for (int j = 0; j < GW; ++j) {
      const int r = (wave + NW * j) * 8 + (lane >> 3);
      const int lc = (lane & 7) ^ (r & 7);
      glds16((const void*)(a.w + (size_t)perm_row(r) * 576 + t * 64 + lc * 8), lds_addr((dst + (wave + NW * j) * 1024)));
    }
  };
  issue_w(0);
  issue_w(1);
  const int fr = lane & 15, fq = lane >> 4;

  // wave -> (row, co half / column half)
  const int r = (NW == 4) ? wave : (wave >> 1);
  const int wc = (CO == 128) ? (wave & 1) : 0;
  const int colbase = (CO == 128 || NW == 4) ? 0 : (wave & 1) * 64;
  f32x4 acc[4][4 * PW];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int i = 0; i < 4 * PW; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};

  // Per-lane LDS byte offsets, loop invariant: the halo swizzle is keyed by the
  // halo COLUMN (hc & 7 = (fr + kw) & 7 for every fragment and row), so each
  // fragment read is one ds_read_b128 at lane offset + compile-time immediate.
  int hoff[3][2], woff[2];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      hoff[kw][kk] = (r * HC + colbase + fr + kw) * 128 + (((kk * 4 + fq) ^ ((fr + kw) & 7)) * 16);
#pragma unroll
  for (int kk = 0; kk < 2; ++kk) woff[kk] = (wc * 64 + fr) * 128 + (((kk * 4 + fq) ^ (fr & 7)) * 16);
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    // tap t's weights (and, for t = 0, the halo) have landed; the ring slot of
    // tap t-1 is free once every wave is past this barrier WITH its tap t-1 LDS
    // reads completed (lgkmcnt(0)): an issued-but-unreturned ds_read of the slot
    // can otherwise be overtaken by the tap t+2 DMA another wave issues next
    if (t + 1 < 9) asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" :: "n"(GW) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (t + 2 < 9) issue_w(t + 2);
    const int kh = t / 3, kw = t % 3;
    const unsigned char* Ab = wring + (t % 3) * WTAP;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      frag8_t af[4], bfr[4 * PW];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        af[j] = __builtin_bit_cast(frag8_t, *reinterpret_cast<const uint4*>(Ab + woff[kk] + j * 2048));
#pragma unroll
      for (int i = 0; i < 4 * PW; ++i)
        bfr[i] = __builtin_bit_cast(frag8_t,
                                    *reinterpret_cast<const uint4*>(halo + hoff[kw][kk] + kh * HC * 128 + i * 2048));
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int i = 0; i < 4 * PW; ++i)
          acc[j][i] = mfma16<DT>(af[j], bfr[i], acc[j][i]);
    }
  }

  // ---- epilogue: lane owns 16 consecutive channels of one pixel per fragment
  const int oh = oh0 + r;
  const int chb = wc * 64 + fq * 16;
  constexpr bool BPART = (EPI == EPI_MASK);
  // bias partials: row = tile * (NW * 64 / CO) + this wave's (row, column-half) slot, written even by a
  // wave whose row is outside the image (zeros)
  float bs[16];
#pragma unroll
  for (int c = 0; c < 16; ++c) bs[c] = 0.f;
  auto flush_bias = [&]() {
    if constexpr (BPART) {
      if (a.bpart != nullptr)
        store_bias_partials(bs, a.bpart + ((size_t)tile * (NW * 64 / CO) + wave / (CO / 64)) * CO + chb, fr);
    }
  };
  // fused pool: every wave's tap reads are done before the halo region becomes the output staging tile
  // (the host guarantees full tiles, so no wave leaves before the barriers)
  if constexpr (EPI == EPI_POOLFWD) __syncthreads();
  if (oh >= a.H) {
    flush_bias();
    return;
  }
  float bias[16];
  if (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_POOLFWD) {
#pragma unroll
    for (int c = 0; c < 16; c += 4) {
      const float4 b4 = *reinterpret_cast<const float4*>(a.bias + chb + c);
      bias[c] = b4.x; bias[c + 1] = b4.y; bias[c + 2] = b4.z; bias[c + 3] = b4.w;
    }
  }
#pragma unroll
  for (int i = 0; i < 4 * PW; ++i) {
    const int ow = ow0 + colbase + i * 16 + fr;
    if (ow >= a.W) continue;
    float v[16];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int q = 0; q < 4; ++q) v[j * 4 + q] = acc[j][i][q];
    if (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_POOLFWD) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        v[c] += bias[c];
        if (EPI != EPI_BIAS) v[c] = fmaxf(v[c], 0.f);
      }
    }
    const size_t off = ((size_t)(n * a.H + oh) * a.W + ow) * CO + chb;
    if (EPI == EPI_MASK) {
      const uint4 m0 = *reinterpret_cast<const uint4*>(a.mask + off);
      const uint4 m1 = *reinterpret_cast<const uint4*>(a.mask + off + 8);
      const unsigned mw[8] = {m0.x, m0.y, m0.z, m0.w, m1.x, m1.y, m1.z, m1.w};
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const unsigned short bits = (unsigned short)(mw[c >> 1] >> ((c & 1) * 16));
        const bool pos = pos_bits(bits);
        v[c] = pos ? v[c] : 0.f;
        bs[c] += v[c];
      }
    }
    const uint4 o0 =
        make_uint4(pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]), pack2<DT>(v[6], v[7]));
    const uint4 o1 =
        make_uint4(pack2<DT>(v[8], v[9]), pack2<DT>(v[10], v[11]), pack2<DT>(v[12], v[13]), pack2<DT>(v[14], v[15]));
    if (EPI != EPI_POOLFWD || a.y != nullptr) {
      *reinterpret_cast<uint4*>(a.y + off) = o0;
      *reinterpret_cast<uint4*>(a.y + off + 8) = o1;
    }
    if constexpr (EPI == EPI_POOLFWD) {
      // staging tile [4 rows][64 cols] x 128 B, 16-B chunk c of column col at slot c ^ (col & 7)
      const int col = i * 16 + fr;
      uint4* st = reinterpret_cast<uint4*>(halo + (r * 64 + col) * 128);
      st[(2 * fq) ^ (col & 7)] = o0;
      st[(2 * fq + 1) ^ (col & 7)] = o1;
    }
  }
  if constexpr (EPI == EPI_POOLFWD) {
    __syncthreads();
    // 2 pooled rows x 32 pooled columns x 8 chunks of 8 channels: 512 outputs, 2 per thread; max of the
    // stored (rounded) values, exactly what maxpool_fwd_kernel computes from the stored map
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int o = tid + 256 * u;
      const int c = o & 7, pc = (o >> 3) & 31, pr = o >> 8;
      float m[8], t[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {     // q = window position in ATen order (row * 2 + column)
        const int rr = 2 * pr + (q >> 1), cc = 2 * pc + (q & 1);
        const uint4 v4 = reinterpret_cast<const uint4*>(halo + (rr * 64 + cc) * 128)[c ^ (cc & 7)];
        unpack8h<DT>(v4, t[q]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) m[k] = fmaxf(fmaxf(t[0][k], t[1][k]), fmaxf(t[2][k], t[3][k]));
      const size_t pp = (size_t)(n * (a.H >> 1) + (oh0 >> 1) + pr) * (a.W >> 1) + (ow0 >> 1) + pc;
      *reinterpret_cast<uint4*>(a.yp + pp * 64 + c * 8) = pack8h<DT>(m);
      if (a.codes != nullptr) {
        uint32_t cw = 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t first = (t[0][k] == m[k]) ? 1u : (t[1][k] == m[k]) ? 2u : (t[2][k] == m[k]) ? 4u : 8u;
          cw |= ((m[k] > 0.f) ? first : 0u) << (4 * k);
        }
        a.codes[pp * 8 + c] = cw;
      }
    }
  }
  flush_bias();
}

// ===========================================================================
// Weight-stationary persistent 3x3 / dilation-1 conv, Cin = Cout = 64 (conv1_2
// forward, its data gradient, the fused-pool forward).  conv_halo64_kernel
// re-fetches the 72 KB of weights per 4 x 64 tile (24576 tiles at batch 8:
// 1.8 GB through the L2) and each tap waits on its weight DMA: ~14 us per tile
// for 1.9 us of MFMA work.  Here each wave keeps its 32 output channels x 576 K
// of weights in registers for the whole kernel (144 VGPRs, loaded once), one
// block per CU walks a contiguous run of tiles DOWN a 64-column strip (the next
// tile's halo shares 2 of its 6 rows with this one: L2 hits), and the halo of
// tile k+1 streams into the other of two LDS buffers while tile k computes.
// Waves: 8 = 4 rows x 2 channel halves (64 px x 32 co each, 8 accumulators).
//
// One s_waitcnt vmcnt(0) per tile, at its end, covers the next halo, this
// tile's mask loads and the previous tile's stores, all issued a whole tile
// earlier (a counted wait would be unsafe: loads and stores retire out of
// order with respect to each other).
// ===========================================================================
// W1G staging of the produced dY tile: tile pixel px (row * 64 + column) = 128-B row of 16 8-byte units (4 channels
// each), unit c8 at c8 ^ (((px >> 1) & 1 | ((px >> 3) & 1) << 1) << 2): the conv1_1 weight-gradient phase reads its
// A fragments (16 channels x 32 pixels, pixel-contiguous per lane) with two ds_read_b64_tr_b16 each
typedef short w1g_s16x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) w1g_s16x4 w1g_lds_s16x4;
__device__ __forceinline__ unsigned w1g_off(int px, int c8) {
  return (unsigned)(px * 128 + ((c8 ^ ((((px >> 1) & 1) | (((px >> 3) & 1) << 1)) << 2)) * 8));
}

template <int DT, int EPI, bool W1G = false>
__global__ void __launch_bounds__(512, 1) conv_ws64_kernel(HaloConvArgs a) {
  // halo rows of 66 pixels stored at a 72-pixel stride: a 1-KiB DMA piece (8 pixels) never straddles two
  // rows, so wave w fetches piece column w of all 6 rows (pixel slot 8w + lane / 8, a per-lane constant)
  // and waves 0-5 the 9th column (slots 64, 65 + padding) of row w: per piece one address add and one
  // column bounds compare, the row bounds are scalar (was: a division by 66 and a 64-bit multiply per piece)
  constexpr int TR = 4, TCOL = 64, HC = TCOL + 2, HCP = 72;
  constexpr int NHI = (TR + 2) * (HCP / 8);                                // 54 one-KiB DMA pieces
  constexpr int HALO_BYTES = NHI * 1024;
  static_assert(EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_NONE || EPI == EPI_MASK ||
                EPI == EPI_POOLFWD, "ws64 epilogues");
  static_assert(!W1G || EPI == EPI_MASK, "W1G: conv1_2 data gradient only");
  // W1G: image halo of the tile in LDS after the two halo buffers, one planar copy per (kw, c) shifted by kw so a
  // B fragment (8 consecutive pixels of one tap / channel) is one aligned 16-B read: [3][4][6 rows][72] 16-bit
  constexpr int IMG_RS = 72, IMG_PLANE = (TR + 2) * IMG_RS;
  // then the raw image halo (6 x 66 pixels x 8 B, LDS-DMA'd at the tile start: 13 waves x 64 dwords) and the
  // wave-private fp32 weight-gradient accumulators (8 waves x 3 x 64 lanes x 16 B; registers only in that phase)
  constexpr int IMG_PLANES_BYTES = 12 * IMG_PLANE * 2, IMG_RAW_BYTES = 13 * 256;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 15, fq = lane >> 4;
  const int r = wave >> 1, h = wave & 1;           // output row of the tile, channel half
  const int chb = h * 32 + fq * 8;                 // this lane's 8 consecutive output channels

  // contiguous tile run of this block; tile index t -> (n, tx, ty) with ty fastest (down a column strip)
  const int ntile = a.N * a.tiles_y * a.tiles_x;
  const int per = (ntile + gridDim.x - 1) / gridDim.x;
  const int t0 = blockIdx.x * per;
  const int t1 = min(ntile, t0 + per);
  if (t0 >= t1) return;                            // whole block: no barrier reached

  auto tile_org = [&](int t, int& n, int& oh0, int& ow0) {
    const int ty = t % a.tiles_y;
    const int rest = t / a.tiles_y;
    ow0 = (rest % a.tiles_x) * TCOL;
    n = rest / a.tiles_x;
    oh0 = ty * TR;
  };
  auto issue_halo = [&](int t, unsigned char* buf) {
    int n, oh0, ow0;
    tile_org(t, n, oh0, ow0);
    int ln = lane;
    asm volatile("" : "+v"(ln));                    // per-lane math stays here (the kernel is at its VGPR cap)
    const int c0 = wave * 8 + (ln >> 3), c1 = 64 + (ln >> 3);          // slots of piece column wave / 8
    const int o0 = c0 * 64 + (((ln & 7) ^ (c0 & 7)) * 8), o1 = c1 * 64 + (((ln & 7) ^ (c1 & 7)) * 8);
    const bool v0 = (unsigned)(ow0 - 1 + c0) < (unsigned)a.W;
    const bool v1 = c1 < HC && (unsigned)(ow0 - 1 + c1) < (unsigned)a.W;
#pragma unroll
    for (int hr = 0; hr < TR + 2; ++hr) {
      const int ih = oh0 - 1 + hr;
      const bool row_in = ih >= 0 && ih < a.H;      // wave-uniform
      const bf16_t* rbase = a.x + ((ptrdiff_t)(n * a.H + ih) * a.W + ow0 - 1) * 64;
      const void* src = (row_in && v0) ? (const void*)(rbase + o0) : (const void*)a.zero;
      glds16(src, lds_addr((buf + (hr * 9 + wave) * 1024)));
      if (wave == hr) {                             // the 9th piece column: one row per wave 0 .. 5
        const void* src1 = (row_in && v1) ? (const void*)(rbase + o1) : (const void*)a.zero;
        glds16(src1, lds_addr((buf + (hr * 9 + 8) * 1024)));
      }
    }
  };

  issue_halo(t0, smem);
  // weights: A fragment (k-step ks = 2 * tap + kk, row block j) of this wave's 32 channels; A row
  // R = j * 16 + fr holds channel h * 32 + (R >> 2 & 3) * 8 + (R >> 4) * 4 + (R & 3), so that D row
  // j * 16 + fq * 4 + q (acc[j][.][q]) is channel chb + j * 4 + q
  frag8_t wf[18][2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int R = j * 16 + fr;
    const int co = h * 32 + ((R >> 2) & 3) * 8 + (R >> 4) * 4 + (R & 3);
    const bf16_t* wr = a.w + (size_t)co * 576 + fq * 8;
#pragma unroll
    for (int ks = 0; ks < 18; ++ks)
      wf[ks][j] = __builtin_bit_cast(frag8_t, *reinterpret_cast<const uint4*>(wr + (ks >> 1) * 64 + (ks & 1) * 32));
  }
  float bias[8];
  if constexpr (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_POOLFWD) {
    const float4 b0 = *reinterpret_cast<const float4*>(a.bias + chb);
    const float4 b1 = *reinterpret_cast<const float4*>(a.bias + chb + 4);
    bias[0] = b0.x; bias[1] = b0.y; bias[2] = b0.z; bias[3] = b0.w;
    bias[4] = b1.x; bias[5] = b1.y; bias[6] = b1.z; bias[7] = b1.w;
  }
  // per-lane halo offsets (swizzle keyed by the halo column: (fr + kw) & 7 for every fragment)
  int hoff[3][2];
#pragma unroll
  for (int kw = 0; kw < 3; ++kw)
#pragma unroll
    for (int kk = 0; kk < 2; ++kk)
      hoff[kw][kk] = (r * HCP + fr + kw) * 128 + (((kk * 4 + fq) ^ ((fr + kw) & 7)) * 16);
  if constexpr (W1G) {
    f32x4* z = reinterpret_cast<f32x4*>(smem + 2 * HALO_BYTES + IMG_PLANES_BYTES + IMG_RAW_BYTES) + wave * 192 + lane;
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) z[nb * 64] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
  // W1G: conv1_1 weight-gradient accumulators of this wave (16 output channels cb*16.., the 3 x 16 k columns
  // n = tap*4 + c (n = 36: the bias, through a column of ones), pixel rows 2*ph, 2*ph + 1 of every tile), kept in
  // LDS between tiles (the main loop is at the VGPR cap)
  unsigned short* imgs = reinterpret_cast<unsigned short*>(smem + 2 * HALO_BYTES);
  unsigned char* imgraw = smem + 2 * HALO_BYTES + IMG_PLANES_BYTES;
  f32x4* waccl = reinterpret_cast<f32x4*>(smem + 2 * HALO_BYTES + IMG_PLANES_BYTES + IMG_RAW_BYTES) + wave * 192 + lane;

  for (int t = t0, it = 0; t < t1; ++t, ++it) {
    unsigned char* cur = smem + (it & 1) * HALO_BYTES;
    if (t + 1 < t1) issue_halo(t + 1, smem + ((it + 1) & 1) * HALO_BYTES);
    int n, oh0, ow0;
    tile_org(t, n, oh0, ow0);
    const int oh = oh0 + r;
    const bool row_ok = oh < a.H;
    if constexpr (W1G) {
      // raw image halo of this tile -> imgraw by LDS-DMA (4 B per lane; dword d = pixel * 2 + half), retired by
      // the wait after the main loop
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int wj = j * 8 + wave;                 // wave-uniform
        if (wj < 13) {
          int ln = lane;
          asm volatile("" : "+v"(ln));
          const int d = wj * 64 + ln, px = d >> 1;
          const int hr = px / 66, hc = px - hr * 66;
          const int ih = oh0 - 1 + hr, iw = ow0 - 1 + hc;
          const bool ok = hr < 6 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
          const void* src = ok ? (const void*)(reinterpret_cast<const unsigned char*>(a.img) +
                                               ((size_t)(n * a.H + ih) * a.W + iw) * 8 + (d & 1) * 4)
                               : (const void*)a.zero;
          glds4(src, lds_addr((imgraw + wj * 256)));
        }
      }
    }
    uint4 mk[4];
    if constexpr (EPI == EPI_MASK) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ow = ow0 + i * 16 + fr;
        mk[i] = make_uint4(0u, 0u, 0u, 0u);
        if (row_ok && ow < a.W)
          mk[i] = *reinterpret_cast<const uint4*>(a.mask + ((size_t)(n * a.H + oh) * a.W + ow) * 64 + chb);
      }
    }
    f32x4 acc[2][4];
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      const int tap = ks >> 1, kk = ks & 1, kh = tap / 3, kw = tap % 3;
      frag8_t bfr[4];
#pragma unroll
      for (int i = 0; i < 4; ++i)
        bfr[i] = __builtin_bit_cast(frag8_t, *reinterpret_cast<const uint4*>(cur + hoff[kw][kk] + kh * HCP * 128 +
                                                                              i * 2048));
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[j][i] = mfma16<DT>(wf[ks][j], bfr[i], acc[j][i]);
    }
    // the next halo, this tile's mask loads and the previous tile's stores have all retired; every wave's
    // reads of `cur` are done after the barrier
    asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int col = i * 16 + fr, ow = ow0 + col;
      float v[8];
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[j * 4 + q] = acc[j][i][q];
      if constexpr (EPI == EPI_BIAS_RELU || EPI == EPI_BIAS || EPI == EPI_POOLFWD) {
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          v[c] += bias[c];
          if (EPI != EPI_BIAS) v[c] = fmaxf(v[c], 0.f);
        }
      }
      if constexpr (EPI == EPI_MASK) {
        const unsigned mw[4] = {mk[i].x, mk[i].y, mk[i].z, mk[i].w};
#pragma unroll
        for (int c = 0; c < 8; ++c)
          v[c] = pos_bits((unsigned short)(mw[c >> 1] >> ((c & 1) * 16))) ? v[c] : 0.f;
      }
      const uint4 o = pack8h<DT>(v);
      if (row_ok && ow < a.W && ((EPI != EPI_POOLFWD && !W1G) || a.y != nullptr))
        *reinterpret_cast<uint4*>(a.y + ((size_t)(n * a.H + oh) * a.W + ow) * 64 + chb) = o;
      if constexpr (EPI == EPI_POOLFWD) {
        // staging tile [4 rows][64 cols] x 128 B in `cur`, 16-B chunk c of column col at slot c ^ (col & 7)
        reinterpret_cast<uint4*>(cur + (r * 64 + col) * 128)[(h * 4 + fq) ^ (col & 7)] = o;
      }
      if constexpr (W1G) {
        // staging tile in `cur` (w1g_off layout): channels chb .. chb + 7 = units 8h + 2fq, 8h + 2fq + 1
        const int px = r * 64 + col, c8 = h * 8 + fq * 2;
        *reinterpret_cast<uint2*>(cur + w1g_off(px, c8)) = make_uint2(o.x, o.y);
        *reinterpret_cast<uint2*>(cur + w1g_off(px, c8 + 1)) = make_uint2(o.z, o.w);
      }
    }
    if constexpr (EPI == EPI_POOLFWD) {
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
      // 2 pooled rows x 32 pooled columns x 8 chunks of 8 channels = 512 outputs, one per thread; max of the
      // stored (rounded) values and the first-max codes, exactly as maxpool_fwd_kernel from the stored map
      const int c = tid & 7, pc = (tid >> 3) & 31, pr = tid >> 8;
      float m[8], tv[4][8];
#pragma unroll
      for (int q = 0; q < 4; ++q) {     // q = window position in ATen order (row * 2 + column)
        const int rr = 2 * pr + (q >> 1), cc = 2 * pc + (q & 1);
        unpack8h<DT>(reinterpret_cast<const uint4*>(cur + (rr * 64 + cc) * 128)[c ^ (cc & 7)], tv[q]);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) m[k] = fmaxf(fmaxf(tv[0][k], tv[1][k]), fmaxf(tv[2][k], tv[3][k]));
      const size_t pp = (size_t)(n * (a.H >> 1) + (oh0 >> 1) + pr) * (a.W >> 1) + (ow0 >> 1) + pc;
      *reinterpret_cast<uint4*>(a.yp + pp * 64 + c * 8) = pack8h<DT>(m);
      if (a.codes != nullptr) {
        uint32_t cw = 0u;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const uint32_t first = (tv[0][k] == m[k]) ? 1u : (tv[1][k] == m[k]) ? 2u : (tv[2][k] == m[k]) ? 4u : 8u;
          cw |= ((m[k] > 0.f) ? first : 0u) << (4 * k);
        }
        a.codes[pp * 8 + c] = cw;
      }
      // staging reads done before the next-but-one halo DMA overwrites `cur`
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
    if constexpr (W1G) {
      // image halo -> 12 shifted planes: imgs[(kw*4 + c)*IMG_PLANE + hr*IMG_RS + j] = img[hr][j + kw][c]
      // (imgraw retired by the wait + barrier after the main loop; the planes' previous readers passed the
      // barrier that ended the previous tile)
      if (tid < 6 * 66) {
        int tl = tid;
        asm volatile("" : "+v"(tl));
        const int hr = tl / 66, hc = tl - hr * 66;
        const uint2 imv = *reinterpret_cast<const uint2*>(imgraw + tl * 8);
        const unsigned short cv[4] = {(unsigned short)(imv.x & 0xffffu), (unsigned short)(imv.x >> 16),
                                      (unsigned short)(imv.y & 0xffffu), (unsigned short)(imv.y >> 16)};
#pragma unroll
        for (int kw = 0; kw < 3; ++kw)
          if (hc - kw >= 0 && hc - kw < IMG_RS)
#pragma unroll
            for (int c = 0; c < 4; ++c) imgs[(kw * 4 + c) * IMG_PLANE + hr * IMG_RS + hc - kw] = cv[c];
      }
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // dY staging tile + image planes
      // dW1[co][n] += sum_p dY[p][co] * img(p + tap)[c], K = this wave's 128 pixels in 4 steps of 32
      const int cb = wave & 3, ph = wave >> 2;
      int ln = lane;
      asm volatile("" : "+v"(ln));                   // lane math stays in this phase (not hoisted out of the loop)
      const int fr = ln & 15, fq = ln >> 4;
      const int qd = (ln & 15) >> 2, p4 = ln & 3;
      f32x4 wacc[3];
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) wacc[nb] = waccl[nb * 64];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const int row = 2 * ph + (s4 >> 1), colb = (s4 & 1) * 32 + fq * 8;
        // A = dY^T (channels cb*16 + fr, pixels colb .. colb + 7 of this lane's k group): lo = pixels + 0..3,
        // hi = + 4..7 (transposed 8-byte reads of units 4cb + p4 of pixel rows 8fq + qd, 8fq + qd + 4)
        const int px0 = row * 64 + (s4 & 1) * 32 + 8 * fq + qd;
        const w1g_s16x4 alo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((w1g_lds_s16x4*)(cur + w1g_off(px0, 4 * cb + p4)));
        const w1g_s16x4 ahi =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((w1g_lds_s16x4*)(cur + w1g_off(px0 + 4, 4 * cb + p4)));
        typedef short s16x8_t __attribute__((ext_vector_type(8)));
        const s16x8_t a8 = {alo[0], alo[1], alo[2], alo[3], ahi[0], ahi[1], ahi[2], ahi[3]};
        const frag8_t afr = __builtin_bit_cast(frag8_t, a8);
#pragma unroll
        for (int nb = 0; nb < 3; ++nb) {
          const int nn = nb * 16 + fr;
          const int tap = (nn < 36) ? (nn >> 2) : 0, c = nn & 3;
          const int kh = tap / 3, kw = tap - kh * 3;
          uint4 bv = *reinterpret_cast<const uint4*>(imgs + (kw * 4 + c) * IMG_PLANE + (row + kh) * IMG_RS + colb);
          if (nn >= 36) {
            const unsigned one2 = (nn == 36) ? ((unsigned)one_bits<DT>() * 0x10001u) : 0u;
            bv = make_uint4(one2, one2, one2, one2);
          }
          wacc[nb] = mfma16<DT>(afr, __builtin_bit_cast(frag8_t, bv), wacc[nb]);
        }
      }
#pragma unroll
      for (int nb = 0; nb < 3; ++nb) waccl[nb * 64] = wacc[nb];
      // staging / image reads done before the next tile's epilogue and the next-but-one halo DMA overwrite them
      asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    }
  }
  if constexpr (W1G) {
    // D row fq*4 + q = channel cb*16 + fq*4 + q, column fr = k column nb*16 + fr; part = 2 * block + ph
    const int cb = wave & 3, ph = wave >> 2;
    const size_t part = (size_t)blockIdx.x * 2 + ph;
#pragma unroll
    for (int nb = 0; nb < 3; ++nb) {
      const int nn = nb * 16 + fr;
      const f32x4 w4 = waccl[nb * 64];
      const float4 v4 = make_float4(w4[0], w4[1], w4[2], w4[3]);
      if (nn < 36)
        *reinterpret_cast<float4*>(a.w1slab + (part * 36 + nn) * 64 + cb * 16 + fq * 4) = v4;
      else if (nn == 36)
        *reinterpret_cast<float4*>(a.w1bslab + part * 64 + cb * 16 + fq * 4) = v4;
    }
  }
}

// grid of launch_ws64 for ntile tiles (W1G: 2 weight-gradient slabs per block)
static int ws64_grid(int ntile, int ncu) {
  const int per = (ntile + ncu - 1) / ncu;
  return (ntile + per - 1) / per;
}

template <int DT, int EPI, bool W1G = false>
static int launch_ws64(const HaloConvArgs& a, hipStream_t s) {
  // 2 halo buffers of 6 rows x 72 pixel slots (+ W1G: 12 shifted image planes of 6 x 72 16-bit words)
  constexpr size_t lds = 2 * (size_t)(6 * 9) * 1024 + (W1G ? 12 * 6 * 72 * 2 + 13 * 256 + 8 * 192 * 16 : 0);
  auto kfn = conv_ws64_kernel<DT, EPI, W1G>;
  static int ncu = 0;
  if (!ncu) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    int dev = 0;
    CAN_HIP_CHECK(hipGetDevice(&dev));
    CAN_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  }
  const int grid = ws64_grid(a.N * a.tiles_y * a.tiles_x, ncu);   // every block gets a non-empty run
  hipLaunchKernelGGL(kfn, dim3(grid), dim3(512), lds, s, a);
  return (int)hipGetLastError();
}

// ws64 (weight-stationary) instead of the halo kernel for Cin = Cout = 64 (dispatch ws64 = 0: halo kernel)
static bool use_ws64() { return g_dispatch.ws64 != 0; }

// ===========================================================================
// First layer (conv1_1: 3 -> 64, 3x3, input NHWC4 bf16 = 8 B per pixel).
// Output-write bound (805 MB of bf16 activations at batch 8 x 768 x 1024), so
// the kernel does the minimum around the stores: the 6 x 130-pixel input halo
// of a 4 x 128 output tile goes to LDS (6.2 KB, plain 8-B loads); the
// weights (packed [64][64], k = tap*4 + c) are MFMA A fragments loaded straight
// into registers; each B fragment is two ds_read_b64 (taps 2q, 2q+1 of one
// pixel, 4 channels each); K = 64 = 2 MFMA k-steps (taps 9..15 are zero).
// Persistent (PF): two blocks per CU walk the tiles; a block loads the NEXT
// tile's halo into registers before it computes and stores the current one and
// parks it in the other LDS buffer afterwards, so its store stream never waits
// on a halo load (one tile per block: 0.268 ms = 3.0 TB/s of stores).
// Lane q of the D layout owns channels 8q .. 8q + 7 and 32 + 8q .. 32 + 8q + 7
// (A row j*16 + 4q + r holds channel 32 (j >> 1) + 8q + 4 (j & 1) + r): each of a
// wave's two 16-B stores covers 64 contiguous bytes of 16 pixels (16-B pieces
// 32 B apart with perm_row: 0.268 -> 0.261 ms).
// ===========================================================================
__device__ __forceinline__ int perm_row_st64(int rho) {
  const int jt = rho >> 4, q = (rho >> 2) & 3, r = rho & 3;
  return ((jt >> 1) << 5) | (q << 3) | ((jt & 1) << 2) | r;
}
// LS (the persistent form's): each 16-pixel fragment goes through a wave-private 2 KiB LDS tile (16-B chunks XOR-
// swizzled by pixel) and leaves as two 1-KiB fully contiguous stores instead of two 64-B-per-pixel ones
// (0.188 -> 0.168 ms, 4.3 -> 4.8 TB/s, profiles/r4/ab_first_layer.txt)
template <int DT, bool PF, bool LS = false>
__global__ void __launch_bounds__(512, 4) conv_first_halo_kernel(HaloConvArgs a) {   // 2 blocks per CU: <= 128 VGPRs
  constexpr int TR = 4, TCOL = 128, HC = TCOL + 2, HPIX = (TR + 2) * HC;
  static_assert(HPIX <= 1024, "two halo pixels per thread");
  __shared__ uint2 halo[PF ? 2 : 1][HPIX];
  __shared__ uint4 stg[LS ? 8 : 1][LS ? 128 : 1];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntile = a.N * a.tiles_y * a.tiles_x;
  const uint2* x8 = reinterpret_cast<const uint2*>(a.x);
  // halo pixels tid and tid + 512 of tile t (zero outside the map / past HPIX)
  auto load = [&](int t, uint2 (&v)[2]) {
    const int tx = t % a.tiles_x, ty = (t / a.tiles_x) % a.tiles_y, n = t / (a.tiles_x * a.tiles_y);
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int hp = tid + 512 * k;
      const int hr = hp / HC, hc = hp - hr * HC;
      const int ih = ty * TR - 1 + hr, iw = tx * TCOL - 1 + hc;
      v[k] = make_uint2(0u, 0u);
      if (hp < HPIX && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W) v[k] = x8[(size_t)(n * a.H + ih) * a.W + iw];
    }
  };
  auto park = [&](int b, const uint2 (&v)[2]) {
    halo[b][tid] = v[0];
    if (tid + 512 < HPIX) halo[b][tid + 512] = v[1];
  };
  const int fr = lane & 15, fq = lane >> 4;
  frag8_t af[2][4];
#pragma unroll
  for (int kk = 0; kk < 2; ++kk)
#pragma unroll
    for (int j = 0; j < 4; ++j)
      af[kk][j] = __builtin_bit_cast(frag8_t, *reinterpret_cast<const uint4*>(a.w + perm_row_st64(j * 16 + fr) * 64 + kk * 32 + fq * 8));
  const int chb = fq * 8;                              // channel of v[0]; v[8] at chb + 32
  float bias[16];
#pragma unroll
  for (int c = 0; c < 16; c += 4) {
    const float4 b4 = *reinterpret_cast<const float4*>(a.bias + chb + (c < 8 ? c : 24 + c));
    bias[c] = b4.x; bias[c + 1] = b4.y; bias[c + 2] = b4.z; bias[c + 3] = b4.w;
  }
  const int r = wave >> 1, colbase = (wave & 1) * 64;

  int t = PF ? (int)blockIdx.x : xcd_remap(blockIdx.x, ntile);
  const int tstep = PF ? (int)gridDim.x : ntile;
  uint2 nv[2];
  load(t, nv);
  park(0, nv);
  __syncthreads();
  for (int it = 0; t < ntile; ++it, t += tstep) {
    const int b = PF ? (it & 1) : 0;
    const bool more = PF && t + tstep < ntile;
    if (more) load(t + tstep, nv);                   // in flight under this tile's MFMAs and stores
    const int tx = t % a.tiles_x, ty = (t / a.tiles_x) % a.tiles_y, n = t / (a.tiles_x * a.tiles_y);
    const int oh = ty * TR + r;
    // one 16-pixel fragment at a time (16 accumulator registers live, not 64: two blocks per CU fit)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f32x4 acc[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      const int c = colbase + i * 16 + fr;
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int t0 = kk * 8 + fq * 2;               // this lane's taps t0, t0+1
        uint2 lo = make_uint2(0u, 0u), hi = make_uint2(0u, 0u);
        if (t0 < 9) {
          const int kh = (t0 * 11) >> 5, kw = t0 - kh * 3;
          lo = halo[b][(r + kh) * HC + c + kw];
        }
        if (t0 + 1 < 9) {
          const int kh = ((t0 + 1) * 11) >> 5, kw = t0 + 1 - kh * 3;
          hi = halo[b][(r + kh) * HC + c + kw];
        }
        const frag8_t bfr = __builtin_bit_cast(frag8_t, make_uint4(lo.x, lo.y, hi.x, hi.y));
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] = mfma16<DT>(af[kk][j], bfr, acc[j]);
      }
      const int ow = tx * TCOL + c;
      if constexpr (LS) {
        float v[16];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int q = 0; q < 4; ++q) v[j * 4 + q] = fmaxf(acc[j][q] + bias[j * 4 + q], 0.f);
        // pixel fr's 16-B chunks fq (channels 8fq..) and 4 + fq (32 + 8fq..) at slot chunk ^ (fr & 7)
        uint4* st = stg[wave];
        st[fr * 8 + (fq ^ (fr & 7))] =
            make_uint4(pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]), pack2<DT>(v[6], v[7]));
        st[fr * 8 + ((4 + fq) ^ (fr & 7))] =
            make_uint4(pack2<DT>(v[8], v[9]), pack2<DT>(v[10], v[11]), pack2<DT>(v[12], v[13]), pack2<DT>(v[14], v[15]));
        // read back pixel-major (wave-private tile: the wave's LDS ops retire in order)
#pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int px = hh * 8 + (lane >> 3), ch = lane & 7;
          const uint4 val = st[px * 8 + (ch ^ (px & 7))];
          const int owp = tx * TCOL + colbase + i * 16 + px;
          if (oh < a.H && owp < a.W)
            *reinterpret_cast<uint4*>(a.y + ((size_t)(n * a.H + oh) * a.W + owp) * 64 + ch * 8) = val;
        }
        continue;
      }
      if (oh >= a.H || ow >= a.W) continue;
      float v[16];
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int q = 0; q < 4; ++q) v[j * 4 + q] = fmaxf(acc[j][q] + bias[j * 4 + q], 0.f);
      const size_t off = ((size_t)(n * a.H + oh) * a.W + ow) * 64 + chb;
      *reinterpret_cast<uint4*>(a.y + off) =
          make_uint4(pack2<DT>(v[0], v[1]), pack2<DT>(v[2], v[3]), pack2<DT>(v[4], v[5]), pack2<DT>(v[6], v[7]));
      *reinterpret_cast<uint4*>(a.y + off + 32) =
          make_uint4(pack2<DT>(v[8], v[9]), pack2<DT>(v[10], v[11]), pack2<DT>(v[12], v[13]), pack2<DT>(v[14], v[15]));
    }
    if (!PF) break;
    if (more) park(b ^ 1, nv);                       // buffer b ^ 1 was last read two tiles ago (barrier since)
    __syncthreads();
  }
}

template <int DT, int CO, int EPI, int TCOL>
static int launch_halo64(const HaloConvArgs& a, hipStream_t s) {
  constexpr int HALO_BYTES = ((6 * (TCOL + 2) + 7) / 8) * 1024;
  constexpr int NW = (CO == 64 && TCOL == 64) ? 4 : 8;
  const size_t lds = HALO_BYTES + 3 * (size_t)CO * 128;
  auto kfn = conv_halo64_kernel<DT, CO, EPI, TCOL>;
  static bool attr = false;
  if (!attr) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  hipLaunchKernelGGL(kfn, dim3(a.N * a.tiles_y * a.tiles_x), dim3(64 * NW), lds, s, a);
  return (int)hipGetLastError();
}

template <int DT, int WC, int WP, int PW, int EPI>
static int launch_glds(const ConvArgs2& a, hipStream_t s) {
  constexpr int TC = 64 * WC, TP = 64 * PW * WP;
  const size_t lds = 2 * (size_t)(TC + TP) * 128;
  auto kfn = conv_glds_kernel<DT, WC, WP, PW, EPI>;
  static bool attr = false;
  if (!attr) {
    CAN_HIP_CHECK(hipFuncSetAttribute((const void*)kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    attr = true;
  }
  const int nct = a.Cout / TC, npt = (a.M + TP - 1) / TP;
  hipLaunchKernelGGL(kfn, dim3(nct * npt), dim3(64 * WC * WP), lds, s, a);
  return (int)hipGetLastError();
}

// default LDS-DMA tile config: v2 (pipelined); 128 x 512 tiles measured faster for K <= 1152
static int glds_default_cfg(int Cin, int Cout, int ksize) {
  const int ktot = ksize * ksize * Cin;
  return (Cout % 256 == 0) ? 21 : (Cout % 128 == 0) ? (ktot <= 1152 ? 25 : 22) : 23;
}
static int glds_cfg_tp(int cfg) {   // pixels per tile of a v2 config
  return (cfg == 21 || cfg == 22) ? 256 : (cfg == 23 || cfg == 25) ? 512 : 0;
}
// rows of the bias-partial matrix an LDS-DMA config writes: pixel tiles x waves along the pixels (0: none); the
// row ring's pixel tiles are per-image row groups x column blocks (rr_np)
static int glds_bpart_rows(int cfg, int M, int H, int W) {
  int tp = 0, wp = 0;
  switch (cfg) {
    case 27: return rr_np(H, W, M, 2) * 2;     // 256 ch x (2 x 128) px, 4 x 2 waves
    case 29: return rr_np(H, W, M, 2) * 4;     // 128 x (2 x 128), 2 x 4
    case 28: return rr_np(H, W, M, 4) * 8;     // 64 x (4 x 128), 1 x 8
    case 11: case 21: tp = 256; wp = 2; break;   // 256 ch x 256 px, 4 x 2 waves
    case 12: case 22: tp = 256; wp = 4; break;   // 128 x 256, 2 x 4
    case 13: case 23: tp = 512; wp = 8; break;   // 64 x 512, 1 x 8
    case 25: tp = 512; wp = 4; break;            // 128 x 512, 2 x 4 (2 fragments per wave)
    default: return 0;
  }
  return ((M + tp - 1) / tp) * wp;
}

template <int DT, int EPI>
static int dispatch_glds(const ConvArgs2& a, int tile_cfg, hipStream_t s, int nb = 1) {
  int cfg = tile_cfg;
  if (cfg == 0) cfg = glds_default_cfg(a.Cin, a.Cout, a.ksize);
  if constexpr (EPI == EPI_POOLFWD) {
    const int tp = glds_cfg_tp(cfg);
    if (tp == 0 || (a.H & 1) || a.W % (tp / 2) || a.yp == nullptr) return -12;
  }
  if constexpr (EPI == EPI_POOLBWD) {
    if (a.pcodes == nullptr) return -14;
  }
  switch (cfg) {
    case 11: if (a.Cout % 256 || EPI == EPI_POOLFWD || nb > 1) return -8; return launch_glds<DT, 4, 2, 2, EPI>(a, s);
    case 12: if (a.Cout % 128 || EPI == EPI_POOLFWD || nb > 1) return -8; return launch_glds<DT, 2, 4, 1, EPI>(a, s);
    case 13: if (EPI == EPI_POOLFWD || nb > 1) return -8; return launch_glds<DT, 1, 8, 1, EPI>(a, s);
    case 21: if (a.Cout % 256) return -8; return launch_glds2<DT, 4, 2, 2, EPI>(a, s, nb);
    case 22: if (a.Cout % 128) return -8; return launch_glds2<DT, 2, 4, 1, EPI>(a, s, nb);
    case 23: return launch_glds2<DT, 1, 8, 1, EPI>(a, s, nb);
    case 25: if (a.Cout % 128) return -8; return launch_glds2<DT, 2, 4, 2, EPI>(a, s, nb);   // 128 x 512, 160 KB LDS
    case 27: case 28: case 29: if (nb > 1) return -8; return launch_rring<DT, EPI>(a, s, cfg);    // row ring
  }
  return -9;
}

static const bf16_t* conv_zero_page() {
  static void* z = nullptr;
  if (!z) {
    if (hipMalloc(&z, 4096) != hipSuccess) return nullptr;
    if (hipMemset(z, 0, 4096) != hipSuccess) return nullptr;
  }
  return (const bf16_t*)z;
}

template <int DT>
static int conv_igemm_impl(const void* x, const void* w, const float* bias, const void* mask, void* y,
                           int N, int H, int W, int Cin, int Cout, int ksize, int dil,
                           int epi, int first, int tile_cfg, void* stream, float* bpart, int bpart_cap,
                           int* bpart_rows) {
  if (bpart_rows) *bpart_rows = 0;
  if (epi != EPI_MASK && epi != EPI_POOLBWD) bpart = nullptr;
  ConvArgs a;
  a.x = (const bf16_t*)x; a.w = (const bf16_t*)w; a.bias = bias; a.mask = (const bf16_t*)mask;
  a.y = (bf16_t*)y; a.N = N; a.H = H; a.W = W; a.Cin = Cin; a.Cout = Cout; a.ksize = ksize; a.dil = dil;
  a.M = N * H * W;
  if (Cout % 64 != 0) return -2;
  if (!first && Cin % 64 != 0) return -3;
  if (first && (Cin != 4 || ksize != 3)) return -4;
  hipStream_t s = (hipStream_t)stream;
#define CAN_EPI_CASE(L, E) \
  if (epi == E) return dispatch_tiles<DT, L, E>(a, tile_cfg, s);
  const bool auto_halo = tile_cfg == 0;
  if (first) {
    if ((tile_cfg == 32 || auto_halo) && Cout == 64 && epi == EPI_BIAS_RELU) {
      HaloConvArgs h;
      h.x = a.x; h.w = a.w; h.bias = a.bias; h.mask = nullptr; h.y = a.y; h.zero = nullptr;
      h.N = N; h.H = H; h.W = W; h.tiles_x = (W + 127) / 128; h.tiles_y = (H + 3) / 4;
      const int ntile = N * h.tiles_y * h.tiles_x;
      if (g_dispatch.first_pf) {
        static int ncu = 0;
        if (!ncu) {
          int dev = 0;
          CAN_HIP_CHECK(hipGetDevice(&dev));
          CAN_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
        }
        hipLaunchKernelGGL((conv_first_halo_kernel<DT, true, true>), dim3(std::min(ntile, 2 * ncu)), dim3(512), 0, s, h);
      } else {
        hipLaunchKernelGGL((conv_first_halo_kernel<DT, false>), dim3(ntile), dim3(512), 0, s, h);
      }
      return (int)hipGetLastError();
    }
    CAN_EPI_CASE(LOAD_FIRST, EPI_BIAS_RELU)
    return -5;
  }
  if (auto_halo && Cin == 64 && ksize == 3 && dil == 1 && (Cout == 64 || Cout == 128) && epi != EPI_SIGMOID &&
      epi != EPI_POOLBWD && epi != EPI_F32)
    tile_cfg = 31;
  if (tile_cfg == 31) {
    // halo-tiled Cin = 64 kernel (explicit; see conv_halo64_kernel)
    if (Cin != 64 || ksize != 3 || dil != 1 || (Cout != 64 && Cout != 128)) return -11;
    HaloConvArgs h;
    h.x = a.x; h.w = a.w; h.bias = a.bias; h.mask = a.mask; h.y = a.y; h.zero = conv_zero_page();
    if (!h.zero) return -10;
    // Cout = 64: 64-column tiles, two blocks per CU
    const bool narrow = Cout == 64;
    h.N = N; h.H = H; h.W = W; h.tiles_x = narrow ? (W + 63) / 64 : (W + 127) / 128; h.tiles_y = (H + 3) / 4;
    if (bpart != nullptr && epi == EPI_MASK) {
      const int rows_per_tile = (Cout == 128) ? 4 : narrow ? 4 : 8;   // NW * 64 / CO
      const long long rows = (long long)N * h.tiles_y * h.tiles_x * rows_per_tile;
      if (rows <= bpart_cap) { h.bpart = bpart; if (bpart_rows) *bpart_rows = (int)rows; }
    }
    if (narrow && h.bpart == nullptr && use_ws64()) {
      switch (epi) {
        case EPI_BIAS_RELU: return launch_ws64<DT, EPI_BIAS_RELU>(h, s);
        case EPI_MASK: return launch_ws64<DT, EPI_MASK>(h, s);
        case EPI_NONE: return launch_ws64<DT, EPI_NONE>(h, s);
        case EPI_BIAS: return launch_ws64<DT, EPI_BIAS>(h, s);
      }
    }
#define CAN_HALO_CASE(E) \
    if (epi == E) return (Cout == 128) ? launch_halo64<DT, 128, E, 128>(h, s) \
                         : narrow ? launch_halo64<DT, 64, E, 64>(h, s) : launch_halo64<DT, 64, E, 128>(h, s);
    CAN_HALO_CASE(EPI_BIAS_RELU)
    CAN_HALO_CASE(EPI_MASK)
    CAN_HALO_CASE(EPI_NONE)
    CAN_HALO_CASE(EPI_BIAS)
#undef CAN_HALO_CASE
    return -6;
  }
  if (tile_cfg == 0 || tile_cfg >= 10) {
    if (H < 2 || W < 2) return -7;
    ConvArgs2 b;
    b.x = a.x; b.w = a.w; b.bias = a.bias; b.mask = a.mask; b.y = a.y; b.zero = conv_zero_page();
    if (!b.zero) return -10;
    if (epi == EPI_POOLBWD) { b.mask = nullptr; b.pcodes = (const uint32_t*)mask; }   // mask = max-pool codes
    b.H = H; b.W = W; b.Cin = Cin; b.Cout = Cout; b.ksize = ksize; b.dil = dil; b.M = a.M;
    if (tile_cfg == 0 && rring_mode() >= dil) tile_cfg = rring_cfg(H, W, Cin, Cout, ksize, dil, epi);
    if (bpart != nullptr) {
      const int rows = glds_bpart_rows(tile_cfg ? tile_cfg : glds_default_cfg(Cin, Cout, ksize), a.M, H, W);
      if (rows > 0 && rows <= bpart_cap) { b.bpart = bpart; if (bpart_rows) *bpart_rows = rows; }
    }
    b.fdW = make_fastdiv((uint32_t)W); b.fdH = make_fastdiv((uint32_t)H);
    switch (epi) {
      case EPI_BIAS_RELU: return dispatch_glds<DT, EPI_BIAS_RELU>(b, tile_cfg, s);
      case EPI_MASK: return dispatch_glds<DT, EPI_MASK>(b, tile_cfg, s);
      case EPI_NONE: return dispatch_glds<DT, EPI_NONE>(b, tile_cfg, s);
      case EPI_BIAS: return dispatch_glds<DT, EPI_BIAS>(b, tile_cfg, s);
      case EPI_SIGMOID: return dispatch_glds<DT, EPI_SIGMOID>(b, tile_cfg, s);
      case EPI_POOLBWD: return dispatch_glds<DT, EPI_POOLBWD>(b, tile_cfg, s);
      case EPI_F32: return dispatch_glds<DT, EPI_F32>(b, tile_cfg, s);
    }
    return -6;
  }
  CAN_EPI_CASE(LOAD_GENERIC, EPI_BIAS_RELU)
  CAN_EPI_CASE(LOAD_GENERIC, EPI_MASK)
  CAN_EPI_CASE(LOAD_GENERIC, EPI_NONE)
  CAN_EPI_CASE(LOAD_GENERIC, EPI_BIAS)
  CAN_EPI_CASE(LOAD_GENERIC, EPI_SIGMOID)
#undef CAN_EPI_CASE
  return -6;
}

// nb independent convs of one shape in ONE launch of the v2 kernel (grid.y = item): the context module's four
// 512 -> 512 1x1 convs (sigmoid forward, plain data gradient).  Items are nb x the single-conv layout at
// element strides xbs / wbs / ybs.
template <int DT>
static int conv_igemm_batched_impl(const void* x, const void* w, const float* bias, void* y, int nb, long long xbs,
                                   long long wbs, long long ybs, int N, int H, int W, int Cin, int Cout, int ksize,
                                   int dil, int epi, int tile_cfg, hipStream_t s) {
  if (nb < 1 || nb > 65535 || Cin % 64 || Cout % 64 || H < 2 || W < 2) return -2;
  if (tile_cfg != 0 && tile_cfg < 20) return -8;
  ConvArgs2 b;
  b.x = (const bf16_t*)x; b.w = (const bf16_t*)w; b.bias = bias; b.mask = nullptr; b.y = (bf16_t*)y;
  b.zero = conv_zero_page();
  if (!b.zero) return -10;
  b.H = H; b.W = W; b.Cin = Cin; b.Cout = Cout; b.ksize = ksize; b.dil = dil; b.M = N * H * W;
  b.fdW = make_fastdiv((uint32_t)W); b.fdH = make_fastdiv((uint32_t)H);
  b.xbs = xbs; b.wbs = wbs; b.ybs = ybs;
  const int cfg = tile_cfg ? tile_cfg : glds_default_cfg(Cin, Cout, ksize);   // always a v2 config
  switch (epi) {
    case EPI_NONE: return dispatch_glds<DT, EPI_NONE>(b, cfg, s, nb);
    case EPI_SIGMOID: return dispatch_glds<DT, EPI_SIGMOID>(b, cfg, s, nb);
    case EPI_BIAS_RELU: return dispatch_glds<DT, EPI_BIAS_RELU>(b, cfg, s, nb);
  }
  return -6;
}

// Linearised context module GEMMs (see "Linearised context module").  fwd = 1: x = fv [M][C], w = W2cat
// [4C][C] -> y = w maps [M][4C], cat [M][2C] (fv | fi); tab0 = t, tab1 = u.  fwd = 0: x = dG [M][4C],
// w = W2cat^T [C][4C], mask = fv, cat = dcat (read) -> y = dfv [M][C]; tab0 = dave.
template <int DT>
static int conv_ctx_impl(int fwd, const void* x, const void* w, const float* tab0, const float* tab1,
                         const void* fv, void* cat, void* y, int N, int H, int W, int C, hipStream_t s) {
  if (C % 256 || W < 64 || H < 1) return -2;       // 256 x 256 tiles; <= 5 image rows per 256-pixel tile
  ConvArgs2 b;
  b.x = (const bf16_t*)x; b.w = (const bf16_t*)w; b.bias = nullptr; b.y = (bf16_t*)y;
  b.zero = conv_zero_page();
  if (!b.zero) return -10;
  b.H = H; b.W = W; b.ksize = 1; b.dil = 1; b.M = N * H * W;
  b.Cin = fwd ? C : 4 * C;
  b.Cout = fwd ? 4 * C : C;
  b.fdW = make_fastdiv((uint32_t)W); b.fdH = make_fastdiv((uint32_t)H);
  b.ctab0 = tab0; b.ctab1 = tab1; b.cat = (bf16_t*)cat; b.cC = C;
  // tiles: 256 x 256 (8 waves, one block per CU) or 128 x 128 (4 waves, 64 KB ring: two blocks per CU, one block's
  // epilogue beside the other's main loop); dispatch ctx_tile_f / ctx_tile_b select
  const int tile = fwd ? g_dispatch.ctx_tile_f : g_dispatch.ctx_tile_b;
  if (fwd) {
    b.mask = nullptr; b.fvp = (const bf16_t*)fv;
    return tile == 128 ? launch_glds2<DT, 2, 2, 1, EPI_CTXF>(b, s) : launch_glds2<DT, 4, 2, 2, EPI_CTXF>(b, s);
  }
  b.mask = (const bf16_t*)fv;
  return tile == 128 ? launch_glds2<DT, 2, 2, 1, EPI_CTXB>(b, s) : launch_glds2<DT, 4, 2, 2, EPI_CTXB>(b, s);
}

// 3x3 / 1x1 conv + bias + ReLU with the 2x2/s2 max-pool fused into the epilogue: yp = pooled output,
// codes = its max-pool codes (what the backward needs), y = the full-resolution output (optional: nullptr
// skips its 2-byte-per-element store).  LDS-DMA v2 kernels and conv1_2's halo kernel.
template <int DT>
static int conv_pool_fwd_impl(const void* x, const void* w, const float* bias, void* y, void* yp, void* codes,
                              int N, int H, int W, int Cin, int Cout, int ksize, int dil, int tile_cfg,
                              hipStream_t s) {
  if (Cout % 64 || Cin % 64 || H < 2 || W < 2) return -3;
  if (ksize == 3 && dil == 1 && H % 2 == 0 && W % 128 == 0 && Cin % 64 == 0 &&
      ((tile_cfg == 0 && g_dispatch.rring_pool && Cout % 256 == 0) || (tile_cfg == 27 && Cout % 256 == 0) ||
       (tile_cfg == 29 && Cout % 128 == 0))) {
    // row ring with the max-pool in the epilogue: 256 x (2 x 128) tiles (Cout % 256 == 0) or 128 x (2 x 128).
    // Default (dispatch rring_pool) only the 256-channel form: conv3_3 + pool 0.429 -> 0.384 ms; the 128-channel
    // one loses to conv_glds2's 128 x 512 tile on conv2_2 (0.588 -> 0.639 ms), profiles/r4/ab_rring_pool.txt
    ConvArgs2 b;
    b.x = (const bf16_t*)x; b.w = (const bf16_t*)w; b.bias = bias; b.mask = nullptr; b.y = (bf16_t*)y;
    b.yp = (bf16_t*)yp; b.codes = (uint32_t*)codes; b.zero = conv_zero_page();
    if (!b.zero) return -10;
    b.H = H; b.W = W; b.Cin = Cin; b.Cout = Cout; b.ksize = ksize; b.dil = dil; b.M = N * H * W;
    b.fdW = make_fastdiv((uint32_t)W); b.fdH = make_fastdiv((uint32_t)H);
    const bool wide = (tile_cfg == 27) || (tile_cfg == 0 && Cout % 256 == 0);
    return wide ? launch_rring_rg<DT, EPI_POOLFWD, 256, 2, 3, 1, false>(b, s)
                : launch_rring_rg<DT, EPI_POOLFWD, 128, 2, 3, 1, false>(b, s);
  }
  if (Cin == 64 && Cout == 64 && ksize == 3 && dil == 1 && tile_cfg == 0) {
    // conv1_2: halo-tiled kernel, 4 x 64 output tiles (full tiles only: the pool epilogue has barriers)
    if (H % 4 || W % 64) return -13;
    HaloConvArgs h;
    h.x = (const bf16_t*)x; h.w = (const bf16_t*)w; h.bias = bias; h.mask = nullptr; h.y = (bf16_t*)y;
    h.yp = (bf16_t*)yp; h.codes = (uint32_t*)codes; h.zero = conv_zero_page();
    if (!h.zero) return -10;
    h.N = N; h.H = H; h.W = W; h.tiles_x = W / 64; h.tiles_y = H / 4;
    if (use_ws64()) return launch_ws64<DT, EPI_POOLFWD>(h, s);
    return launch_halo64<DT, 64, EPI_POOLFWD, 64>(h, s);
  }
  ConvArgs2 b;
  b.x = (const bf16_t*)x; b.w = (const bf16_t*)w; b.bias = bias; b.mask = nullptr; b.y = (bf16_t*)y;
  b.yp = (bf16_t*)yp; b.codes = (uint32_t*)codes; b.zero = conv_zero_page();
  if (!b.zero) return -10;
  b.H = H; b.W = W; b.Cin = Cin; b.Cout = Cout; b.ksize = ksize; b.dil = dil; b.M = N * H * W;
  b.fdW = make_fastdiv((uint32_t)W); b.fdH = make_fastdiv((uint32_t)H);
  return dispatch_glds<DT, EPI_POOLFWD>(b, tile_cfg, s);
}

// conv1_2's data gradient (ws64, EPI_MASK: dX = relu-masked, mask = conv1_1's output) with conv1_1's weight
// gradient accumulated from each produced tile (W1G); dX stored only when y is not null.  Writes 2 * grid slabs to
// w1slab [S][36][64] / w1bslab [S][64]; returns S (> 0) or a negative error.
template <int DT>
static int conv_ws64_dgrad_w1g_impl(const void* dy, const void* w, const void* mask, const void* img, void* y,
                                    float* w1slab, float* w1bslab, int slab_cap, int N, int H, int W, hipStream_t s) {
  HaloConvArgs h;
  h.x = (const bf16_t*)dy; h.w = (const bf16_t*)w; h.bias = nullptr; h.mask = (const bf16_t*)mask;
  h.y = (bf16_t*)y; h.zero = conv_zero_page();
  if (!h.zero) return -10;
  h.img = (const bf16_t*)img; h.w1slab = w1slab; h.w1bslab = w1bslab;
  h.N = N; h.H = H; h.W = W; h.tiles_x = (W + 63) / 64; h.tiles_y = (H + 3) / 4;
  int dev = 0, ncu = 0;
  CAN_HIP_CHECK(hipGetDevice(&dev));
  CAN_HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  const int S = 2 * ws64_grid(N * h.tiles_y * h.tiles_x, ncu);
  if (S > slab_cap) return -12;
  const int rc = launch_ws64<DT, EPI_MASK, true>(h, s);
  return rc ? -rc : S;
}

}  // namespace can

extern "C" int can_conv_ws64_dgrad_w1g(const void* dy, const void* w, const void* mask, const void* img, void* y,
                                       float* w1slab, float* w1bslab, int slab_cap, int N, int H, int W, int dt,
                                       void* stream) {
  CAN_DT_DISPATCH(dt, can::conv_ws64_dgrad_w1g_impl<DT>(dy, w, mask, img, y, w1slab, w1bslab, slab_cap, N, H, W,
                                                        (hipStream_t)stream));
}

// dt: element type of x / w / mask / y (DT_BF16 = 0, DT_F16 = 1)
// bpart (optional, EPI_MASK / EPI_POOLBWD): fp32 [bpart_cap][Cout] buffer for the bias-gradient partials of the
// produced gradient; *bpart_rows = rows written (0: this kernel path does not produce them)
extern "C" int can_conv_igemm(const void* x, const void* w, const float* bias, const void* mask, void* y,
                              int N, int H, int W, int Cin, int Cout, int ksize, int dil,
                              int epi, int first, int tile_cfg, int dt, void* stream, float* bpart, int bpart_cap,
                              int* bpart_rows) {
  CAN_DT_DISPATCH(dt, can::conv_igemm_impl<DT>(x, w, bias, mask, y, N, H, W, Cin, Cout, ksize, dil, epi, first,
                                              tile_cfg, stream, bpart, bpart_cap, bpart_rows));
}

extern "C" int can_conv_igemm_batched(const void* x, const void* w, const float* bias, void* y, int nb, long long xbs,
                                      long long wbs, long long ybs, int N, int H, int W, int Cin, int Cout, int ksize,
                                      int dil, int epi, int tile_cfg, int dt, void* stream) {
  CAN_DT_DISPATCH(dt, can::conv_igemm_batched_impl<DT>(x, w, bias, y, nb, xbs, wbs, ybs, N, H, W, Cin, Cout, ksize, dil,
                                                      epi, tile_cfg, (hipStream_t)stream));
}

extern "C" int can_conv_ctx(int fwd, const void* x, const void* w, const float* tab0, const float* tab1, const void* fv,
                            void* cat, void* y, int N, int H, int W, int C, int dt, void* stream) {
  CAN_DT_DISPATCH(dt, can::conv_ctx_impl<DT>(fwd, x, w, tab0, tab1, fv, cat, y, N, H, W, C, (hipStream_t)stream));
}

extern "C" int can_conv_pool_fwd(const void* x, const void* w, const float* bias, void* y, void* yp, void* codes,
                                 int N, int H, int W, int Cin, int Cout, int ksize, int dil, int tile_cfg, int dt,
                                 void* stream) {
  CAN_DT_DISPATCH(dt, can::conv_pool_fwd_impl<DT>(x, w, bias, y, yp, codes, N, H, W, Cin, Cout, ksize, dil, tile_cfg,
                                              (hipStream_t)stream));
}

// the kernel configuration conv_igemm picks for a (non-first-layer) conv with tile_cfg 0: 31 = halo kernel (Cin = 64),
// 33 = its weight-stationary ws64 form (Cin = Cout = 64), 27 / 28 / 29 = row ring, else the LDS-DMA tile config
extern "C" int can_conv_plan(int H, int W, int Cin, int Cout, int ksize, int dil, int epi) {
  using namespace can;
  if (Cin == 64 && ksize == 3 && dil == 1 && (Cout == 64 || Cout == 128) && epi != EPI_SIGMOID &&
      epi != EPI_POOLBWD && epi != EPI_F32)
    return (Cout == 64 && use_ws64()) ? 33 : 31;
  const int rr = (rring_mode() >= dil) ? rring_cfg(H, W, Cin, Cout, ksize, dil, epi) : 0;
  return rr ? rr : glds_default_cfg(Cin, Cout, ksize);
}

// pixels per tile of the kernel conv_pool_fwd runs for this layer (tile_cfg 0 = default): the fused pool
// needs H even and W % (tp / 2) == 0
extern "C" int can_conv_pool_tp(int Cin, int Cout, int ksize, int tile_cfg) {
  if (Cin == 64 && Cout == 64 && ksize == 3 && tile_cfg == 0) return 128;   // halo kernel: W % 64 (and H % 4)
  // row ring (2 x 128 tiles, 3x3 only): explicit cfg 27 (Cout % 256) / 29 (Cout % 128)
  if (tile_cfg == 27 || tile_cfg == 29) return (ksize == 3 && Cout % (tile_cfg == 27 ? 256 : 128) == 0) ? 256 : 0;
  return can::glds_cfg_tp(tile_cfg ? tile_cfg : can::glds_default_cfg(Cin, Cout, ksize));
}
