// Shared helpers for the gfx950 (CDNA4, MI355X) kernels of this framework.
// Written for wave64 / MFMA / 160 KiB LDS; no CUDA shims, no dual paths.
#pragma once
#include "dispatch.h"
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define CAN_HIP_CHECK(expr)                                                     \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) return (int)_e;                                       \
  } while (0)

namespace can {

using bf16_t = unsigned short;  // raw bf16 bits; converted explicitly
typedef short bf16x8 __attribute__((ext_vector_type(8)));
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float bf2f(unsigned short v) {
  return __uint_as_float(((unsigned)v) << 16);
}
// round-to-nearest-even fp32 -> bf16 (NaN stays NaN): the gfx950 hardware
// conversion v_cvt_pk_bf16_f32 (one instruction per PAIR; the integer RNE
// sequence it replaces cost ~5 VALU per value in every epilogue)
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned short f2bf(float f) {
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}
__device__ __forceinline__ unsigned pack2bf(float lo, float hi) {
  const f32x2_t v = {lo, hi};
  return __builtin_bit_cast(unsigned, __builtin_convertvector(v, bf16x2_t));
}

// ---------------------------------------------------------------------------
// 16-bit activation / weight-pack element types.  Every NHWC activation, packed
// weight and MFMA operand of the network is one of these two (selected per
// launch from the tensors' dtype); accumulation, master weights, gradients
// slabs and optimizer state are always fp32.  Kernels move the raw 16-bit
// words (LDS-DMA, transposed LDS reads) type-blind; only the MFMA instruction,
// the constant 1.0 and the fp32 <-> 16-bit conversions depend on the type.
// ---------------------------------------------------------------------------
enum { DT_BF16 = 0, DT_F16 = 1 };

typedef __bf16 frag8_t __attribute__((ext_vector_type(8)));     // 8 x 16-bit MFMA operand (bits)
typedef _Float16 f16x8_t __attribute__((ext_vector_type(8)));

template <int DT>
__device__ __forceinline__ f32x4 mfma16(const frag8_t& a, const frag8_t& b, const f32x4& c) {
  if constexpr (DT == DT_F16)
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_t, a), __builtin_bit_cast(f16x8_t, b), c,
                                                  0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
// bit pattern of 1.0
template <int DT>
__device__ __forceinline__ constexpr unsigned short one_bits() { return DT == DT_F16 ? 0x3C00 : 0x3F80; }
template <int DT>
__device__ __forceinline__ frag8_t ones_frag() {
  const short o = (short)one_bits<DT>();
  typedef short s16x8_ __attribute__((ext_vector_type(8)));
  const s16x8_ v = {o, o, o, o, o, o, o, o};
  return __builtin_bit_cast(frag8_t, v);
}
template <int DT>
__device__ __forceinline__ float h2f(unsigned short v) {
  if constexpr (DT == DT_F16) return (float)__builtin_bit_cast(_Float16, v);
  else return bf2f(v);
}
template <int DT>
__device__ __forceinline__ unsigned short f2h(float f) {
  if constexpr (DT == DT_F16) return __builtin_bit_cast(unsigned short, (_Float16)f);   // RNE, +-inf on overflow
  else return f2bf(f);
}
template <int DT>
__device__ __forceinline__ unsigned pack2(float lo, float hi) {
  if constexpr (DT == DT_F16) return (unsigned)f2h<DT>(lo) | ((unsigned)f2h<DT>(hi) << 16);
  else return pack2bf(lo, hi);
}
// 8 packed 16-bit values (one 16-B vector) <-> 8 floats
template <int DT>
__device__ __forceinline__ void unpack8h(const uint4& v, float* f) {
  const unsigned w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if constexpr (DT == DT_F16) {
      f[2 * i] = h2f<DT>((unsigned short)(w[i] & 0xffffu));
      f[2 * i + 1] = h2f<DT>((unsigned short)(w[i] >> 16));
    } else {
      f[2 * i] = __uint_as_float(w[i] << 16);
      f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
  }
}
template <int DT>
__device__ __forceinline__ uint4 pack8h(const float* f) {
  return make_uint4(pack2<DT>(f[0], f[1]), pack2<DT>(f[2], f[3]), pack2<DT>(f[4], f[5]), pack2<DT>(f[6], f[7]));
}
// x > 0 on the raw bits (same test for both types: sign clear, not +0)
__device__ __forceinline__ bool pos_bits(unsigned short b) { return ((b & 0x8000u) == 0) && ((b & 0x7fffu) != 0); }

// Dispatch a launcher templated on the element type: CAN_DT(dt, F<DT>(args)).
#define CAN_DT_DISPATCH(dt, ...)                                 \
  do {                                                           \
    if ((dt) == ::can::DT_F16) {                                 \
      constexpr int DT = ::can::DT_F16;                          \
      return __VA_ARGS__;                                        \
    } else if ((dt) == ::can::DT_BF16) {                         \
      constexpr int DT = ::can::DT_BF16;                         \
      return __VA_ARGS__;                                        \
    }                                                            \
    return -20;                                                  \
  } while (0)

// Launch kernel template K<DT> for a runtime element type (returns -20 from the
// enclosing function on an unknown dt).
#define CAN_LAUNCH_DT(dt, K, ...)                                  \
  do {                                                             \
    if ((dt) == ::can::DT_F16)                                     \
      hipLaunchKernelGGL(K<::can::DT_F16>, __VA_ARGS__);           \
    else if ((dt) == ::can::DT_BF16)                               \
      hipLaunchKernelGGL(K<::can::DT_BF16>, __VA_ARGS__);          \
    else                                                           \
      return -20;                                                  \
  } while (0)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Bias-gradient partials from a conv epilogue: lane (fr = lane & 15, fq = lane >> 4) holds 16 per-channel
// sums bs[0..15] over its pixels; the 16 lanes of a row (same fq, same channels) are summed by a
// transposing butterfly (each xor round halves the channels a lane keeps: 15 swaps instead of 64), after
// which lane fr holds the total of channel fr, and the 64 lanes store 64 consecutive floats
// part[chb0 + fq * 16 + fr].  Fixed order: deterministic.
__device__ __forceinline__ void store_bias_partials(float (&bs)[16], float* __restrict__ part, int fr) {
  float t8[8], t4[4], t2[2];
  const bool h8 = fr & 8, h4 = fr & 4, h2 = fr & 2, h1 = fr & 1;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float send = h8 ? bs[j] : bs[j + 8];
    t8[j] = (h8 ? bs[j + 8] : bs[j]) + __shfl_xor(send, 8, 64);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float send = h4 ? t8[j] : t8[j + 4];
    t4[j] = (h4 ? t8[j + 4] : t8[j]) + __shfl_xor(send, 4, 64);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const float send = h2 ? t4[j] : t4[j + 2];
    t2[j] = (h2 ? t4[j + 2] : t4[j]) + __shfl_xor(send, 2, 64);
  }
  const float send = h1 ? t2[0] : t2[1];
  part[fr] = (h1 ? t2[1] : t2[0]) + __shfl_xor(send, 1, 64);
}

// A-operand row order of the 16x16x32 MFMA convs: LDS / fragment row rho -> output channel, so
// that lane q of the D layout (rows q*4+r of tile jt) owns channels q*16 + jt*4 + r, i.e. 16
// CONSECUTIVE channels of one pixel per lane (two 16-B stores, no LDS round trip in epilogues).
__device__ __forceinline__ int perm_row(int rho) {
  // LDS weight row rho -> local output channel, so that lane q of the MFMA
  // D layout (rows q*4+r of tile jt) owns channels q*16 + jt*4 + r.
  const int rl = rho & 63;
  return (rho & ~63) | (((rl >> 2) & 3) << 4) | ((rl >> 4) << 2) | (rl & 3);
}

// LDS-DMA part placement in the MFMA groups of a stage's second K half, per kernel family, compile-time (a run-time
// switch pushed the 256 x 256 kernels into scratch; A/B builds: -D...=n, scripts/gpu/ab_variant_build.sh):
// 0 = part g before group g, 1 = part g after group g, 2 = parts 0 / 1 after groups 0 / 1, parts 2 + 3 after group 2.
// Per layer at batch 8 x 768 x 1024 (profiles/r3/ab_dma_order.txt): conv_glds2 best at 0 (1: +2..4 %), the row ring
// at 1 (-2..3 %), the weight-gradient GEMM at 2 (-2..4 %).
#ifndef CANNET_DMA_ORDER_CONV
#define CANNET_DMA_ORDER_CONV 0
#endif
#ifndef CANNET_DMA_ORDER_RR
#define CANNET_DMA_ORDER_RR 1
#endif
#ifndef CANNET_DMA_ORDER_WG
#define CANNET_DMA_ORDER_WG 2
#endif


// ---------------------------------------------------------------------------
// LDS-DMA through inline asm.  With the __builtin_amdgcn_{global,raw_ptr_buffer}_load_lds builtins hipcc (ROCm
// 7.2) knows an LDS write is in flight and, unable to tell the DMA's destination buffer from the one a later
// ds_read reads, emits s_waitcnt vmcnt(0) before that read: in a ring that issues stage s+2 between the MFMAs of
// stage s and the fragment reads of stage s+1, every stage then waits out the DMA it has just issued (its full
// latency, twice per stage in the weight-gradient GEMM).  Issued as asm the DMA is invisible to hipcc's counters;
// every kernel using these orders it itself: a counted s_waitcnt vmcnt(N) and an s_barrier before the first
// ds_read of the staged buffer (cdna_hip_programming.md: M0 is written and restored inside the statement).
// lds: the wave-uniform LDS byte address of the 1-KiB destination (lane l writes lds + 16 l).
// Invariants every caller keeps (nothing checks them at run time):
//  * the destination is wave-uniform: lds_addr() takes lane 0's address (readfirstlane), so a lane-divergent
//    destination would silently land at lane 0's; swizzled images are made by permuting the per-lane SOURCE;
//  * the issuing waves retire their own DMA with a counted s_waitcnt vmcnt(N) and pass an s_barrier before any
//    wave ds_reads the buffer (hipcc inserts no wait for asm DMA); tests/test_gpu_conv.py compares every LDS-DMA
//    kernel against an fp32 reference at tight tolerance, which a missing wait fails.
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(const __attribute__((address_space(3))) void*)p);
}
__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void glds4(const void* gsrc, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds) : "memory");
}
__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t rsrc, unsigned voff, unsigned soff, unsigned lds) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %2, %3 offen lds\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(rsrc), "s"(soff), "s"(lds) : "memory");
}

// TCOL = 64 (CO = 64 only): 4 waves, one per output row, 75 KB of LDS, so TWO
// blocks share a CU and one block's halo fetch overlaps the other's MFMAs (the
// 128-column block is alone on its CU: fetch, then compute, then store).
// Bijective XCD-aware remap of a 1-D block id (MI355X: 8 XCDs, blocks dealt
// round-robin).  Consecutive logical tiles land on the same XCD/L2.
__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int nx = 8;
  if (nwg < nx) return bid;
  int q = nwg / nx, r = nwg % nx, x = bid % nx, i = bid / nx;
  int base = (x < r) ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + i;
}

}  // namespace can
