// MFMA shape probe: v_mfma_f32_16x16x32_bf16 vs v_mfma_f32_32x32x16_bf16 on the conv kernels' wave tile.
//
// Each wave owns a 64 (rows) x 128 (cols) fp32 accumulator tile (the conv_glds2 wave tile: 64 channels x
// 128 pixels) and streams K through a 64-K bf16 LDS image exactly like the conv mainloop: every operand
// fragment is re-read from LDS with ds_read_b128 (XOR-swizzled 16-B chunks), random data, 2 waves per SIMD
// (8 waves per block, 1 block per CU), no global traffic inside the loop.  Both variants read the same LDS
// bytes and issue the same FLOPs; only the MFMA shape differs:
//   16x16x32: per 32-K step 4 A + 8 B fragments, 32 MFMAs (16 cycles each)
//   32x32x16: per 16-K step 2 A + 4 B fragments,  8 MFMAs (32 cycles each)
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/probe/mfma_shape.hip -o scripts/probe/mfma_shape
// Run:   scripts/probe/mfma_shape [iters]   -> one line per shape: ms, TF/s
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 frag8_t __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

constexpr int NW = 8;                 // waves per block (2 per SIMD)
constexpr int AROWS = 64 * 4;         // A image: 4 wave-rows of 64 channels
constexpr int BROWS = 128 * 2;        // B image: 2 wave-cols of 128 pixels
constexpr int LDS_BYTES = (AROWS + BROWS) * 128;   // 64 K (128 B) per row

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ (row & 7); }

template <int SHAPE>
__global__ void __launch_bounds__(64 * NW, 1) mfma_probe(const uint4* __restrict__ src, float* __restrict__ out,
                                                       int iters) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave & 3, wp = wave >> 2;
  uint4* s4 = reinterpret_cast<uint4*>(smem);
  for (int i = tid; i < LDS_BYTES / 16; i += 64 * NW) s4[i] = src[(blockIdx.x * 131 + i) & 65535];
  __syncthreads();
  const uint4* As = s4;
  const uint4* Bs = s4 + AROWS * 8;
  if constexpr (SHAPE == 16) {
    f32x4 acc[4][8];
    for (int j = 0; j < 4; ++j)
      for (int i = 0; i < 8; ++i) acc[j][i] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fr = lane & 15, fq = lane >> 4;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        const int chunk = kk * 4 + fq;
        frag8_t af[4], bf[8];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = wc * 64 + j * 16 + fr;
          af[j] = __builtin_bit_cast(frag8_t, As[row * 8 + swz(row, chunk)]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int row = wp * 128 + i * 16 + fr;
          bf[i] = __builtin_bit_cast(frag8_t, Bs[row * 8 + swz(row, chunk)]);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[j], bf[i], acc[j][i], 0, 0, 0);
      }
    }
    float s = 0.f;
    for (int j = 0; j < 4; ++j)
      for (int i = 0; i < 8; ++i) s += acc[j][i][0] + acc[j][i][1] + acc[j][i][2] + acc[j][i][3];
    out[blockIdx.x * 64 * NW + tid] = s;
  } else {
    f32x16 acc[2][4];
    for (int j = 0; j < 2; ++j)
      for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) acc[j][i][r] = 0.f;
    const int r32 = lane & 31, h = lane >> 5;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {          // 4 K16 steps = the same 64 K as two 16x16x32 K32 steps
        const int chunk = ks * 2 + h;
        frag8_t af[2], bf[4];
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int row = wc * 64 + j * 32 + r32;
          af[j] = __builtin_bit_cast(frag8_t, As[row * 8 + swz(row, chunk)]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int row = wp * 128 + i * 32 + r32;
          bf[i] = __builtin_bit_cast(frag8_t, Bs[row * 8 + swz(row, chunk)]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[j][i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[j], bf[i], acc[j][i], 0, 0, 0);
      }
    }
    float s = 0.f;
    for (int j = 0; j < 2; ++j)
      for (int i = 0; i < 4; ++i)
        for (int r = 0; r < 16; ++r) s += acc[j][i][r];
    out[blockIdx.x * 64 * NW + tid] = s;
  }
}

template <int SHAPE>
static void run(const uint4* src, float* out, int blocks, int iters) {
  auto k = mfma_probe<SHAPE>;
  CHECK(hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * NW), LDS_BYTES, 0, src, out, iters);
  CHECK(hipDeviceSynchronize());
  const int reps = 10;
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * NW), LDS_BYTES, 0, src, out, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  ms /= reps;
  // per block: 256 x 256 outputs x 64 K per iteration
  const double flops = 2.0 * 256 * 256 * 64 * (double)iters * blocks;
  printf("mfma_%s  blocks %d iters %d  %.3f ms  %.1f TF/s\n", SHAPE == 16 ? "16x16x32_bf16" : "32x32x16_bf16", blocks,
         iters, ms, flops / ms * 1e-9);
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 4096;
  int ncu = 0;
  CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int blocks = ncu * 4;
  std::vector<unsigned short> h(65536 * 8);
  unsigned s = 12345u;
  for (auto& v : h) {            // random bf16 in [-1, 1): sign, exponent 126/127, random mantissa
    s = s * 1664525u + 1013904223u;
    v = (unsigned short)(((s >> 31) << 15) | ((126u + ((s >> 20) & 1u)) << 7) | ((s >> 8) & 0x7Fu));
  }
  uint4* src;
  float* out;
  CHECK(hipMalloc(&src, h.size() * 2));
  CHECK(hipMalloc(&out, (size_t)blocks * 64 * NW * 4));
  CHECK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
  for (int round = 0; round < 3; ++round) {    // interleaved arms
    run<16>(src, out, blocks, iters);
    run<32>(src, out, blocks, iters);
  }
  CHECK(hipFree(src));
  CHECK(hipFree(out));
  return 0;
}
