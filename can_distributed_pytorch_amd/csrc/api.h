// C ABI of the HIP kernel translation units (one launcher per kernel family).
// Return value: 0 ok, >0 hipError_t, <0 argument/shape error.
#pragma once
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

int can_conv_igemm(const void* x, const void* w, const float* bias, const void* mask, void* y, int N, int H, int W,
                   int Cin, int Cout, int ksize, int dil, int epi, int first, int tile_cfg, void* stream);

#ifdef __cplusplus
}
#endif
