// Division by a runtime-invariant divisor via multiply-high (Granlund-Montgomery),
// exact for every 32-bit unsigned numerator; divisor >= 2 (host computes the pair).
#pragma once
#include <stdint.h>

struct FastDiv {
  uint32_t d, m, s;   // s = l - 1 where l = ceil(log2 d)
};

static inline FastDiv make_fastdiv(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t l = 0;
  while ((1ull << l) < d) ++l;
  if (l == 0) l = 1;   // d == 1 is handled by d itself below (m = 0 path)
  f.m = (uint32_t)(((1ull << 32) * ((1ull << l) - d)) / d + 1);
  f.s = l - 1;
  if (d == 1) { f.m = 0; f.s = 0; }
  return f;
}

#ifdef __HIPCC__
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  if (f.d == 1) return n;
  const uint32_t t = __umulhi(n, f.m);
  return (t + ((n - t) >> 1)) >> f.s;
}
#endif
