// Python bindings of the native runtime (pybind11, no torch C++ headers).
//
// Every entry point takes raw device pointers (tensor.data_ptr()) and the raw
// hipStream_t of the caller's current stream, so launches are graph-capturable
// and the kernels TUs compile without the torch headers.  Shape/dtype/layout
// validation happens in the Python wrappers (ops/*.py) BEFORE any launch.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>
#include <stdexcept>
#include <string>
#include <hip/hip_runtime.h>

#include "api.h"

namespace py = pybind11;

static void check(int rc, const char* what) {
  if (rc != 0) {
    std::string msg = std::string(what) + " failed: rc=" + std::to_string(rc);
    if (rc > 0) msg += std::string(" (") + hipGetErrorString((hipError_t)rc) + ")";
    throw std::runtime_error(msg);
  }
}

#define P(x) reinterpret_cast<void*>(x)

PYBIND11_MODULE(_C, m) {
  m.doc() = "gfx950 native kernels and runtime for can_distributed_pytorch_amd";

  m.def("arch", []() {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return std::string("none");
    return std::string(prop.gcnArchName);
  });

  m.def("conv_igemm", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t mask, uintptr_t y, int N, int H, int W,
                         int Cin, int Cout, int ksize, int dil, int epi, int first, int tile_cfg, uintptr_t stream) {
    check(can_conv_igemm(P(x), P(w), (const float*)bias, P(mask), P(y), N, H, W, Cin, Cout, ksize, dil, epi, first,
                         tile_cfg, P(stream)),
          "conv_igemm");
  });
}
