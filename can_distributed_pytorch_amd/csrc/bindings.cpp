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

void register_rccl(py::module_& m);   // rccl_reducer.cpp

static void check(int rc, const char* what) {
  if (rc != 0) {
    std::string msg = std::string(what) + " failed: rc=" + std::to_string(rc);
    if (rc > 0) msg += std::string(" (") + hipGetErrorString((hipError_t)rc) + ")";
    throw std::runtime_error(msg);
  }
}

#define P(x) reinterpret_cast<void*>(x)

#ifndef CAN_MODULE_NAME
#define CAN_MODULE_NAME _C   // _C_asan: the host-AddressSanitizer build (build_native.py --asan)
#endif

PYBIND11_MODULE(CAN_MODULE_NAME, m) {
  m.doc() = "gfx950 native kernels and runtime for can_distributed_pytorch_amd";
  register_rccl(m);

  m.def("arch", []() {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&prop, dev) != hipSuccess) return std::string("none");
    return std::string(prop.gcnArchName);
  });

  m.def("conv_igemm", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t mask, uintptr_t y, int N, int H, int W,
                         int Cin, int Cout, int ksize, int dil, int epi, int first, int tile_cfg, int dt, uintptr_t stream,
                         uintptr_t bpart, int bpart_cap) {
    int rows = 0;
    check(can_conv_igemm(P(x), P(w), (const float*)bias, P(mask), P(y), N, H, W, Cin, Cout, ksize, dil, epi, first,
                         tile_cfg, dt, P(stream), (float*)bpart, bpart_cap, &rows),
          "conv_igemm");
    return rows;
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("mask"), py::arg("y"), py::arg("N"), py::arg("H"),
     py::arg("W"), py::arg("Cin"), py::arg("Cout"), py::arg("ksize"), py::arg("dil"), py::arg("epi"), py::arg("first"),
     py::arg("tile_cfg"), py::arg("dt"), py::arg("stream"), py::arg("bpart") = 0, py::arg("bpart_cap") = 0);

  m.def("conv_igemm_batched", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, int nb, long long xbs,
                                 long long wbs, long long ybs, int N, int H, int W, int Cin, int Cout, int ksize,
                                 int dil, int epi, int tile_cfg, int dt, uintptr_t stream) {
    check(can_conv_igemm_batched(P(x), P(w), (const float*)bias, P(y), nb, xbs, wbs, ybs, N, H, W, Cin, Cout, ksize,
                                 dil, epi, tile_cfg, dt, P(stream)),
          "conv_igemm_batched");
  });
  m.def("wgrad_plan", [](int M, int Cin, int Cout, int ksize, int first, int target_blocks, int dil) {
    int S = 0, ms = 0, cfg = 0;
    check(can_wgrad_plan(M, Cin, Cout, ksize, first, target_blocks, &S, &ms, &cfg, dil), "wgrad_plan");
    return py::make_tuple(S, ms, cfg);
  }, py::arg("M"), py::arg("Cin"), py::arg("Cout"), py::arg("ksize"), py::arg("first"), py::arg("target_blocks"),
     py::arg("dil") = 1);
  m.def("conv_wgrad", [](uintptr_t dy, uintptr_t x, uintptr_t ws, uintptr_t wsb, uintptr_t dw, uintptr_t db, int N,
                         int H, int W, int Cin, int Cout, int ksize, int dil, int first, int S, int mslice, int cfg,
                         float beta, float scale, uintptr_t dscale, int dt, uintptr_t stream, uintptr_t bext,
                         int bext_rows) {
    check(can_conv_wgrad(P(dy), P(x), (float*)ws, (float*)wsb, (float*)dw, (float*)db, N, H, W, Cin, Cout, ksize, dil,
                         first, S, mslice, cfg, beta, scale, (const float*)dscale, dt, P(stream), (const float*)bext,
                         bext_rows),
          "conv_wgrad");
  }, py::arg("dy"), py::arg("x"), py::arg("ws"), py::arg("wsb"), py::arg("dw"), py::arg("db"), py::arg("N"),
     py::arg("H"), py::arg("W"), py::arg("Cin"), py::arg("Cout"), py::arg("ksize"), py::arg("dil"), py::arg("first"),
     py::arg("S"), py::arg("mslice"), py::arg("cfg"), py::arg("beta"), py::arg("scale"), py::arg("dscale"),
     py::arg("dt"), py::arg("stream"), py::arg("bext") = 0, py::arg("bext_rows") = 0);

  m.def("bias_rows_reduce", [](uintptr_t in, uintptr_t out, int R, int C, int rows_out, uintptr_t st) {
    const int g = can_bias_rows_reduce((const float*)in, (float*)out, R, C, rows_out, P(st));
    if (g < 0) check(g, "bias_rows_reduce");
    return g;
  });
  m.def("conv_wgrad_1x1_batched", [](uintptr_t dy, uintptr_t x, uintptr_t ws, uintptr_t dw, int M, int W, int Cin,
                                     int Cout, int nb, long long dy_bs, long long x_bs, long long dw_bs, int S,
                                     int mslice, float beta, float scale, uintptr_t dscale, int dt, uintptr_t stream) {
    check(can_conv_wgrad_1x1_batched(P(dy), P(x), (float*)ws, (float*)dw, M, W, Cin, Cout, nb, dy_bs, x_bs, dw_bs, S,
                                     mslice, beta, scale, (const float*)dscale, dt, P(stream)),
          "conv_wgrad_1x1_batched");
  });

  m.def("conv_pool_fwd", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t y, uintptr_t yp, uintptr_t codes,
                            int N, int H, int W, int Cin, int Cout, int ksize, int dil, int tile_cfg, int dt,
                            uintptr_t stream) {
    check(can_conv_pool_fwd(P(x), P(w), (const float*)bias, P(y), P(yp), P(codes), N, H, W, Cin, Cout, ksize, dil,
                            tile_cfg, dt, P(stream)),
          "conv_pool_fwd");
  });
  m.def("conv_pool_tp", &can_conv_pool_tp);

  m.def("conv_f1", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t img, uintptr_t w1, uintptr_t b1, uintptr_t y,
                      int N, int H, int W, int epi, int dt, uintptr_t stream) {
    check(can_conv_f1(P(x), P(w), (const float*)bias, P(img), P(w1), (const float*)b1, P(y), N, H, W, epi, dt,
                      P(stream)),
          "conv_f1");
  });
  m.def("conv_ws64_dgrad_w1g", [](uintptr_t dy, uintptr_t w, uintptr_t mask, uintptr_t img, uintptr_t y,
                                  uintptr_t w1slab, uintptr_t w1bslab, int slab_cap, int N, int H, int W, int dt,
                                  uintptr_t stream) {
    const int S = can_conv_ws64_dgrad_w1g(P(dy), P(w), P(mask), P(img), P(y), (float*)w1slab, (float*)w1bslab,
                                          slab_cap, N, H, W, dt, P(stream));
    if (S <= 0) check(S == 0 ? -1 : S, "conv_ws64_dgrad_w1g");
    return S;
  });
  m.def("wgrad_reduce_first", [](uintptr_t ws, uintptr_t wsb, uintptr_t dw, uintptr_t db, int S, float beta,
                                 float scale, uintptr_t dscale, uintptr_t stream) {
    check(can_wgrad_reduce_first((const float*)ws, (const float*)wsb, (float*)dw, (float*)db, S, beta, scale,
                                 (const float*)dscale, P(stream)),
          "wgrad_reduce_first");
  });
  m.def("conv_wgrad_f1", [](uintptr_t dy, uintptr_t img, uintptr_t w1, uintptr_t b1, uintptr_t ws, uintptr_t wsb,
                            uintptr_t dw, uintptr_t db, int N, int H, int W, int S, float beta, float scale,
                            uintptr_t dscale, int dt, uintptr_t stream) {
    check(can_conv_wgrad_f1(P(dy), P(img), P(w1), (const float*)b1, (float*)ws, (float*)wsb, (float*)dw, (float*)db,
                            N, H, W, S, beta, scale, (const float*)dscale, dt, P(stream)),
          "conv_wgrad_f1");
  });

  // ---- elementwise
  m.def("maxpool_fwd", [](uintptr_t x, uintptr_t y, int N, int H, int W, int C, int dt, uintptr_t st,
                          uintptr_t codes) {
    check(can_maxpool_fwd(P(x), P(y), P(codes), N, H, W, C, dt, P(st)), "maxpool_fwd");
  }, py::arg("x"), py::arg("y"), py::arg("N"), py::arg("H"), py::arg("W"), py::arg("C"), py::arg("dt"),
     py::arg("st"), py::arg("codes") = 0);
  m.def("maxpool_bwd_codes", [](uintptr_t codes, uintptr_t dy, uintptr_t dx, int N, int H, int W, int C, int dt,
                                uintptr_t st) {
    check(can_maxpool_bwd_codes(P(codes), P(dy), P(dx), N, H, W, C, dt, P(st)), "maxpool_bwd_codes");
  });
  m.def("maxpool_bwd_relu", [](uintptr_t x, uintptr_t dy, uintptr_t dx, int N, int H, int W, int C, int dt,
                               uintptr_t st) {
    check(can_maxpool_bwd_relu(P(x), P(dy), P(dx), N, H, W, C, dt, P(st)), "maxpool_bwd_relu");
  });
  m.def("head_fwd", [](uintptr_t y, uintptr_t w, uintptr_t b, uintptr_t et, int Pn, int dt, uintptr_t st) {
    check(can_head_fwd(P(y), (const float*)w, (const float*)b, (float*)et, Pn, dt, P(st)), "head_fwd");
  });
  m.def("head_train", [](uintptr_t y, uintptr_t w, uintptr_t b, uintptr_t gt, uintptr_t et, uintptr_t dy,
                         uintptr_t part, int nblk, uintptr_t dw, uintptr_t db, uintptr_t loss, int Pn, float gscale,
                         float beta, uintptr_t lscale, uintptr_t nonfinite, int dt, uintptr_t st) {
    check(can_head_train(P(y), (const float*)w, (const float*)b, (const float*)gt, (float*)et, P(dy), (float*)part,
                         nblk, (float*)dw, (float*)db, (float*)loss, Pn, gscale, beta, (const float*)lscale,
                         (float*)nonfinite, dt, P(st)),
          "head_train");
  });
  m.def("sgd_momentum", [](uintptr_t p, uintptr_t buf, uintptr_t g, size_t n, float lr, float mom, float gscale,
                           int first, uintptr_t flags, uintptr_t lr_dev, uintptr_t st) {
    check(can_sgd_momentum((float*)p, (float*)buf, (const float*)g, n, lr, mom, gscale, first, (float*)flags,
                           (const float*)lr_dev, P(st)),
          "sgd_momentum");
  });
  m.def("split_x3", [](uintptr_t src, uintptr_t dst, long long M, int C, int stride, int mode, int pattern,
                       uintptr_t st) {
    check(can_split_x3((const float*)src, (void*)dst, M, C, stride, mode, pattern, P(st)), "split_x3");
  });
  m.def("grad_nonfinite", [](uintptr_t g, size_t n, uintptr_t flags, uintptr_t st) {
    check(can_grad_nonfinite((const float*)g, n, (float*)flags, P(st)), "grad_nonfinite");
  });
  m.def("scale_update", [](uintptr_t flags, uintptr_t scaler, int interval, float growth, float backoff, float max_scale,
                           uintptr_t st) {
    check(can_scale_update((const float*)flags, (float*)scaler, interval, growth, backoff, max_scale, P(st)),
          "scale_update");
  });
  m.def("pack_conv", [](uintptr_t w, uintptr_t fwd, uintptr_t dgr, int Co, int Ci, int taps, int first, int dt,
                        uintptr_t st) {
    check(can_pack_conv((const float*)w, P(fwd), P(dgr), Co, Ci, taps, first, dt, P(st)), "pack_conv");
  });
  m.def("pack_multi", [](uintptr_t desc, int layers, int max_tiles, int dt, uintptr_t st) {
    check(can_pack_multi((const long long*)desc, layers, max_tiles, dt, P(st)), "pack_multi");
  });
  m.def("img_to_nhwc4", [](uintptr_t img, uintptr_t out, int N, int H, int W, int dt, uintptr_t st) {
    check(can_img_to_nhwc4((const float*)img, P(out), N, H, W, dt, P(st)), "img_to_nhwc4");
  });
  // ---- context module
  m.def("ctx_reduce", [](int mode, uintptr_t in0, uintptr_t sdir, uintptr_t dc, uintptr_t rowacc, uintptr_t cells,
                         int N, int h, int w, int C, int dt, uintptr_t st) {
    check(can_ctx_reduce(mode, P(in0), P(sdir), P(dc), (float*)rowacc, (float*)cells, N, h, w, C, dt, P(st)),
          "ctx_reduce");
  });
  m.def("ctx_expand", [](uintptr_t fv, uintptr_t T, uintptr_t cs, int N, int h, int w, int C, int dt, uintptr_t st) {
    check(can_ctx_expand(P(fv), (const float*)T, P(cs), N, h, w, C, dt, P(st)), "ctx_expand");
  });
  m.def("ctx_fuse", [](uintptr_t fv, uintptr_t ws, uintptr_t T, uintptr_t cat, int N, int h, int w, int C, int dt,
                       uintptr_t st) {
    check(can_ctx_fuse(P(fv), P(ws), (const float*)T, P(cat), N, h, w, C, dt, P(st)), "ctx_fuse");
  });
  m.def("ctx_bwd_e1", [](uintptr_t dcat, uintptr_t ws, uintptr_t T, uintptr_t dz, uintptr_t sdir, int N, int h, int w,
                         int C, int dt, uintptr_t st) {
    check(can_ctx_bwd_e1(P(dcat), P(ws), (const float*)T, P(dz), P(sdir), N, h, w, C, dt, P(st)), "ctx_bwd_e1");
  });
  m.def("ctx_gemm", [](int mode, uintptr_t x, uintptr_t y, std::vector<uintptr_t> w, uintptr_t out,
                       std::vector<uintptr_t> gw, int N, int C, float beta, float scale, uintptr_t dscale, uintptr_t st) {
    if ((!w.empty() && w.size() != 4) || (!gw.empty() && gw.size() != 4)) throw std::runtime_error("ctx_gemm: 4 scales");
    const float* wp[4] = {nullptr, nullptr, nullptr, nullptr};
    float* gp[4] = {nullptr, nullptr, nullptr, nullptr};
    for (size_t i = 0; i < w.size(); ++i) wp[i] = (const float*)w[i];
    for (size_t i = 0; i < gw.size(); ++i) gp[i] = (float*)gw[i];
    check(can_ctx_gemm(mode, (const float*)x, (const float*)y, wp, (float*)out, gp, N, C, beta, scale,
                       (const float*)dscale, P(st)),
          "ctx_gemm");
  });
  m.def("conv_ctx", [](int fwd, uintptr_t x, uintptr_t w, uintptr_t tab0, uintptr_t tab1, uintptr_t fv, uintptr_t cat,
                       uintptr_t y, int N, int H, int W, int C, int dt, uintptr_t st) {
    check(can_conv_ctx(fwd, P(x), P(w), (const float*)tab0, (const float*)tab1, P(fv), P(cat), P(y), N, H, W, C, dt,
                       P(st)),
          "conv_ctx");
  });
  m.def("ctx_bwd_lin", [](uintptr_t dcat, uintptr_t wts, uintptr_t U, uintptr_t dg, uintptr_t rowacc, int N, int h,
                          int w, int C, int dt, uintptr_t st) {
    check(can_ctx_bwd_lin(P(dcat), P(wts), (const float*)U, P(dg), (float*)rowacc, N, h, w, C, dt, P(st)),
          "ctx_bwd_lin");
  });
  m.def("ctx_cells", [](uintptr_t rowacc, uintptr_t cells, int N, int h, int C, uintptr_t st) {
    check(can_ctx_cells((const float*)rowacc, (float*)cells, N, h, C, P(st)), "ctx_cells");
  });
  m.def("ctx_w2_scatter", [](uintptr_t tmp, std::vector<uintptr_t> dst, int C, float beta, uintptr_t st) {
    if (dst.size() != 4) throw std::runtime_error("ctx_w2_scatter: 4 scales");
    float* d[4] = {(float*)dst[0], (float*)dst[1], (float*)dst[2], (float*)dst[3]};
    check(can_ctx_w2_scatter((const float*)tmp, d, C, beta, P(st)), "ctx_w2_scatter");
  });
  m.def("ctx_bwd_final", [](uintptr_t dcat, uintptr_t dc, uintptr_t dave, uintptr_t fv, uintptr_t dfv, int N, int h,
                            int w, int C, int dt, uintptr_t st) {
    check(can_ctx_bwd_final(P(dcat), P(dc), (const float*)dave, P(fv), P(dfv), N, h, w, C, dt, P(st)),
          "ctx_bwd_final");
  });
  // ---- density maps
  m.def("density_map", [](uintptr_t pts, int n, int H, int W, uintptr_t sig, uintptr_t out, int max_r, uintptr_t st,
                          float fixed_sigma) {
    check(can_density_map((const float*)pts, n, H, W, (float*)sig, (float*)out, max_r, P(st), fixed_sigma),
          "density_map");
  }, py::arg("pts"), py::arg("n"), py::arg("H"), py::arg("W"), py::arg("sig"), py::arg("out"), py::arg("max_r"),
     py::arg("st"), py::arg("fixed_sigma") = 0.f);
  // ---- input pipeline
  m.def("preprocess_image", [](uintptr_t img, int H0, int W0, int C, int flip, uintptr_t out, int Ho, int Wo, int dt,
                               uintptr_t st) {
    check(can_preprocess_image(P(img), H0, W0, C, flip, P(out), Ho, Wo, dt, P(st)), "preprocess_image");
  });
  m.def("preprocess_batch", [](uintptr_t imgs, uintptr_t dens, uintptr_t desc, int n, uintptr_t x4, uintptr_t gt,
                               int Ho, int Wo, int ds, int dt, uintptr_t st) {
    check(can_preprocess_batch(P(imgs), (const float*)dens, (const long long*)desc, n, P(x4), (float*)gt, Ho, Wo, ds,
                               dt, P(st)),
          "preprocess_batch");
  });
  m.def("synth_render", [](uintptr_t dens, uintptr_t noise, uintptr_t dmax, uintptr_t x4, uintptr_t gt, int n, int H,
                           int W, int dt, uintptr_t st) {
    check(can_synth_render((const float*)dens, (const float*)noise, (float*)dmax, P(x4), (float*)gt, n, H, W, dt,
                           P(st)),
          "synth_render");
  });
  m.def("preprocess_density", [](uintptr_t d, int H0, int W0, int flip, uintptr_t out, int Ho, int Wo, float mult,
                                 uintptr_t st) {
    check(can_preprocess_density((const float*)d, H0, W0, flip, (float*)out, Ho, Wo, mult, P(st)),
          "preprocess_density");
  });
}
