// C ABI of the HIP kernel translation units (one launcher per kernel family).
// Return value: 0 ok, >0 hipError_t, <0 argument/shape error.
// dt selects the 16-bit element type of activations / weight packs: 0 = bf16, 1 = fp16.
#pragma once
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

int can_conv_igemm_batched(const void* x, const void* w, const float* bias, void* y, int nb, long long xbs,
                           long long wbs, long long ybs, int N, int H, int W, int Cin, int Cout, int ksize, int dil,
                           int epi, int tile_cfg, int dt, void* stream);
int can_conv_igemm(const void* x, const void* w, const float* bias, const void* mask, void* y, int N, int H, int W,
                   int Cin, int Cout, int ksize, int dil, int epi, int first, int tile_cfg, int dt, void* stream,
                   float* bpart, int bpart_cap, int* bpart_rows);

int can_wgrad_plan(int M, int Cin, int Cout, int ksize, int first, int target_blocks, int* S_out, int* mslice_out,
                   int* cfg_out, int dil, int W);
int can_conv_wgrad(const void* dy, const void* x, float* ws, float* wsb, float* dw, float* db, int N, int H, int W,
                   int Cin, int Cout, int ksize, int dil, int first, int S, int mslice, int cfg, float beta,
                   float scale, const float* dscale, int dt, void* stream, const float* bext, int bext_rows);

// [R][C] fp32 rows -> <= rows_out rows (fixed-order block sums); returns the rows written (< 0: error)
int can_bias_rows_reduce(const float* in, float* out, int R, int C, int rows_out, void* stream);
int can_conv_wgrad_1x1_batched(const void* dy, const void* x, float* ws, float* dw, int M, int W, int Cin, int Cout,
                               int nb, long long dy_bs, long long x_bs, long long dw_bs, int S, int mslice, float beta,
                               float scale, const float* dscale, int dt, void* stream);

// conv + bias + ReLU with the 2x2/s2 max-pool fused into the epilogue (y full resolution, yp pooled)
// codes: max-pool codes uint32 [N][H/2][W/2][Cout/8] (optional), y optional (nullptr: not written)
int can_conv_pool_fwd(const void* x, const void* w, const float* bias, void* y, void* yp, void* codes, int N, int H,
                      int W, int Cin, int Cout, int ksize, int dil, int tile_cfg, int dt, void* stream);
int can_conv_pool_tp(int Cin, int Cout, int ksize, int tile_cfg);

// conv1_2 with conv1_1's output recomputed from the NHWC4 image (never stored)

// conv1_2's data gradient with conv1_1's weight gradient fused (slabs [S][36][64] + [S][64]; returns S or < 0)
int can_conv_ws64_dgrad_w1g(const void* dy, const void* w, const void* mask, const void* img, void* y, float* w1slab,
                            float* w1bslab, int slab_cap, int N, int H, int W, int dt, void* stream);
int can_wgrad_reduce_first(const float* ws, const float* wsb, float* dw, float* db, int S, float beta, float scale,
                           const float* dscale, void* stream);

// elementwise.hip
int can_maxpool_fwd(const void* x, void* y, void* codes, int N, int H, int W, int C, int dt, void* stream);
int can_maxpool_bwd_codes(const void* codes, const void* dy, void* dx, int N, int H, int W, int C, int dt,
                          void* stream);
int can_maxpool_bwd_relu(const void* x, const void* dy, void* dx, int N, int H, int W, int C, int dt, void* stream);
int can_head_fwd(const void* y, const float* w, const float* b, float* et, int P, int dt, void* stream);
int can_head_train(const void* y, const float* w, const float* b, const float* gt, float* et, void* dy, float* part,
                   int nblk, float* dw, float* db, float* loss, int P, float gscale, float beta, const float* lscale,
                   float* nonfinite, int dt, void* stream);
int can_sgd_momentum(float* p, float* buf, const float* g, size_t n, float lr, float momentum, float gscale,
                     int first, float* flags, const float* lr_dev, void* stream);
int can_grad_nonfinite(const float* g, size_t n, float* flags, void* stream);
int can_split_x3(const float* src, void* dst, long long M, int C, int stride, int mode, int pattern, void* stream);
int can_scale_update(const float* flags, float* scaler, int interval, float growth, float backoff, float max_scale,
                     void* stream);
int can_pack_conv(const float* w, void* fwd, void* dgr, int Co, int Ci, int taps, int first, int dt, void* stream);
int can_pack_multi(const long long* desc, int layers, int max_tiles, int dt, void* stream);
int can_img_to_nhwc4(const float* img, void* out, int N, int H, int W, int dt, void* stream);

// context.hip
int can_ctx_reduce(int mode, const void* in0, const void* sdir, const void* dc, float* rowacc, float* cells, int N,
                   int h, int w, int C, int dt, void* stream);
int can_ctx_expand(const void* fv, const float* T, void* cs, int N, int h, int w, int C, int dt, void* stream);
int can_ctx_fuse(const void* fv, const void* ws, const float* T, void* cat, int N, int h, int w, int C, int dt,
                 void* stream);
int can_ctx_bwd_e1(const void* dcat, const void* ws, const float* T, void* dz, void* sdir, int N, int h, int w, int C,
                   int dt, void* stream);
int can_ctx_gemm(int mode, const float* x, const float* y, const float* const* w, float* out, float* const* gw, int N,
                 int C, float beta, float scale, const float* dscale, void* stream);
// linearised context module (conv_igemm.hip EPI_CTXF / EPI_CTXB + context.hip ctx_bwd_lin)
int can_conv_ctx(int fwd, const void* x, const void* w, const float* tab0, const float* tab1, const void* fv, void* cat,
                 void* y, int N, int H, int W, int C, int dt, void* stream);
int can_ctx_bwd_lin(const void* dcat, const void* wts, const float* U, void* dg, float* rowacc, int N, int h, int w,
                    int C, int dt, void* stream);
int can_ctx_cells(const float* rowacc, float* cells, int N, int h, int C, void* stream);
int can_ctx_w2_scatter(const float* tmp, float* const* dst, int C, float beta, void* stream);
int can_ctx_bwd_final(const void* dcat, const void* dc, const float* dave, const void* fv, void* dfv, int N, int h,
                      int w, int C, int dt, void* stream);

// density.hip
int can_density_map(const float* pts, int n, int H, int W, float* sigma_ws, float* out, int max_r, void* stream,
                    float fixed_sigma);

// preprocess.hip
int can_preprocess_image(const void* img, int H0, int W0, int C, int flip, void* out, int Ho, int Wo, int dt,
                         void* stream);
// one launch per batch: packed uint8 images / fp32 densities, desc [n][8] int64 (device)
int can_preprocess_batch(const void* imgs, const float* dens, const long long* desc, int n, void* x4, float* gt,
                         int Ho, int Wo, int ds, int dt, void* stream);
// synthetic batch: full-res densities [n][H][W] + coarse noise [n][3][H/16][W/16] -> x4 NHWC4, gt [n][H/8][W/8]
int can_synth_render(const float* dens, const float* noise, float* dmax, void* x4, float* gt, int n, int H, int W,
                     int dt, void* stream);
int can_preprocess_density(const float* d, int H0, int W0, int flip, float* out, int Ho, int Wo, float mult,
                           void* stream);

int can_conv_plan(int H, int W, int Cin, int Cout, int ksize, int dil, int epi);

#ifdef __cplusplus
}
#endif
