// Kernel-dispatch configuration of the native extension: ONE validated struct, no getenv anywhere in the
// launch paths.  The production values are the defaults below; the Python side (ops/dispatch.py) parses the
// single opt-in override string $CANNET_DISPATCH once (unknown keys and out-of-range values are errors) and
// pushes it here through set_dispatch(); tests switch variants with dispatch.override(...).  A stray
// environment variable can therefore never change the default training step.
#pragma once

namespace can {

struct DispatchConfig {
  // forward / data-gradient conv (conv_igemm.hip)
  int rring = 2;          // row-ring 3x3 kernels: 0 off, 1 dilation-1 layers, 2 every dilation
  int rring64 = 1;        // cfg 28 (64-channel, 4-row tiles)
  int rring128 = 1;       // cfg 29 (128 x (2 x 128)): 1 K > 1152 dilation 1, 2 + K <= 1152, 3 + dilation 2, 0 off
  int ws64 = 1;           // weight-stationary kernel for Cin = Cout = 64 (0: the halo kernel)
  int ctx_tile_f = 256;   // linearised context GEMM tiles (256 or 128), forward / backward
  int ctx_tile_b = 256;
  // weight gradient (conv_wgrad.hip, wgrad_ring.inc)
  int wgrad_halo_ring = 1;  // full-resolution layers: row-ring kernel (0: 2-row tiles with a full halo)
  int ring_fast = 1;        // row-ring weight gradient: in-image fast addressing when the shape allows it
  int ring_skew = 1;        // row-ring weight gradient: skewed DMA issue across waves
  int reduce_tiled = 1;     // slab reduction: tiled kernel where it applies (0: grid-stride kernel)
  // tap-ring weight gradient (cfg 12): 0 off, 1 the v2-GEMM layers, 2 (default) + the Cout = 128 full-resolution ring
  // ones, 3 + the Cout = 64 layers (64-channel tile, two blocks per CU): step 495.6 -> 511.8 (1) / 516.5 (2) img/s, 3 interleaved rounds (profiles/r4/ab_wgrad_tap.txt)
  int wgrad_tap = 3;        // 3: 521.4 vs 518.4 img/s (2), 3 interleaved rounds (profiles/r4/ab_wgrad_tap_variants.txt)
  int wgrad_tap_adb = 1;    // tap ring: double-buffered dY fragments (step +0.45 %, same file)
  int first_pf = 1;        // conv1_1: persistent, next halo loaded under the current stores (0.272 -> 0.189 ms)
  int rring_pool = 1;       // conv + 2x2 max-pool on the row ring (Cout % 256: conv3_3 -10 %, step +0.2 %)
};

// the process-wide configuration (defined in bindings.cpp)
extern DispatchConfig g_dispatch;

}  // namespace can
