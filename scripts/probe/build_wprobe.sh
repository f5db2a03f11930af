#!/bin/bash
# Throwaway diagnostic builds of conv_wgrad.hip (NOT part of the package): CAN_WPROBE=1 drops the DMA,
# 2 replaces the LDS fragment reads by register values, 3 both (ring + v2 weight-gradient kernels).
# Results are garbage; only the timing matters (where the weight-gradient mainloops lose their cycles).
cd "$(dirname "$0")/../.." || exit 1
mkdir -p scripts/probe/bin
for m in 0 1 2 3; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -x hip -O3 -fPIC -shared -std=c++17 -DCAN_WPROBE=$m \
    -Ican_distributed_pytorch_amd/csrc can_distributed_pytorch_amd/csrc/conv_wgrad.hip -o scripts/probe/bin/wgrad_probe$m.so &
done
wait
ls -la scripts/probe/bin
