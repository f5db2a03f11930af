#!/bin/bash
# Throwaway diagnostic builds of conv_igemm.hip (NOT part of the package): CAN_PROBE=1 drops the activation
# DMA, 2 drops all DMA, 3 also replaces the LDS fragment reads by register constants.  Results are garbage;
# only the timing matters (where the v2 conv mainloop loses its cycles).
cd "$(dirname "$0")/../.." || exit 1
for m in 0 1 2 3 4; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -x hip -O3 -fPIC -shared -std=c++17 -DCAN_PROBE=$m \
    -Ican_distributed_pytorch_amd/csrc can_distributed_pytorch_amd/csrc/conv_igemm.hip -o build/probe/conv_probe$m.so &
done
wait
ls -la build/probe
