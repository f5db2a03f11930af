#!/bin/bash
# Build a variant of the CURRENT tree with extra hipcc defines into ab_<NAME>/ (self-contained package + scripts +
# bench.py) so one GPU call can time several compile-time variants on the same box.  Run HERE (CPU):
#   scripts/gpu/ab_variant_build.sh v1 "-DCANNET_DMA_ORDER_RR=0 -DCANNET_DMA_ORDER_WG=0"
# then e.g. `python ab_v1/scripts/bench_convs.py ...` / `python ab_v1/bench.py ...` on the box.
set -e
name=$1; flags=$2
cd "$(dirname "$0")/../.."
rm -rf "ab_$name"
mkdir -p "ab_$name"
cp -r can_distributed_pytorch_amd scripts bench.py "ab_$name/"
rm -f ab_$name/can_distributed_pytorch_amd/_C*.so
(cd "ab_$name" && CANNET_EXTRA_HIPFLAGS="$flags" python -m can_distributed_pytorch_amd.build_native -j 8 >/dev/null)
rm -rf "ab_$name/build" "ab_$name/can_distributed_pytorch_amd/csrc"
echo "ab_$name built with $flags"
