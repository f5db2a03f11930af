#!/bin/bash
# v2 LDS-DMA conv kernel: numerics, then per-layer timing v1 vs v2
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -m pytest tests/test_gpu_conv.py -q -rf -x || exit $?
$S convs_v1 300 python scripts/bench_convs.py --no-ref --tile 0 || exit $?
$S convs_v2 300 python scripts/bench_convs.py --no-ref --tile 21 || exit $?
echo done
