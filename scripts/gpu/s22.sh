#!/bin/bash
# v2 conv default + v2 wgrad (+ fewer slices) + halo Cin=64 conv: numerics, per-layer timing, full step
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -m pytest tests/test_gpu_conv.py -q -rf || exit $?
$S convs_v2 300 python scripts/bench_convs.py --no-ref || exit $?
$S convs_halo 300 python scripts/bench_convs.py --no-ref --halo --layers F2,F3 || exit $?
CANNET_WGRAD_MANY_SLICES=1 $S convs_v2_many 300 python scripts/bench_convs.py --no-ref || exit $?
CANNET_WGRAD_V1=1 CANNET_WGRAD_MANY_SLICES=1 $S convs_wg_v1 300 python scripts/bench_convs.py --no-ref || exit $?
$S bench_g1 600 python bench.py --steps 20 --warmup 5 || exit $?
$S comp_tests 600 python -m pytest tests/test_gpu_components.py -q -rf || exit $?
$S exec_tests 900 python -m pytest tests/test_gpu_executor.py -q -rf || exit $?
echo done
