#!/bin/bash
# conv1_1 recompute inside conv1_2 (fwd / dgrad / wgrad): numerics + same-box A/B
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q -rf -k "recomputed or halo or first" --timeout 240 --timeout-method thread || exit $?
$S gpu_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread || exit $?
$S bench_new 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_F1_FUSED=0 $S bench_old 600 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_new2 600 python bench.py --steps 30 --warmup 5 || exit $?
echo done
