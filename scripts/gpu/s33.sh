#!/bin/bash
# A/B in one box: coalesced reduce3 vs reduce2, v2 half-tile wgrad vs v1
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_executor.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S bench_new 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_REDUCE_V2=1 $S bench_red2 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_WGRAD_NO_HALF=1 $S bench_nohalf 600 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_new2 600 python bench.py --steps 30 --warmup 5 || exit $?
echo done
