#!/bin/bash
# v2 wgrad cfg 10 / 11 (F5, B5 shapes)
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fp16.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S convs 300 python scripts/bench_convs.py --no-ref --layers F5,B5,B6 || exit $?
$S bench_g1 600 python bench.py --steps 20 --warmup 5 || exit $?
echo done
