#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -m pytest tests/test_gpu_conv.py -q -rf || exit $?
$S convs_22 300 python scripts/bench_convs.py --no-ref --tile 22 --layers F4,F5,B4,B5,B6 || exit $?
$S convs_25 300 python scripts/bench_convs.py --no-ref --tile 25 --layers F4,F5,B4,B5,B6 || exit $?
echo done
