#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S pytest_conv 600 python -m pytest tests/test_gpu_conv.py -q -rf -k "wgrad" || exit $?
$S convs_small 600 python scripts/bench_convs.py --no-ref --layers F2,F3,F4 || exit $?
$S pytest_gpu 900 python -m pytest tests -m gpu -q -rf || exit $?
$S bench_native 600 python bench.py --steps 20 --warmup 3 || exit $?
echo done
