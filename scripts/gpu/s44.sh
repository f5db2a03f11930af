#!/bin/bash
# tiled slab reduction: bitwise test, wgrad tests, step A/B against the grid-stride reduction
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S red_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q -rf -k "wgrad" --timeout 240 --timeout-method thread || exit $?
$S bench_new 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_REDUCE_GRIDSTRIDE=1 $S bench_old 600 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_new2 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_REDUCE_GRIDSTRIDE=1 $S bench_old2 600 python bench.py --steps 30 --warmup 5 || exit $?
echo done
