#!/bin/bash
# max-pool fused into the conv epilogue: bitwise tests, executor tests, step A/B
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S pool_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q -rf -k "pool" --timeout 240 --timeout-method thread || exit $?
$S exec_tests 600 python -u -m pytest tests/test_gpu_executor.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S bench_new 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_POOL_FWD_FUSED=0 $S bench_old 600 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_new2 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_POOL_FWD_FUSED=0 $S bench_old2 600 python bench.py --steps 30 --warmup 5 || exit $?
echo done
