#!/bin/bash
# conv1_2 max-pool fused into the halo kernel epilogue + conv1_1 wgrad on the compute stream: tests, step A/B
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S pool_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q -rf -k "pool" --timeout 240 --timeout-method thread || exit $?
$S exec_tests 600 python -u -m pytest tests/test_gpu_executor.py tests/test_gpu_fp16.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
for r in 1 2; do
  CANNET_POOL_FWD_FUSED=0 CANNET_F1_WGRAD_MAIN=0 $S bench_base$r 600 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_F1_WGRAD_MAIN=0 $S bench_pool$r 600 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_POOL_FWD_FUSED=0 $S bench_f1main$r 600 python bench.py --steps 30 --warmup 5 || exit $?
  $S bench_both$r 600 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
