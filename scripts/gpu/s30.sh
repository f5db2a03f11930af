#!/bin/bash
# fp16 native path: full GPU tier, bf16 + fp16 step benches
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S fp16_tests 600 python -u -m pytest tests/test_gpu_fp16.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S gpu_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread || exit $?
$S bench_g1 600 python bench.py --steps 20 --warmup 5 || exit $?
$S bench_fp16 600 python bench.py --steps 20 --warmup 5 --dtype fp16 || exit $?
echo done
