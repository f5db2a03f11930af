#!/bin/bash
# fused max-pool backward epilogue: GPU tier + same-box A/B (eager + side stream default)
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S gpu_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread || exit $?
$S bench_new 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_POOLBWD_FUSED=0 $S bench_old 600 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_new2 600 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_fp16 600 python bench.py --steps 30 --warmup 5 --dtype fp16 || exit $?
echo done
