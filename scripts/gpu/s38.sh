#!/bin/bash
# weight gradients on a side stream (fork/join) vs in-order: full GPU tier + same-box A/B
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S gpu_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread || exit $?
$S bench_new 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_WGRAD_STREAM=0 $S bench_old 600 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_new_eager 600 python bench.py --steps 30 --warmup 5 --graph 0 || exit $?
CANNET_WGRAD_STREAM=0 $S bench_old_eager 600 python bench.py --steps 30 --warmup 5 --graph 0 || exit $?
echo done
