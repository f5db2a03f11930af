#!/bin/bash
# stored vs recomputed conv1_1 output: per-kernel times of conv1_2 fwd / dgrad / wgrad, step A/B
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S f1_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q -rf -k "recomputed" --timeout 240 --timeout-method thread || exit $?
$S bench_f1 300 python scripts/bench_f1.py || exit $?
$S bench_new 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_F1_FUSED=0 $S bench_old 600 python bench.py --steps 30 --warmup 5 || exit $?
echo done
