#!/bin/bash
# conv1_1 wgrad on the main stream (overlaps conv1_2's side-stream wgrad) + loss flags on the side stream:
# executor / train / dp / fp16 tests, step A/B, profile
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tests 600 python -u -m pytest tests/test_gpu_executor.py tests/test_gpu_train.py tests/test_gpu_dp.py tests/test_gpu_fp16.py tests/test_gpu_components.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
for r in 1 2; do
  CANNET_WGRAD1_MAIN=0 $S bench_side$r 600 python bench.py --steps 30 --warmup 5 || exit $?
  $S bench_main$r 600 python bench.py --steps 30 --warmup 5 || exit $?
done
$S bench_graph 600 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof54 -o step -- python3 bench.py --graph 0 --steps 3 --warmup 2 || exit $?
echo done
