#!/bin/bash
# bias column sums at 1024 threads/block + tiled slab reduction with 2 rows x S slabs of loads in flight:
# conv / executor tests, same-box step A/B against the previous build (ab_old/), both profiled
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tests 900 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_executor.py tests/test_gpu_components.py tests/test_gpu_fp16.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
for r in 1 2 3; do
  $S bench_old$r 600 python ab_old/bench.py --steps 30 --warmup 5 || exit $?
  $S bench_new$r 600 python bench.py --steps 30 --warmup 5 || exit $?
done
$S prof_old 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof55_old -o step -- python3 ab_old/bench.py --graph 0 --steps 3 --warmup 2 || exit $?
$S prof_new 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof55_new -o step -- python3 bench.py --graph 0 --steps 3 --warmup 2 || exit $?
echo done
