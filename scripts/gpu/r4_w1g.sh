#!/bin/bash
# r4_w1g.sh: conv1_1's fused weight gradient with transposed LDS reads of the staged dY tile: tests, the W1G cost
# (scripts/bench_w1g.py), step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S w1g_tests 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_executor.py tests/test_gpu_runtime.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "w1g or W1G or ws64 or first" || exit $?
grep -q " passed" gpurun_out/w1g_tests.log && ! grep -q "failed\|error" gpurun_out/w1g_tests.log || { echo "w1g_tests failed: stop"; exit 1; }
$S w1g_cost 300 python scripts/bench_w1g.py || exit $?
for r in 1 2 3; do
  $S step_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
