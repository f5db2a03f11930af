#!/bin/bash
# r4_early.sh: two-part optimizer step (dispatch early_sgd): its tests, then step arms interleaved (eager and graph).
# (dispatch early_sgd was removed after this A/B: profiles/r4/ab_early_sgd.txt)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S early_tests 400 python -u -m pytest tests/test_gpu_executor.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider || exit $?
grep -q " passed" gpurun_out/early_tests.log && ! grep -q "failed\|error" gpurun_out/early_tests.log || { echo "early_tests failed: stop"; exit 1; }
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=early_sgd=1 $S step_early_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
$S graph_base 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
CANNET_DISPATCH=early_sgd=1 $S graph_early 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
echo done
