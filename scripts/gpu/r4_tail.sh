#!/bin/bash
# r4_tail.sh: the step's tail in image halves (dispatch tail_split) — its executor test, then the step interleaved
# against the default, 4 rounds, plus a kernel trace of the split step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tail_tests 400 python -u -m pytest tests/test_gpu_executor.py -x -q -rf --timeout 240 --timeout-method thread -p no:cacheprovider -k "tail_split or w1g" || exit $?
grep -q " passed" gpurun_out/tail_tests.log && ! grep -q "failed\|error" gpurun_out/tail_tests.log || { echo "tail_tests failed: stop"; exit 1; }
for r in 1 2 3 4; do
  $S step_def_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=tail_split=1 $S step_split_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
CANNET_DISPATCH=tail_split=1 $S p_split 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_split -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
echo done
