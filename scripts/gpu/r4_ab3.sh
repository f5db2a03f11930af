#!/bin/bash
# r4_ab3.sh: row-ring pooled forward (dispatch rring_pool) and conv1_1's 64-B store segments (first_st64): tests,
# per-kernel timings, step arms interleaved.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S ab3_tests 400 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "first_layer or pool_fwd" || exit $?
grep -q " passed" gpurun_out/ab3_tests.log && ! grep -q "failed\|error" gpurun_out/ab3_tests.log || { echo "ab3_tests failed: stop"; exit 1; }
$S pool_layers 300 python scripts/bench_pool_fwd.py || exit $?
$S first_layer 300 python scripts/bench_first_layer.py || exit $?
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=rring_pool=1 $S step_rpool_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=first_st64=1 $S step_st64_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=rring_pool=1,first_st64=1 $S step_both_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
