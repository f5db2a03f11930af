#!/bin/bash
# r4_first.sh: conv1_1 as a persistent kernel prefetching the next tile's halo (dispatch first_pf) vs one tile per
# block: tests, kernel timings, step arms interleaved (rring_pool at its new default 1).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S first_tests 400 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "first_layer or pool_fwd" || exit $?
grep -q " passed" gpurun_out/first_tests.log && ! grep -q "failed\|error" gpurun_out/first_tests.log || { echo "first_tests failed: stop"; exit 1; }
$S first_layer 300 python scripts/bench_first_layer.py || exit $?
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=first_pf=1 $S step_pf_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=rring_pool=0 $S step_norp_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
