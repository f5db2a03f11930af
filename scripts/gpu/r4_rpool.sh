#!/bin/bash
# r4_rpool.sh: conv + max-pool forward on the row ring (dispatch rring_pool) — its tests, per-layer kernel timings and
# the step, interleaved against the default (conv_glds2 pool epilogue).
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S pool_tests 400 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "pool_fwd" || exit $?
grep -q " passed" gpurun_out/pool_tests.log && ! grep -q "failed\|error" gpurun_out/pool_tests.log || { echo "pool_tests failed: stop"; exit 1; }
$S pool_layers 300 python scripts/bench_pool_fwd.py || exit $?
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=rring_pool=1 $S step_rpool_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
