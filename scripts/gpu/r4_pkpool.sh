#!/bin/bash
# r4_pkpool.sh: max-pool epilogue on packed 16-bit patterns (v_pk_max_u16 etc.): pool tests, pooled-layer timings,
# step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S pk_tests 400 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_executor.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "pool or stepper" || exit $?
grep -q " passed" gpurun_out/pk_tests.log && ! grep -q "failed\|error" gpurun_out/pk_tests.log || { echo "pk_tests failed: stop"; exit 1; }
$S pool_layers 300 python scripts/bench_pool_fwd.py || exit $?
for r in 1 2 3; do
  $S step_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
