#!/bin/bash
# r4_flds.sh: conv1_1 with LDS-staged fully contiguous stores (dispatch first_lds): tests, kernel timings, step arms
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S flds_tests 300 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "first_layer" || exit $?
grep -q " passed" gpurun_out/flds_tests.log && ! grep -q "failed\|error" gpurun_out/flds_tests.log || { echo "flds_tests failed: stop"; exit 1; }
$S first_layer 300 python scripts/bench_first_layer.py || exit $?
$S poolbwd 300 python scripts/bench_poolbwd.py || exit $?
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=first_lds=1 $S step_lds_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
