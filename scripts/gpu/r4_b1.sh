#!/bin/bash
# r4_b1.sh: first backend conv's data gradient before its weight gradient (dispatch b1_dgrad_first): test, isolated
# (dispatch b1_dgrad_first was removed after this A/B: profiles/r4/ab_b1_order.txt)
# fwd / dgrad per-layer timings, step arms interleaved.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S b1_tests 300 python -u -m pytest tests/test_gpu_executor.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "b1_order or matches_autograd" || exit $?
grep -q " passed" gpurun_out/b1_tests.log && ! grep -q "failed\|error" gpurun_out/b1_tests.log || { echo "b1_tests failed: stop"; exit 1; }
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=b1_dgrad_first=1 $S step_b1_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
$S convs_fd 300 python scripts/bench_convs.py --no-ref --passes fwd,dgrad --iters 20 || exit $?
echo done
