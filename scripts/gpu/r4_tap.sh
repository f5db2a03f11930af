#!/bin/bash
# r4_tap.sh: the tap-ring weight gradient (cfg 12, dispatch wgrad_tap) — its numerics tests first (stop on any
# failure), then per-layer weight-gradient timings (v2 / ring kernels vs tap ring, interleaved), then the step with
# wgrad_tap = 0 / 1 / 2 and the s_setprio build (ab_prio), interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tap_tests 400 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "wgrad" || exit $?
grep -q " passed" gpurun_out/tap_tests.log && ! grep -q "failed\|error" gpurun_out/tap_tests.log || { echo "tap_tests failed: stop"; exit 1; }
for r in 1 2; do
  $S wconv_base_$r 300 python scripts/bench_convs.py --no-ref --passes wgrad --iters 20 || exit $?
  CANNET_DISPATCH=wgrad_tap=2 $S wconv_tap_$r 300 python scripts/bench_convs.py --no-ref --passes wgrad --iters 20 || exit $?
done
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=wgrad_tap=1 $S step_tap1_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=wgrad_tap=2 $S step_tap2_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  $S step_prio_$r 300 python ab_prio/bench.py --steps 30 --warmup 5 || exit $?
done
echo done
