#!/bin/bash
# r4_w8.sh: 8-wave 32-channel form of the Cout = 64 tap-ring weight gradient (dispatch wgrad_tap_w8) — its tests,
# per-layer weight-gradient timings and the step, interleaved against the default.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tap_tests 400 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "tap" || exit $?
grep -q " passed" gpurun_out/tap_tests.log && ! grep -q "failed\|error" gpurun_out/tap_tests.log || { echo "tap_tests failed: stop"; exit 1; }
for r in 1 2; do
  $S wconv_base_$r 300 python scripts/bench_convs.py --no-ref --passes wgrad --iters 20 || exit $?
  CANNET_DISPATCH=wgrad_tap_w8=1 $S wconv_w8_$r 300 python scripts/bench_convs.py --no-ref --passes wgrad --iters 20 || exit $?
done
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=wgrad_tap_w8=1 $S step_w8_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
