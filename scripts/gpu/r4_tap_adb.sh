#!/bin/bash
# r4_tap_adb.sh: tap-ring weight gradient with double-buffered dY fragments (dispatch wgrad_tap_adb) — its tests,
# per-layer weight-gradient timings and the step, interleaved against the default; then hipGraph runtime knobs.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S tap_tests 400 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider -k "tap" || exit $?
grep -q " passed" gpurun_out/tap_tests.log && ! grep -q "failed\|error" gpurun_out/tap_tests.log || { echo "tap_tests failed: stop"; exit 1; }
for r in 1 2; do
  $S wconv_base_$r 300 python scripts/bench_convs.py --no-ref --passes wgrad --iters 20 || exit $?
  CANNET_DISPATCH=wgrad_tap_adb=1 $S wconv_adb_$r 300 python scripts/bench_convs.py --no-ref --passes wgrad --iters 20 || exit $?
  CANNET_DISPATCH=wgrad_tap=3 $S wconv_tap3_$r 300 python scripts/bench_convs.py --no-ref --passes wgrad --iters 20 || exit $?
done
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=wgrad_tap_adb=1 $S step_adb_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=wgrad_tap=3 $S step_tap3_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
for q in 1 2 4; do
  DEBUG_HIP_FORCE_GRAPH_QUEUES=$q $S graph_q$q 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
done
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 $S graph_nopc 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
$S graph_def 300 python bench.py --steps 30 --warmup 5 --graph 1 || exit $?
echo done
