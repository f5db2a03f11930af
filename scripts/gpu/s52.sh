#!/bin/bash
# halo conv tap barrier now waits for the wave's LDS reads (WAR on the weight ring): determinism probe,
# conv tests, step
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S f1_probe 300 python scripts/debug_f1_dgrad.py || exit $?
$S conv_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S convs 300 python scripts/bench_convs.py --no-ref --layers F2,F3,F4 || exit $?
for r in 1 2; do
  $S bench$r 600 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
