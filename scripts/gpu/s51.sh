#!/bin/bash
# row-ring halo weight gradient: tests (ring on/off), per-layer wgrad A/B, step A/B
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S ring_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q -rf -k "halo or conv1_2 or tiled_reduction" --timeout 240 --timeout-method thread || exit $?
$S convs_ring 300 python scripts/bench_convs.py --no-ref --layers F2,F3,F4 || exit $?
CANNET_WGRAD_RING=0 $S convs_noring 300 python scripts/bench_convs.py --no-ref --layers F2,F3,F4 || exit $?
for r in 1 2; do
  CANNET_WGRAD_RING=0 $S bench_noring$r 600 python bench.py --steps 30 --warmup 5 || exit $?
  $S bench_ring$r 600 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
