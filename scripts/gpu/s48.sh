#!/bin/bash
# v3 conv kernel (4 waves, 128x128 per wave): bitwise tests vs v2, per-layer A/B, step A/B
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S v3_tests 600 python -u -m pytest tests/test_gpu_conv.py -x -q -rf -k "v3" --timeout 240 --timeout-method thread || exit $?
$S convs_v2 300 python scripts/bench_convs.py --no-ref --layers F5,F6,F8,F9,B1,B2,B4,B5 || exit $?
CANNET_CONV_V3=1 $S convs_v3 300 python scripts/bench_convs.py --no-ref --layers F5,F6,F8,F9,B1,B2,B4,B5 || exit $?
CANNET_CONV_V3=2 $S convs_v3b 300 python scripts/bench_convs.py --no-ref --layers F3,F4,F5,B5 || exit $?
$S bench_v2 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_CONV_V3=1 $S bench_v3 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_CONV_V3=2 $S bench_v3b 600 python bench.py --steps 30 --warmup 5 || exit $?
$S bench_v2b 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_CONV_V3=1 $S bench_v3c 600 python bench.py --steps 30 --warmup 5 || exit $?
echo done
