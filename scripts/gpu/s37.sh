#!/bin/bash
# halo conv: 64-column tiles / 2 blocks per CU vs 128-column tiles, same box
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -u -m pytest tests/test_gpu_conv.py tests/test_gpu_fp16.py -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S convs_new 300 python scripts/bench_convs.py --no-ref --layers F2,F3 || exit $?
CANNET_HALO_TCOL128=1 $S convs_old 300 python scripts/bench_convs.py --no-ref --layers F2,F3 || exit $?
$S bench_new 600 python bench.py --steps 30 --warmup 5 || exit $?
CANNET_HALO_TCOL128=1 $S bench_old 600 python bench.py --steps 30 --warmup 5 || exit $?
echo done
