#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
NCCL_DEBUG=WARN $S pytest_gpu 900 python -m pytest tests -m gpu -q -rf || exit $?
$S convs_cfg5 600 python scripts/bench_convs.py --no-ref --layers F6,F8,F9,B1,B2,B4 || exit $?
CANNET_WGRAD_CFG=7 $S convs_cfg7 600 python scripts/bench_convs.py --no-ref --layers F6,F8,F9,B1,B2,B4 || exit $?
$S convs_small 600 python scripts/bench_convs.py --no-ref --layers F2,F3,F4,F5,B5,B6 || exit $?
$S bench_native 600 python bench.py --steps 20 --warmup 3 || exit $?
export TMPDIR=/tmp
$S list_counters 120 rocprofv3 --list-avail || exit $?
echo done
