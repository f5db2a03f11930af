#!/bin/bash
# wgrad v2 + grid-stride reduce + batched packs: numerics, per-layer, step bench, kernel profile
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S conv_tests 600 python -m pytest tests/test_gpu_conv.py -q -rf || exit $?
$S comp_tests 600 python -m pytest tests/test_gpu_components.py -q -rf || exit $?
$S exec_tests 900 python -m pytest tests/test_gpu_executor.py -q -rf || exit $?
$S convs 300 python scripts/bench_convs.py --no-ref || exit $?
$S bench_g1 600 python bench.py --steps 20 --warmup 5 || exit $?
export TMPDIR=/tmp
$S prof_native 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_native23" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --graph 0 --steps 3 --warmup 2 || exit $?
echo done
