#!/bin/bash
# hardware bf16 conversion + batched context wgrad: full GPU tier, benches, per-layer, step profile
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S gpu_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 300 --timeout-method thread || exit $?
$S bench_g1 600 python bench.py --steps 20 --warmup 5 || exit $?
$S bench_fp16 600 python bench.py --steps 20 --warmup 5 --dtype fp16 || exit $?
$S convs 300 python scripts/bench_convs.py --no-ref || exit $?
export TMPDIR=/tmp
$S prof_native 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof31" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --graph 0 --steps 3 --warmup 2 || exit $?
echo done
