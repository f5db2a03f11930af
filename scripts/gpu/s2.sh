#!/bin/bash
# GPU session 2: native executor numerics + first native bench + profile.
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S pytest_gpu 900 python -m pytest tests -m gpu -x -q -rf || exit $?
$S bench_native_nograph 600 python bench.py --impl hip --graph 0 --steps 10 --warmup 3 || exit $?
$S bench_native_graph 600 python bench.py --impl hip --graph 1 --steps 10 --warmup 3 || exit $?
export TMPDIR=/tmp
$S prof_native 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_native" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --impl hip --graph 0 --steps 3 --warmup 2 || exit $?
echo done
