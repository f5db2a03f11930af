#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S pytest_gpu 900 python -m pytest tests -m gpu -q -rf || exit $?
$S bench_convs 600 python scripts/bench_convs.py --no-ref --json gpurun_out/bench_convs5.json || exit $?
$S bench_native 600 python bench.py --steps 20 --warmup 3 || exit $?
export TMPDIR=/tmp
$S prof_native 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_native5" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --graph 0 --steps 3 --warmup 2 || exit $?
echo done
