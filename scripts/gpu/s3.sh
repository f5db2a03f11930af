#!/bin/bash
# GPU session 3: new LDS-DMA conv kernels: numerics, per-layer microbench vs MIOpen, full bench + profile.
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S pytest_conv 600 python -m pytest tests/test_gpu_conv.py -x -q -rf || exit $?
$S bench_convs 900 python scripts/bench_convs.py --json gpurun_out/bench_convs.json || exit $?
$S pytest_exec 600 python -m pytest tests/test_gpu_executor.py -q -rf || exit $?
$S bench_native 600 python bench.py --impl hip --steps 10 --warmup 3 || exit $?
export TMPDIR=/tmp
$S prof_native 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_native3" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --impl hip --graph 0 --steps 3 --warmup 2 || exit $?
echo done
