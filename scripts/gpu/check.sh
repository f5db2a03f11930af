#!/bin/bash
# GPU check: new runtime tests first, then all GPU tests, 1-GPU bench, one kernel-trace profile of the step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S rt 600 python -u -m pytest tests/test_gpu_runtime.py -x -v -rf --timeout 240 --timeout-method thread || exit $?
$S tests 1000 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S bench 600 python bench.py --steps 30 --warmup 5 || exit $?
$S prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_check -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
echo done
