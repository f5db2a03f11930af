#!/bin/bash
# GPU session 4: component numerics + determinism, executor tests, bench.
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S pytest_comp 600 python -m pytest tests/test_gpu_components.py -q -rf || exit $?
$S pytest_exec 600 python -m pytest tests/test_gpu_executor.py -q -rf || exit $?
echo done
