#!/bin/bash
# re-entry check (container re-created, _C rebuilt): smoke, full GPU test tier, 1-GPU bench
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $?
$S gpu_tests 900 python -u -m pytest tests -m gpu -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S bench 600 python bench.py --steps 30 --warmup 5 || exit $?
echo done
