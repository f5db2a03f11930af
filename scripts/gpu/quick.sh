#!/bin/bash
# quick.sh "<pytest -k expr or test files>" : listed GPU tests, 1-GPU bench, kernel-trace profile (prof_quick)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S qtests 900 python -u -m pytest $1 -x -q -rf --timeout 240 --timeout-method thread || exit $?
$S bench 600 python bench.py --steps 30 --warmup 5 || exit $?
scripts/gpu/prof_step.sh prof_quick || exit $?
echo done
