#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S pytest_gpu 900 python -m pytest tests -m gpu -q -rf || exit $?
$S debug_seeds 400 python scripts/debug_seeds.py || exit $?
