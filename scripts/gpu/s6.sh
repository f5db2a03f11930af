#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S debug_layers 300 python scripts/debug_layers.py 64 96 || exit $?
$S debug_layers2 300 python scripts/debug_layers.py 72 120 || exit $?
echo done
