#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
scripts/gpu/run_step.sh debug_layers_t 300 python scripts/debug_layers.py 64 96 test || exit $?
