#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
scripts/gpu/run_step.sh debug_seeds 400 python scripts/debug_seeds.py || exit $?
