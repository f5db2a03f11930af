#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
scripts/gpu/run_step.sh debug_e2e2 300 python scripts/debug_e2e2.py || exit $?
