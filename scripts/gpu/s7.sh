#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
scripts/gpu/run_step.sh debug_e2e 600 python scripts/debug_e2e.py || exit $?
