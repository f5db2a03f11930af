#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
scripts/gpu/run_step.sh debug_poison 300 python scripts/debug_poison.py || exit $?
