#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
scripts/gpu/run_step.sh debug_head 300 python scripts/debug_head.py || exit $?
