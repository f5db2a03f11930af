#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 2
S=scripts/gpu/run_step.sh
$S probe 300 python scripts/probe/conv_probe.py || exit $?
echo done
