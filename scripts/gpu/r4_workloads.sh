#!/bin/bash
# r4_workloads.sh: convergence parity (scripts/gpu/r4_convergence.sh) and the reference's own workload shapes
# (scripts/gpu/ragged_train.sh) in one session.
cd "$GRAFT_REPO_ROOT" || exit 2
bash scripts/gpu/r4_convergence.sh || exit $?
bash scripts/gpu/ragged_train.sh || exit $?
echo done
