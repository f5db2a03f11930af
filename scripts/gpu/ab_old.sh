#!/bin/bash
# Build the committed HEAD (or $1) of the package into ab_old/ (a self-contained copy with its own _C.so) so a
# GPU call can time old and new binaries on the same box.  Run HERE (CPU), before the gpurun call.
set -e
ref=${1:-HEAD}
rm -rf /tmp/ab_wt ab_old
git worktree prune
git worktree add -f /tmp/ab_wt "$ref" >/dev/null
(cd /tmp/ab_wt && python -m can_distributed_pytorch_amd.build_native -j 8 >/dev/null)
mkdir -p ab_old
cp -r /tmp/ab_wt/can_distributed_pytorch_amd /tmp/ab_wt/scripts /tmp/ab_wt/bench.py ab_old/
rm -rf ab_old/can_distributed_pytorch_amd/csrc
git worktree remove --force /tmp/ab_wt
echo "ab_old = $(git rev-parse --short $ref)"
