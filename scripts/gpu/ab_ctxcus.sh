#!/bin/bash
# A/B/C of the context 1x1 weight-gradient grid size (dispatch ctx_wgrad_cus): interleaved rounds on one box.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
R=${1:-3}
for r in $(seq $R); do
  for c in 256 224 192 160; do
    CANNET_DISPATCH=ctx_wgrad_cus=$c $S ab_ctx${c}_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  done
done
echo done
