#!/bin/bash
# r4_r128.sh: dispatch rring128 = 2 (conv2_2's data gradient on the 128-channel row ring instead of conv_glds2's
# 128 x 512 tile) vs the default, on the final kernels; step arms interleaved
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=rring128=2 $S step_r128_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
