#!/bin/bash
# r4_ab_prio.sh: s_setprio around the MFMA groups (ab_prio, -DCANNET_SETPRIO=1) vs this tree, interleaved on one
# box: per-layer conv timings (2 rounds) and the step (3 rounds); then the per-layer tile search of this tree and a
# kernel trace of the default step.
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
for r in 1 2; do
  $S convs_base_$r 300 python scripts/bench_convs.py --no-ref --iters 20 || exit $?
  $S convs_prio_$r 300 python ab_prio/scripts/bench_convs.py --no-ref --iters 20 || exit $?
done
for r in 1 2 3; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  $S step_prio_$r 300 python ab_prio/bench.py --steps 30 --warmup 5 || exit $?
done
$S p_eager 600 rocprofv3 --kernel-trace --stats -d gpurun_out/p_eager -o step -- python3 bench.py --steps 3 --warmup 2 --comm-steps 0 || exit $?
$S tune 900 python scripts/tune_tiles.py --out gpurun_out/tiles_768x1024.json || exit $?
echo done
