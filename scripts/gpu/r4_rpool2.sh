#!/bin/bash
# r4_rpool2.sh: per-layer timings of the pooled-layer forward kernels (glds2 / halo vs row ring) and two more step
# pairs (dispatch rring_pool)
cd "$GRAFT_REPO_ROOT" || exit 2
export TMPDIR=/tmp
S=scripts/gpu/run_step.sh
$S pool_layers 300 python scripts/bench_pool_fwd.py || exit $?
grep -q '"layer"' gpurun_out/pool_layers.log || { echo "pool_layers failed: stop"; exit 1; }
for r in 4 5; do
  $S step_base_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
  CANNET_DISPATCH=rring_pool=1 $S step_rpool_$r 300 python bench.py --steps 30 --warmup 5 || exit $?
done
echo done
